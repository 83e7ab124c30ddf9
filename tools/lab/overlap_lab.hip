// Kernel lab: how much of route_fc2 (latency-bound) hides under fc1_wgrad_adam
// (HBM-bound) when both run concurrently?  Upper bound for a horizontal fusion.
//   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/overlap_lab.hip
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn { void init_fwd_attributes() {} }
#include <cstdio>
using namespace p2cnn;
int main() {
  const size_t np = 6600000, nw = size_t(kHid) * kFeat;
  uint16_t *dH, *a1, *w1bf, *w1t, *w1t2, *dc2m, *H; uint8_t* am2; float *p, *m, *v, *gb, *dlog; int* t;
  P2_CHECK(hipMalloc(&dH, 32 * kHid * 2)); P2_CHECK(hipMalloc(&a1, 32 * kFeat * 2)); P2_CHECK(hipMalloc(&H, 32 * kHid * 2));
  P2_CHECK(hipMalloc(&w1bf, nw * 2)); P2_CHECK(hipMalloc(&w1t, nw * 2)); P2_CHECK(hipMalloc(&w1t2, nw * 2));
  P2_CHECK(hipMalloc(&dc2m, 32 * 64 * 224 * 2)); P2_CHECK(hipMalloc(&am2, 32 * kFeat)); P2_CHECK(hipMalloc(&gb, 32 * kFeat * 4));
  P2_CHECK(hipMalloc(&dlog, 320 * 4)); P2_CHECK(hipMalloc(&p, np * 4)); P2_CHECK(hipMalloc(&m, np * 4)); P2_CHECK(hipMalloc(&v, np * 4));
  P2_CHECK(hipMalloc(&t, 4));
  P2_CHECK(hipMemset(dH, 0, 32 * kHid * 2)); P2_CHECK(hipMemset(a1, 0, 32 * kFeat * 2)); P2_CHECK(hipMemset(H, 0, 32 * kHid * 2));
  P2_CHECK(hipMemset(w1t, 0, nw * 2)); P2_CHECK(hipMemset(am2, 1, 32 * kFeat)); P2_CHECK(hipMemset(dlog, 0, 1280));
  P2_CHECK(hipMemset(p, 0, np * 4)); P2_CHECK(hipMemset(m, 0, np * 4)); P2_CHECK(hipMemset(v, 0, np * 4)); P2_CHECK(hipMemset(t, 0, 4));
  Offsets off{0, 832, 896, 52096, 52160, 6474816, 6476864, 6497344};
  AdamCfg cfg{1e-3f, 0.9f, 0.999f, 1e-8f, 0.f};
  hipStream_t s1, s2;
  P2_CHECK(hipStreamCreate(&s1)); P2_CHECK(hipStreamCreate(&s2));
  hipEvent_t a, b, e1, e2;
  P2_CHECK(hipEventCreate(&a)); P2_CHECK(hipEventCreate(&b)); P2_CHECK(hipEventCreate(&e1)); P2_CHECK(hipEventCreate(&e2));
  auto route = [&](hipStream_t s) { route_fc2(dH, w1t, am2, 32, 32, dc2m, gb, dlog, H, p, m, v, nullptr, off, t, 1, cfg, s); };
  auto fc1 = [&](hipStream_t s) { fc1_wgrad_adam(dH, a1, 32, p, m, v, nullptr, w1bf, w1t2, off, t, 1, cfg, s); };
  const int reps = 100;
  for (int mode = 0; mode < 3; ++mode) {
    for (int i = 0; i < 5; ++i) { route(s1); fc1(s1); }
    P2_CHECK(hipDeviceSynchronize());
    P2_CHECK(hipEventRecord(a, s1));
    for (int i = 0; i < reps; ++i) {
      if (mode == 0) { route(s1); fc1(s1); }                  // serial
      else if (mode == 1) {                                    // concurrent, fc1 first
        P2_CHECK(hipEventRecord(e1, s1)); P2_CHECK(hipStreamWaitEvent(s2, e1, 0));
        fc1(s1); route(s2);
        P2_CHECK(hipEventRecord(e2, s2)); P2_CHECK(hipStreamWaitEvent(s1, e2, 0));
      } else {                                                 // concurrent, route first
        P2_CHECK(hipEventRecord(e1, s1)); P2_CHECK(hipStreamWaitEvent(s2, e1, 0));
        route(s2); fc1(s1);
        P2_CHECK(hipEventRecord(e2, s2)); P2_CHECK(hipStreamWaitEvent(s1, e2, 0));
      }
    }
    P2_CHECK(hipEventRecord(b, s1));
    P2_CHECK(hipEventSynchronize(b));
    float ms; P2_CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%-28s %7.2f us per (route + fc1)\n", mode == 0 ? "serial" : mode == 1 ? "two streams, fc1 first" : "two streams, route first", ms * 1000 / reps);
  }
  return 0;
}
