// PyTorch bindings of the p2pfl_amd HIP kernels (module p2pfl_amd._C).
// Every entry validates shapes/dtypes/devices on the host BEFORE launching,
// so a mismatched call fails with a Python exception instead of a GPU fault.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <cmath>
#include <vector>

#include "kernels.h"
#include "cnn.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

void check_arena(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 || t.scalar_type() == torch::kBFloat16, name, " must be float32 or bfloat16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

void weighted_sum(std::vector<torch::Tensor> srcs, std::vector<double> weights, torch::Tensor out,
                  c10::optional<torch::Tensor> acc_in, double scale) {
  TORCH_CHECK(srcs.size() == weights.size(), "weighted_sum: bad inputs");
  check_arena(out, "out");
  const bool out_bf16 = out.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(!out_bf16 || srcs.size() <= size_t(p2::kMaxInputs), "weighted_sum: bf16 output supports at most ",
              p2::kMaxInputs, " inputs");
  const c10::DeviceGuard guard(out.device());
  const int64_t n = out.numel();
  const float* acc = nullptr;
  if (acc_in.has_value() && acc_in->defined()) {
    check_arena(*acc_in, "acc_in");
    TORCH_CHECK(acc_in->scalar_type() == torch::kFloat32 && acc_in->numel() == n && acc_in->device() == out.device(),
                "weighted_sum: acc_in must be an fp32 arena of the output's size and device");
    acc = acc_in->data_ptr<float>();
  }
  TORCH_CHECK(!srcs.empty() || acc != nullptr, "weighted_sum: no inputs");
  std::vector<const void*> ptrs;
  std::vector<int> bf;
  std::vector<float> w;
  for (size_t i = 0; i < srcs.size(); ++i) {
    check_arena(srcs[i], "src");
    TORCH_CHECK(srcs[i].numel() == n, "weighted_sum: size mismatch");
    TORCH_CHECK(srcs[i].device() == out.device(), "weighted_sum: device mismatch");
    ptrs.push_back(srcs[i].data_ptr());
    bf.push_back(srcs[i].scalar_type() == torch::kBFloat16 ? 1 : 0);
    w.push_back(float(weights[i]));
  }
  p2::weighted_sum(ptrs.data(), bf.data(), w.data(), int(ptrs.size()), acc, float(scale), out.data_ptr(),
                   out_bf16 ? 1 : 0, n, stream());
}

uint16_t* opt_bf16(const c10::optional<torch::Tensor>& t, int64_t n) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kBFloat16 && t->is_contiguous() && t->numel() >= n,
              "bf16 shadow must be a contiguous bf16 GPU tensor of the arena size");
  return reinterpret_cast<uint16_t*>(t->data_ptr());
}

void adam_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> pbf,
               double lr, double b1, double b2, double eps, double wd, int64_t step, bool decoupled) {
  for (auto* t : {&p, &g, &m, &v}) check_f32(*t, "adam operand");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  TORCH_CHECK(n % 4 == 0, "adam: arena length must be a multiple of 4");
  const c10::DeviceGuard guard(p.device());
  p2::AdamParams h{};
  h.lr = float(lr);
  h.beta1 = float(b1);
  h.beta2 = float(b2);
  h.eps = float(eps);
  h.weight_decay = float(wd);
  h.step_size = float(lr / (1.0 - std::pow(b1, double(step))));
  h.inv_sqrt_bc2 = float(1.0 / std::sqrt(1.0 - std::pow(b2, double(step))));
  h.decoupled = decoupled ? 1 : 0;
  p2::adam_step(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), opt_bf16(pbf, n),
                n, h, stream());
}

void sgd_step(torch::Tensor p, torch::Tensor g, c10::optional<torch::Tensor> buf, c10::optional<torch::Tensor> pbf,
              double lr, double momentum, double dampening, double wd, bool nesterov, bool first_step) {
  check_f32(p, "p");
  check_f32(g, "g");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && n % 4 == 0, "sgd: size mismatch");
  float* b = nullptr;
  if (buf.has_value() && buf->defined()) {
    check_f32(*buf, "buf");
    TORCH_CHECK(buf->numel() == n, "sgd: buf size mismatch");
    b = buf->data_ptr<float>();
  }
  const c10::DeviceGuard guard(p.device());
  p2::SgdParams h{float(lr), float(momentum), float(dampening), float(wd), nesterov ? 1 : 0, first_step ? 1 : 0};
  p2::sgd_step(p.data_ptr<float>(), g.data_ptr<float>(), b, opt_bf16(pbf, n), n, h, stream());
}

// ---- multi-tensor optimizer steps (mixed-precision learners) ----------------
// tens: int64 [T, 4] (offset, numel, flags, chunk) on the GPU; chunks: int32 [C, 2]
// (tensor, first element) on the GPU; grads: one entry per tensor (None = skip).
torch::Tensor grad_table(const std::vector<c10::optional<torch::Tensor>>& grads, const std::vector<int64_t>& numels,
                         const std::vector<bool>& grad_bf16, const std::vector<bool>& grad_cl, const torch::Device& dev) {
  const size_t T = grads.size();
  TORCH_CHECK(numels.size() == T && grad_bf16.size() == T && grad_cl.size() == T,
              "multi-tensor step: table size mismatch");
  auto host = torch::empty({int64_t(T)}, torch::dtype(torch::kInt64)).pin_memory();
  auto* hp = host.data_ptr<int64_t>();
  for (size_t t = 0; t < T; ++t) {
    hp[t] = 0;
    if (!grads[t].has_value() || !grads[t]->defined()) continue;
    const auto& g = *grads[t];
    // channels-last tensors (flag bit 2): the gradient arrives in the
    // weight's (O, kh, kw, I) memory order
    const bool dense = grad_cl[t] ? (g.dim() == 4 && g.is_contiguous(at::MemoryFormat::ChannelsLast)) : g.is_contiguous();
    TORCH_CHECK(g.device() == dev && dense && g.numel() == numels[t], "grad ", t,
                " must be a dense GPU tensor of the parameter's size and layout");
    TORCH_CHECK(g.scalar_type() == (grad_bf16[t] ? torch::kBFloat16 : torch::kFloat32), "grad ", t,
                " has an unexpected dtype");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "grad ", t, " must be 16-byte aligned");
    hp[t] = int64_t(reinterpret_cast<uintptr_t>(g.data_ptr()));
  }
  return host.to(dev, /*non_blocking=*/true);
}

void check_tables(const torch::Tensor& tens, const torch::Tensor& chunks, const torch::Device& dev) {
  TORCH_CHECK(tens.device() == dev && tens.scalar_type() == torch::kInt64 && tens.dim() == 2 && tens.size(1) == 4 &&
                  tens.is_contiguous(),
              "tensor table must be int64 [T, 4] on the arena's device");
  TORCH_CHECK(chunks.device() == dev && chunks.scalar_type() == torch::kInt32 && chunks.dim() == 2 &&
                  chunks.size(1) == 2 && chunks.is_contiguous(),
              "chunk table must be int32 [C, 2] on the arena's device");
}

// gtab (optional): a persistent device table of gradient addresses (int64 [T])
// used instead of `grads` -- for steps captured in a HIP graph, whose gradient
// buffers have fixed addresses filled in after capture.
torch::Tensor grad_ptrs(const c10::optional<torch::Tensor>& gtab, const std::vector<c10::optional<torch::Tensor>>& grads,
                        const std::vector<int64_t>& numels, const std::vector<bool>& grad_bf16,
                        const std::vector<bool>& grad_cl, const torch::Tensor& tens, const torch::Device& dev) {
  if (gtab.has_value() && gtab->defined()) {
    TORCH_CHECK(gtab->device() == dev && gtab->scalar_type() == torch::kInt64 && gtab->is_contiguous() &&
                    gtab->numel() == tens.size(0),
                "gtab must be a contiguous int64 [T] tensor on the arena's device");
    return *gtab;
  }
  TORCH_CHECK(tens.size(0) == int64_t(grads.size()), "multi-tensor step: one gradient per tensor");
  return grad_table(grads, numels, grad_bf16, grad_cl, dev);
}

void adam_mt_step(torch::Tensor p, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> pbf,
                  torch::Tensor tens, torch::Tensor chunks, std::vector<c10::optional<torch::Tensor>> grads,
                  std::vector<int64_t> numels, std::vector<bool> grad_bf16, std::vector<bool> grad_cl, double lr,
                  double b1, double b2, double eps,
                  double wd, int64_t step, bool decoupled, c10::optional<torch::Tensor> gtab,
                  c10::optional<torch::Tensor> t_dev) {
  for (auto* t : {&p, &m, &v}) check_f32(*t, "adam operand");
  const int64_t n = p.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n, "adam: size mismatch");
  check_tables(tens, chunks, p.device());
  const c10::DeviceGuard guard(p.device());
  auto gp = grad_ptrs(gtab, grads, numels, grad_bf16, grad_cl, tens, p.device());
  p2::AdamParams h{};
  h.lr = float(lr);
  h.beta1 = float(b1);
  h.beta2 = float(b2);
  h.eps = float(eps);
  h.weight_decay = float(wd);
  h.step_size = float(lr / (1.0 - std::pow(b1, double(step))));
  h.inv_sqrt_bc2 = float(1.0 / std::sqrt(1.0 - std::pow(b2, double(step))));
  h.decoupled = decoupled ? 1 : 0;
  if (t_dev.has_value() && t_dev->defined()) {
    TORCH_CHECK(t_dev->device() == p.device() && t_dev->scalar_type() == torch::kInt32 && t_dev->numel() == 1,
                "t_dev must be an int32 [1] tensor on the arena's device");
    h.t_dev = t_dev->data_ptr<int32_t>();
  }
  p2::adam_mt_step(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), opt_bf16(pbf, n),
                   reinterpret_cast<const p2::MTTensor*>(tens.data_ptr<int64_t>()),
                   reinterpret_cast<const int2*>(chunks.data_ptr<int32_t>()), int(chunks.size(0)),
                   reinterpret_cast<const uint64_t*>(gp.data_ptr<int64_t>()), h, stream());
}

void sgd_mt_step(torch::Tensor p, c10::optional<torch::Tensor> buf, c10::optional<torch::Tensor> pbf,
                 torch::Tensor tens, torch::Tensor chunks, std::vector<c10::optional<torch::Tensor>> grads,
                 std::vector<int64_t> numels, std::vector<bool> grad_bf16, std::vector<bool> grad_cl, double lr,
                 double momentum,
                 double dampening, double wd, bool nesterov, bool first_step, c10::optional<torch::Tensor> gtab) {
  check_f32(p, "p");
  const int64_t n = p.numel();
  float* b = nullptr;
  if (buf.has_value() && buf->defined()) {
    check_f32(*buf, "buf");
    TORCH_CHECK(buf->numel() == n, "sgd: buf size mismatch");
    b = buf->data_ptr<float>();
  }
  check_tables(tens, chunks, p.device());
  const c10::DeviceGuard guard(p.device());
  auto gp = grad_ptrs(gtab, grads, numels, grad_bf16, grad_cl, tens, p.device());
  p2::SgdParams h{float(lr), float(momentum), float(dampening), float(wd), nesterov ? 1 : 0, first_step ? 1 : 0};
  p2::sgd_mt_step(p.data_ptr<float>(), b, opt_bf16(pbf, n), reinterpret_cast<const p2::MTTensor*>(tens.data_ptr<int64_t>()),
                  reinterpret_cast<const int2*>(chunks.data_ptr<int32_t>()), int(chunks.size(0)),
                  reinterpret_cast<const uint64_t*>(gp.data_ptr<int64_t>()), h, stream());
}

// A stream owned by its caller.  torch.cuda.Stream() hands out streams from a
// fixed pool of 32 per device, round robin: two learners (virtual peers) can
// then share one HIP stream, and an event one records on it while the other
// captures a graph on it becomes part of that capture (hipErrorCapturedEvent).
// priority: 0 the default queue priority, > 0 the device's lowest, < 0 its highest
int64_t new_stream(int64_t device, int64_t priority) {
  const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, c10::DeviceIndex(device)));
  hipStream_t s = nullptr;
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  TORCH_CHECK(e == hipSuccess, "new_stream: ", hipGetErrorString(e));
  const int prio = priority > 0 ? least : (priority < 0 ? greatest : 0);
  e = prio == 0 ? hipStreamCreateWithFlags(&s, hipStreamNonBlocking) : hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio);
  TORCH_CHECK(e == hipSuccess, "new_stream: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(s);
}
void destroy_stream(int64_t s) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(s)); }

}  // namespace

void register_cnn(pybind11::module& m);
void register_fused(pybind11::module& m);
void register_bn(pybind11::module& m);
void register_rccl(pybind11::module& m);
void register_gemm(pybind11::module& m);
void register_conv(pybind11::module& m);
void register_head(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "p2pfl_amd native HIP/CDNA4 kernels (gfx950)";
  m.def("weighted_sum", &weighted_sum,
        "out = scale * (acc_in + sum_i w_i * src_i) (flat arenas, fp32/bf16 in, fp32/bf16 out, fp32 running sum)",
        pybind11::arg("srcs"), pybind11::arg("weights"), pybind11::arg("out"), pybind11::arg("acc_in") = pybind11::none(),
        pybind11::arg("scale") = 1.0);
  m.def("adam_step", &adam_step, "fused whole-arena Adam/AdamW step");
  m.def("sgd_step", &sgd_step, "fused whole-arena SGD(+momentum/nesterov) step");
  m.def("adam_mt_step", &adam_mt_step, "multi-tensor Adam/AdamW over per-tensor grads into flat fp32 state",
        pybind11::arg("p"), pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("pbf"), pybind11::arg("tens"),
        pybind11::arg("chunks"), pybind11::arg("grads"), pybind11::arg("numels"), pybind11::arg("grad_bf16"), pybind11::arg("grad_cl"),
        pybind11::arg("lr"), pybind11::arg("beta1"), pybind11::arg("beta2"), pybind11::arg("eps"),
        pybind11::arg("weight_decay"), pybind11::arg("step"), pybind11::arg("decoupled"),
        pybind11::arg("gtab") = pybind11::none(), pybind11::arg("t_dev") = pybind11::none());
  m.def("sgd_mt_step", &sgd_mt_step, "multi-tensor SGD over per-tensor grads into flat fp32 state", pybind11::arg("p"),
        pybind11::arg("buf"), pybind11::arg("pbf"), pybind11::arg("tens"), pybind11::arg("chunks"),
        pybind11::arg("grads"), pybind11::arg("numels"), pybind11::arg("grad_bf16"), pybind11::arg("grad_cl"), pybind11::arg("lr"),
        pybind11::arg("momentum"), pybind11::arg("dampening"), pybind11::arg("weight_decay"),
        pybind11::arg("nesterov"), pybind11::arg("first_step"), pybind11::arg("gtab") = pybind11::none());
  m.def("new_stream", &new_stream, "create a private non-blocking HIP stream on a device (returns its handle)",
        pybind11::arg("device"), pybind11::arg("priority") = 0);
  m.def("destroy_stream", &destroy_stream, "destroy a stream made by new_stream");
  register_cnn(m);
  register_fused(m);
  register_bn(m);
  register_rccl(m);
  register_gemm(m);
  register_conv(m);
  register_head(m);
}
