// PyTorch bindings of the classification-head kernels (csrc/head.hip):
// global average pool + Linear (N <= 64) + softmax cross-entropy in one
// launch forward and one backward.  Every shape / dtype / device assumption of
// the kernels is checked here.
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace p2 {
void head_fwd(const uint16_t* f, const void* w, int w_bf16, const float* bias, const int64_t* y, float* pooled,
              float* logits, float* loss_rows, float* loss, float* acc, int* ctr, int B, int HW, int C, int N,
              hipStream_t s);
void head_bwd(const float* gloss, const float* logits, const int64_t* y, const float* pooled, const void* w, int w_bf16,
              uint16_t* df, void* dw, float* db, int B, int HW, int C, int N, hipStream_t s);
}  // namespace p2

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_w(const torch::Tensor& w, const torch::Tensor& f, int64_t C) {
  TORCH_CHECK(w.is_cuda() && w.device() == f.device() && w.dim() == 2 && w.is_contiguous() && w.size(1) == C &&
                  (w.scalar_type() == torch::kFloat32 || w.scalar_type() == torch::kBFloat16),
              "head: w must be a contiguous fp32/bf16 [N, C] tensor on f's device");
  TORCH_CHECK(w.size(0) >= 1 && w.size(0) <= 64, "head: 1 <= N <= 64 classes");
}

// f: [B, H, W, C] bf16 contiguous (channels-last storage) -> {pooled [B, C], logits [B, N], mean loss (), accuracy ()}
std::vector<torch::Tensor> head_fwd(torch::Tensor f, torch::Tensor w, c10::optional<torch::Tensor> bias,
                                    c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> counter) {
  TORCH_CHECK(f.is_cuda() && f.scalar_type() == torch::kBFloat16 && f.dim() == 4 && f.is_contiguous(),
              "head: f must be a contiguous bf16 [B, H, W, C] GPU tensor");
  const int64_t B = f.size(0), HW = f.size(1) * f.size(2), C = f.size(3);
  TORCH_CHECK(B >= 1 && HW >= 1 && C >= 1 && B * HW * C < (int64_t(1) << 31), "head: bad feature shape");
  check_w(w, f, C);
  const int64_t N = w.size(0);
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->device() == f.device() && bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() &&
                    bias->numel() == N,
                "head: bias must be a contiguous fp32 [N] tensor");
    bp = bias->data_ptr<float>();
  }
  const int64_t* yp = nullptr;
  int* cp = nullptr;
  if (y.has_value() && y->defined()) {
    TORCH_CHECK(y->device() == f.device() && y->scalar_type() == torch::kInt64 && y->is_contiguous() && y->numel() == B,
                "head: y must be a contiguous int64 [B] tensor");
    TORCH_CHECK(counter.has_value() && counter->defined() && counter->device() == f.device() &&
                    counter->scalar_type() == torch::kInt32 && counter->numel() >= 1,
                "head: a loss needs a zeroed int32 counter");
    yp = y->data_ptr<int64_t>();
    cp = counter->data_ptr<int>();
  }
  auto opt = f.options().dtype(torch::kFloat32);
  auto pooled = torch::empty({B, C}, opt), logits = torch::empty({B, N}, opt);
  auto rows = torch::empty({2 * B}, opt), loss = torch::empty({}, opt), acc = torch::empty({}, opt);
  const c10::DeviceGuard g(f.device());
  p2::head_fwd(reinterpret_cast<const uint16_t*>(f.data_ptr()), w.data_ptr(), w.scalar_type() == torch::kBFloat16, bp, yp,
               pooled.data_ptr<float>(), logits.data_ptr<float>(), rows.data_ptr<float>(), loss.data_ptr<float>(),
               acc.data_ptr<float>(), cp,
               int(B), int(HW), int(C), int(N), stream());
  return {pooled, logits, loss, acc};
}

// -> {df [B, H, W, C] bf16, dw [N, C] (w's dtype), db [N] fp32}
std::vector<torch::Tensor> head_bwd(torch::Tensor gloss, torch::Tensor logits, torch::Tensor y, torch::Tensor pooled,
                                    torch::Tensor w, std::vector<int64_t> fshape) {
  TORCH_CHECK(fshape.size() == 4, "head_bwd: fshape is (B, H, W, C)");
  const int64_t B = fshape[0], HW = fshape[1] * fshape[2], C = fshape[3];
  TORCH_CHECK(pooled.is_cuda() && pooled.scalar_type() == torch::kFloat32 && pooled.is_contiguous() &&
                  pooled.numel() == B * C,
              "head_bwd: pooled must be fp32 [B, C]");
  check_w(w, pooled, C);
  const int64_t N = w.size(0);
  TORCH_CHECK(logits.device() == pooled.device() && logits.scalar_type() == torch::kFloat32 && logits.is_contiguous() &&
                  logits.numel() == B * N,
              "head_bwd: logits must be fp32 [B, N]");
  TORCH_CHECK(y.device() == pooled.device() && y.scalar_type() == torch::kInt64 && y.is_contiguous() && y.numel() == B,
              "head_bwd: y must be int64 [B]");
  TORCH_CHECK(gloss.device() == pooled.device() && gloss.scalar_type() == torch::kFloat32 && gloss.numel() == 1,
              "head_bwd: gloss must be an fp32 scalar tensor");
  auto gl = gloss.contiguous();
  auto df = torch::empty({B, fshape[1], fshape[2], C}, pooled.options().dtype(torch::kBFloat16));
  auto dw = torch::empty_like(w);
  auto db = torch::empty({N}, pooled.options());
  const c10::DeviceGuard g(pooled.device());
  p2::head_bwd(gl.data_ptr<float>(), logits.data_ptr<float>(), y.data_ptr<int64_t>(), pooled.data_ptr<float>(),
               w.data_ptr(), w.scalar_type() == torch::kBFloat16, reinterpret_cast<uint16_t*>(df.data_ptr()), dw.data_ptr(),
               db.data_ptr<float>(), int(B), int(HW), int(C), int(N), stream());
  return {df, dw, db};
}

}  // namespace

void register_head(pybind11::module& m) {
  namespace py = pybind11;
  auto h = m.def_submodule("head", "global average pool + Linear + softmax cross-entropy (two launches)");
  h.def("fwd", &head_fwd, py::arg("f"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("counter"));
  h.def("bwd", &head_bwd, py::arg("gloss"), py::arg("logits"), py::arg("y"), py::arg("pooled"), py::arg("w"),
        py::arg("fshape"));
}
