// PyTorch bindings of the fused BatchNorm kernels (batchnorm.hip).
// Activations are [M, C] views of channels-last NHWC tensors.
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "batchnorm.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

bool act(const torch::Tensor& t, const torch::Tensor& like, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 2, name, " must be a contiguous [M, C] GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name, " must be bf16 or fp32");
  TORCH_CHECK(t.sizes() == like.sizes() && t.scalar_type() == like.scalar_type() && t.device() == like.device(), name,
              " must match x");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
  return t.scalar_type() == torch::kBFloat16;
}

float* f32(const torch::Tensor& t, int64_t C, const torch::Tensor& x, const char* name) {
  TORCH_CHECK(t.device() == x.device() && t.is_contiguous() && t.scalar_type() == torch::kFloat32 && t.numel() == C,
              name, " must be a contiguous fp32 [C] tensor on x's device");
  return t.data_ptr<float>();
}

float* opt_f32(const c10::optional<torch::Tensor>& t, int64_t C, const torch::Tensor& x, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  return f32(*t, C, x, name);
}

// zeroed int32 arrival counter of the statistics + finalize kernels (ops/splitk.py ring), or null
int* opt_ctr(const c10::optional<torch::Tensor>& t, const torch::Tensor& x) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->device() == x.device() && t->scalar_type() == torch::kInt32 && t->numel() >= 1,
              "counters must be a zeroed int32 tensor on x's device");
  return t->data_ptr<int>();
}

// partial rows for whichever kernel runs
int64_t part_rows(int64_t M, int64_t C, bool fused) {
  const auto p = p2bn::bn_plan(int(M), int(C));
  const auto f = p2bn::bn_fused_plan(int(M), int(C));
  return fused && f.S > p.S ? f.S : p.S;
}

void check_shape(const torch::Tensor& x) {
  TORCH_CHECK(x.dim() == 2, "x must be [M, C]");
  const int64_t M = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0 && C > 0, "C must be a positive multiple of 8");
  TORCH_CHECK(M > 0 && M * C < (int64_t(1) << 31) * 8 && M < (int64_t(1) << 31), "M out of range");
}

// returns {y, mean, rstd}
std::vector<torch::Tensor> bn_fwd_train(torch::Tensor x, torch::Tensor w, torch::Tensor b,
                                        c10::optional<torch::Tensor> residual,
                                        c10::optional<torch::Tensor> running_mean,
                                        c10::optional<torch::Tensor> running_var,
                                        c10::optional<torch::Tensor> num_batches_tracked, double momentum, double eps,
                                        bool relu, c10::optional<torch::Tensor> counters) {
  const c10::DeviceGuard g(x.device());
  check_shape(x);
  const int64_t M = x.size(0), C = x.size(1);
  const bool bf = act(x, x, "x");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    act(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  float* rm = opt_f32(running_mean, C, x, "running_mean");
  float* rv = opt_f32(running_var, C, x, "running_var");
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean and running_var go together");
  int64_t* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->device() == x.device() && num_batches_tracked->scalar_type() == torch::kInt64 &&
                    num_batches_tracked->numel() == 1,
                "num_batches_tracked must be an int64 scalar on x's device");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  auto y = torch::empty_like(x);
  auto opt = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({C}, opt), rstd = torch::empty({C}, opt), coef = torch::empty({3, C}, opt);
  int* ctr = opt_ctr(counters, x);
  auto part = torch::empty({2, part_rows(M, C, ctr != nullptr), C}, opt);
  p2bn::bn_fwd_train(bf, x.data_ptr(), rp, f32(w, C, x, "weight"), f32(b, C, x, "bias"), rm, rv, nbt, float(momentum),
                     float(eps), y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), coef.data_ptr<float>(),
                     part.data_ptr<float>(), ctr, int(M), int(C), relu, stream());
  return {y, mean, rstd};
}

// y = act((x - coef[0]) * coef[1] + coef[2] [+ residual]) with precomputed coefficients
torch::Tensor bn_apply_train(torch::Tensor x, c10::optional<torch::Tensor> residual, torch::Tensor coef, bool relu) {
  const c10::DeviceGuard g(x.device());
  check_shape(x);
  const int64_t M = x.size(0), C = x.size(1);
  const bool bf = act(x, x, "x");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    act(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  TORCH_CHECK(coef.device() == x.device() && coef.is_contiguous() && coef.scalar_type() == torch::kFloat32 &&
                  coef.numel() == 3 * C,
              "coef must be a contiguous fp32 [3, C] tensor on x's device");
  auto y = torch::empty_like(x);
  p2bn::bn_apply_train(bf, x.data_ptr(), rp, coef.data_ptr<float>(), y.data_ptr(), int(M), int(C), relu, stream());
  return y;
}

// dx = A dz' + B (x - mean) + D (bf16 [M, C]); y: BN output (ReLU mask) or undefined
torch::Tensor bn_apply_bwd(torch::Tensor dy, c10::optional<torch::Tensor> y, torch::Tensor x, torch::Tensor mean,
                           torch::Tensor coef) {
  const c10::DeviceGuard g(x.device());
  check_shape(x);
  const int64_t M = x.size(0), C = x.size(1);
  TORCH_CHECK(act(x, x, "x"), "apply_bwd: bf16 only");
  act(dy, x, "dy");
  const bool relu = y.has_value() && y->defined();
  if (relu) act(*y, x, "y");
  TORCH_CHECK(coef.device() == x.device() && coef.is_contiguous() && coef.scalar_type() == torch::kFloat32 &&
                  coef.numel() == 3 * C,
              "coef must be a contiguous fp32 [3, C] tensor on x's device");
  auto dx = torch::empty_like(x);
  p2bn::bn_apply_bwd_only(dy.data_ptr(), relu ? y->data_ptr() : nullptr, x.data_ptr(), f32(mean, C, x, "mean"),
                          coef.data_ptr<float>(), dx.data_ptr(), int(M), int(C), relu, stream());
  return dx;
}

torch::Tensor bn_fwd_eval(torch::Tensor x, torch::Tensor w, torch::Tensor b, c10::optional<torch::Tensor> residual,
                          torch::Tensor running_mean, torch::Tensor running_var, double eps, bool relu) {
  const c10::DeviceGuard g(x.device());
  check_shape(x);
  const int64_t M = x.size(0), C = x.size(1);
  const bool bf = act(x, x, "x");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    act(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  for (const auto* t : {&w, &b, &running_mean, &running_var})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "eval BN parameters must be 16-byte aligned");
  auto y = torch::empty_like(x);
  auto coef = torch::empty({3, C}, x.options().dtype(torch::kFloat32));
  p2bn::bn_fwd_eval(bf, x.data_ptr(), rp, f32(w, C, x, "weight"), f32(b, C, x, "bias"),
                    f32(running_mean, C, x, "running_mean"), f32(running_var, C, x, "running_var"), float(eps),
                    y.data_ptr(), coef.data_ptr<float>(), int(M), int(C), relu, stream());
  return y;
}

// returns {dx, dw, db} or {dx, dw, db, dres}; dy2 (optional): a second gradient of the output, summed with dy
std::vector<torch::Tensor> bn_bwd(torch::Tensor dy, torch::Tensor y, torch::Tensor x, torch::Tensor w,
                                  torch::Tensor mean, torch::Tensor rstd, bool relu, bool need_dres,
                                  c10::optional<torch::Tensor> counters, c10::optional<torch::Tensor> dy2) {
  const c10::DeviceGuard g(x.device());
  check_shape(x);
  const int64_t M = x.size(0), C = x.size(1);
  const bool bf = act(x, x, "x");
  act(dy, x, "dy");
  const bool two = dy2.has_value() && dy2->defined();
  if (two) act(*dy2, x, "dy2");
  if (relu) act(y, x, "y");
  auto dx = torch::empty_like(x);
  auto dres = need_dres ? torch::empty_like(x) : torch::Tensor();
  auto opt = x.options().dtype(torch::kFloat32);
  auto dw = torch::empty({C}, opt), db = torch::empty({C}, opt), coef = torch::empty({3, C}, opt);
  int* ctr = opt_ctr(counters, x);
  auto part = torch::empty({2, part_rows(M, C, ctr != nullptr), C}, opt);
  p2bn::bn_bwd(bf, dy.data_ptr(), two ? dy2->data_ptr() : nullptr, relu ? y.data_ptr() : nullptr, x.data_ptr(), f32(w, C, x, "weight"),
               f32(mean, C, x, "mean"), f32(rstd, C, x, "rstd"), dx.data_ptr(), need_dres ? dres.data_ptr() : nullptr,
               dw.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(), part.data_ptr<float>(), ctr, int(M),
               int(C), relu, stream());
  if (need_dres) return {dx, dw, db, dres};
  return {dx, dw, db};
}

}  // namespace

void register_bn(pybind11::module& m) {
  namespace py = pybind11;
  auto f = m.def_submodule("bn", "fused BatchNorm (+ residual) (+ ReLU) on channels-last [M, C] activations");
  f.def("fwd_train", &bn_fwd_train, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("residual") = py::none(),
        py::arg("running_mean") = py::none(), py::arg("running_var") = py::none(),
        py::arg("num_batches_tracked") = py::none(), py::arg("momentum") = 0.1, py::arg("eps") = 1e-5,
        py::arg("relu") = true, py::arg("counters") = py::none());
  f.def("apply_train", &bn_apply_train, py::arg("x"), py::arg("residual"), py::arg("coef"), py::arg("relu"));
  f.def("apply_bwd", &bn_apply_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("mean"), py::arg("coef"));
  f.def("fwd_eval", &bn_fwd_eval, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("residual") = py::none(),
        py::arg("running_mean"), py::arg("running_var"), py::arg("eps") = 1e-5, py::arg("relu") = true);
  f.def("bwd", &bn_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("w"), py::arg("mean"), py::arg("rstd"),
        py::arg("relu"), py::arg("need_dres"), py::arg("counters") = py::none(), py::arg("dy2") = py::none());
  f.def("fused_rows", [](int64_t M, int64_t C) { return p2bn::bn_fused_plan(int(M), int(C)).S; },
        "partial rows of the statistics + finalize kernels for an [M, C] activation (0: not eligible)");
}
