// torch bindings of the gfx950 kernels (module `_C`).  Validates shapes/dtypes/devices,
// allocates outputs and launches on the current HIP stream.  No fallbacks: a failing
// launch raises.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include "kernels.h"

namespace {

int dt_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat:
      return smpk::F32;
    case at::kHalf:
      return smpk::F16;
    case at::kBFloat16:
      return smpk::BF16;
    default:
      TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " launch failed with code ", rc); }

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

const void* opt_ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------ optimizers
void fused_adam(c10::optional<at::Tensor> param, at::Tensor grad, at::Tensor master, at::Tensor m, at::Tensor v,
                double lr, double beta1, double beta2, double eps, double wd, double bc1, double bc2,
                double grad_scale, bool adamw) {
  check_gpu(grad, "grad");
  check_gpu(master, "master");
  TORCH_CHECK(master.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "fused_adam: master/m/v must be fp32");
  const int64_t n = master.numel();
  TORCH_CHECK(grad.numel() == n && m.numel() == n && v.numel() == n, "fused_adam: size mismatch");
  if (param.has_value()) TORCH_CHECK(param->numel() == n && param->is_contiguous(), "fused_adam: bad param");
  check(smpk::fused_adam(param.has_value() ? dt_code(*param) : 0, param.has_value() ? param->data_ptr() : nullptr,
                         dt_code(grad), grad.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                         v.data_ptr<float>(), n, lr, beta1, beta2, eps, wd, bc1, bc2, grad_scale, adamw ? 1 : 0,
                         stream()),
        "fused_adam");
}

void fused_sgd(c10::optional<at::Tensor> param, at::Tensor grad, at::Tensor master, c10::optional<at::Tensor> mom,
               double lr, double momentum, double dampening, double wd, bool nesterov, bool first, double grad_scale) {
  check_gpu(grad, "grad");
  const int64_t n = master.numel();
  check(smpk::fused_sgd(param.has_value() ? dt_code(*param) : 0, param.has_value() ? param->data_ptr() : nullptr,
                        dt_code(grad), grad.data_ptr(), master.data_ptr<float>(),
                        mom.has_value() ? mom->data_ptr<float>() : nullptr, n, lr, momentum, dampening, wd,
                        nesterov ? 1 : 0, first ? 1 : 0, grad_scale, stream()),
        "fused_sgd");
}

void fused_adagrad(c10::optional<at::Tensor> param, at::Tensor grad, at::Tensor master, at::Tensor sum, double lr,
                   double eps, double wd, double grad_scale) {
  check_gpu(grad, "grad");
  check(smpk::fused_adagrad(param.has_value() ? dt_code(*param) : 0,
                            param.has_value() ? param->data_ptr() : nullptr, dt_code(grad), grad.data_ptr(),
                            master.data_ptr<float>(), sum.data_ptr<float>(), master.numel(), lr, eps, wd, grad_scale,
                            stream()),
        "fused_adagrad");
}

void lamb_stage1(at::Tensor grad, at::Tensor master, at::Tensor m, at::Tensor v, at::Tensor update, double beta1,
                 double beta2, double eps, double wd, double bc1, double bc2, double grad_scale) {
  check_gpu(grad, "grad");
  check(smpk::lamb_stage1(dt_code(grad), grad.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                          v.data_ptr<float>(), update.data_ptr<float>(), master.numel(), beta1, beta2, eps, wd, bc1,
                          bc2, grad_scale, stream()),
        "lamb_stage1");
}

void lamb_stage2(c10::optional<at::Tensor> param, at::Tensor master, at::Tensor update, double lr, at::Tensor pn,
                 at::Tensor un, bool use_trust) {
  check(smpk::lamb_stage2(param.has_value() ? dt_code(*param) : 0, param.has_value() ? param->data_ptr() : nullptr,
                          master.data_ptr<float>(), update.data_ptr<float>(), master.numel(), lr, pn.data_ptr<float>(),
                          un.data_ptr<float>(), use_trust ? 1 : 0, stream()),
        "lamb_stage2");
}

void sumsq_(at::Tensor x, at::Tensor out, double scale) {
  check_gpu(x, "x");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_cuda(), "out must be fp32 GPU");
  check(smpk::sumsq(dt_code(x), x.data_ptr(), x.numel(), scale, out.data_ptr<float>(), stream()), "sumsq");
}

void nonfinite_(at::Tensor x, at::Tensor out) {
  check_gpu(x, "x");
  check(smpk::nonfinite(dt_code(x), x.data_ptr(), x.numel(), out.data_ptr<float>(), stream()), "nonfinite");
}

void axpby_(at::Tensor x, at::Tensor y, double a, double b) {
  check_gpu(x, "x");
  check_gpu(y, "y");
  TORCH_CHECK(x.scalar_type() == y.scalar_type() && x.numel() == y.numel(), "axpby: mismatch");
  check(smpk::axpby(dt_code(x), x.data_ptr(), y.data_ptr(), x.numel(), a, b, stream()), "axpby");
}

void cast_copy_(at::Tensor src, at::Tensor dst, double scale) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "cast_copy: size mismatch");
  check(smpk::cast_copy(dt_code(src), src.data_ptr(), dt_code(dst), dst.data_ptr(), src.numel(), scale, stream()),
        "cast_copy");
}

// ------------------------------------------------------------------- layernorm
std::vector<at::Tensor> layernorm_fwd(at::Tensor x, c10::optional<at::Tensor> residual,
                                      c10::optional<at::Tensor> w, c10::optional<at::Tensor> b, double eps) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  auto y = at::empty_like(x);
  auto opts = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, opts);
  auto rstd = at::empty({rows}, opts);
  at::Tensor xo;
  if (residual.has_value()) {
    check_gpu(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual mismatch");
    xo = at::empty_like(x);
  }
  int wdt = w.has_value() ? dt_code(*w) : dt_code(x);
  if (w.has_value()) TORCH_CHECK(w->numel() == cols && w->is_contiguous(), "weight mismatch");
  if (b.has_value()) TORCH_CHECK(b->numel() == cols && b->is_contiguous() && dt_code(*b) == wdt, "bias mismatch");
  check(smpk::layernorm_fwd(dt_code(x), x.data_ptr(), opt_ptr(residual), residual.has_value() ? xo.data_ptr() : nullptr,
                            wdt, opt_ptr(w), opt_ptr(b), y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                            rows, cols, eps, stream()),
        "layernorm_fwd");
  if (residual.has_value()) return {y, mean, rstd, xo};
  return {y, mean, rstd};
}

std::vector<at::Tensor> layernorm_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> w, at::Tensor mean,
                                      at::Tensor rstd, bool need_wgrad, bool need_bgrad,
                                      c10::optional<at::Tensor> dres) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  auto dx = at::empty_like(x);
  const bool aligned = ((reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(dy.data_ptr()) |
                         reinterpret_cast<uintptr_t>(dx.data_ptr()) |
                         (dres.has_value() ? reinterpret_cast<uintptr_t>(dres->data_ptr()) : 0)) &
                        15) == 0;
  const int parts = smpk::layernorm_bwd_num_parts(dt_code(x), rows, cols, aligned);
  at::Tensor dwp, dbp, dw, db;
  int wdt = w.has_value() ? dt_code(*w) : dt_code(x);
  if (need_wgrad || need_bgrad) {
    auto fo = x.options().dtype(at::kFloat);
    dwp = at::empty({parts, cols}, fo);
    dbp = at::empty({parts, cols}, fo);
  }
  if (dres.has_value()) {
    check_gpu(*dres, "dres");
    TORCH_CHECK(dres->sizes() == x.sizes(), "dres mismatch");
  }
  check(smpk::layernorm_bwd(dt_code(x), dy.data_ptr(), x.data_ptr(), wdt, opt_ptr(w), mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), dx.data_ptr(), dwp.defined() ? dwp.data_ptr<float>() : nullptr,
                            dbp.defined() ? dbp.data_ptr<float>() : nullptr, rows, cols, parts, opt_ptr(dres),
                            stream()),
        "layernorm_bwd");
  if (dwp.defined()) {
    auto wo = w.has_value() ? w->options() : x.options();
    dw = at::empty({cols}, wo);
    db = at::empty({cols}, wo);
    check(smpk::layernorm_bwd_reduce(wdt, dwp.data_ptr<float>(), dbp.data_ptr<float>(), dw.data_ptr(), db.data_ptr(),
                                     parts, cols, stream()),
          "layernorm_bwd_reduce");
  }
  return {dx, dw, db};
}

at::Tensor layernorm_apply_stats(at::Tensor x, c10::optional<at::Tensor> w, c10::optional<at::Tensor> b,
                                 at::Tensor mean, at::Tensor var, at::Tensor rstd_out, double eps) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  auto y = at::empty_like(x);
  int wdt = w.has_value() ? dt_code(*w) : dt_code(x);
  check(smpk::layernorm_apply_stats(dt_code(x), x.data_ptr(), wdt, opt_ptr(w), opt_ptr(b), mean.data_ptr<float>(),
                                    var.data_ptr<float>(), y.data_ptr(), rstd_out.data_ptr<float>(), rows, cols, eps,
                                    stream()),
        "layernorm_apply_stats");
  return y;
}

// ------------------------------------------------------------------------ gelu
at::Tensor bias_gelu_fwd(at::Tensor x, c10::optional<at::Tensor> bias) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  if (bias.has_value()) TORCH_CHECK(bias->numel() == cols && bias->scalar_type() == x.scalar_type(), "bias mismatch");
  auto y = at::empty_like(x);
  check(smpk::bias_gelu_fwd(dt_code(x), x.data_ptr(), opt_ptr(bias), y.data_ptr(), x.numel() / cols, cols, stream()),
        "bias_gelu_fwd");
  return y;
}

at::Tensor bias_gelu_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> bias) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  auto dx = at::empty_like(x);
  check(smpk::bias_gelu_bwd(dt_code(x), dy.data_ptr(), x.data_ptr(), opt_ptr(bias), dx.data_ptr(), x.numel() / cols,
                            cols, stream()),
        "bias_gelu_bwd");
  return dx;
}

at::Tensor col_sum(at::Tensor x) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  int64_t parts = (rows + 63) / 64;
  if (parts > 256) parts = 256;
  auto ws = at::empty({std::max<int64_t>(parts, 1), cols}, x.options().dtype(at::kFloat));
  auto out = at::empty({cols}, x.options());
  check(smpk::col_sum(dt_code(x), x.data_ptr(), out.data_ptr(), ws.data_ptr<float>(), rows, cols, stream()), "col_sum");
  return out;
}

// --------------------------------------------------------------------- softmax
at::Tensor scaled_masked_softmax_fwd(at::Tensor x, c10::optional<at::Tensor> mask, double scale) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 4, "x must be [b, np, sq, sk]");
  auto y = at::empty_like(x);
  int64_t mb = 1;
  const uint8_t* mp = nullptr;
  if (mask.has_value()) {
    check_gpu(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == at::kByte || mask->scalar_type() == at::kBool, "mask must be uint8/bool");
    TORCH_CHECK(mask->dim() == 4 && mask->size(1) == 1 && mask->size(2) == x.size(2) && mask->size(3) == x.size(3),
                "mask must be [b, 1, sq, sk]");
    mb = mask->size(0);
    mp = static_cast<const uint8_t*>(mask->data_ptr());
  }
  check(smpk::scaled_masked_softmax_fwd(dt_code(x), x.data_ptr(), mp, y.data_ptr(), x.size(0), x.size(1), x.size(2),
                                        x.size(3), mb, scale, stream()),
        "scaled_masked_softmax_fwd");
  return y;
}

at::Tensor scaled_upper_triang_softmax_fwd(at::Tensor x, double scale) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 3, "x must be [attn_batches, sq, sk]");
  auto y = at::empty_like(x);
  check(smpk::scaled_upper_triang_softmax_fwd(dt_code(x), x.data_ptr(), y.data_ptr(), x.size(0), x.size(1), x.size(2),
                                              scale, stream()),
        "scaled_upper_triang_softmax_fwd");
  return y;
}

at::Tensor scaled_softmax_bwd(at::Tensor dy, at::Tensor y, double scale) {
  check_gpu(dy, "dy");
  check_gpu(y, "y");
  auto dx = at::empty_like(y);
  const int64_t cols = y.size(-1);
  check(smpk::scaled_softmax_bwd(dt_code(y), dy.data_ptr(), y.data_ptr(), dx.data_ptr(), y.numel() / cols, cols, scale,
                                 stream()),
        "scaled_softmax_bwd");
  return dx;
}

// --------------------------------------------------------------- cross entropy
std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor target, int64_t vocab_start, int64_t ignore_index) {
  check_gpu(logits, "logits");
  check_gpu(target, "target");
  TORCH_CHECK(logits.dim() == 2 && target.dim() == 1 && target.size(0) == logits.size(0), "xent_fwd: shapes");
  TORCH_CHECK(target.scalar_type() == at::kLong, "target must be int64");
  const int64_t rows = logits.size(0), vocab = logits.size(1);
  auto fo = logits.options().dtype(at::kFloat);
  auto mx = at::empty({rows}, fo), se = at::empty({rows}, fo), tl = at::empty({rows}, fo);
  check(smpk::xent_fwd_stats(dt_code(logits), logits.data_ptr(), target.data_ptr<int64_t>(), rows, vocab, vocab_start,
                             mx.data_ptr<float>(), se.data_ptr<float>(), tl.data_ptr<float>(), ignore_index, stream()),
        "xent_fwd");
  return {mx, se, tl};
}

at::Tensor xent_bwd(at::Tensor logits, at::Tensor target, at::Tensor lse, at::Tensor grad_rows, int64_t vocab_start,
                    int64_t ignore_index) {
  check_gpu(logits, "logits");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && grad_rows.scalar_type() == at::kFloat, "lse/grad must be fp32");
  TORCH_CHECK(grad_rows.is_contiguous() && lse.is_contiguous(), "lse/grad contiguous");
  auto d = at::empty_like(logits);
  check(smpk::xent_bwd(dt_code(logits), logits.data_ptr(), target.data_ptr<int64_t>(), lse.data_ptr<float>(),
                       grad_rows.data_ptr<float>(), d.data_ptr(), logits.size(0), logits.size(1), vocab_start,
                       ignore_index, stream()),
        "xent_bwd");
  return d;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "smdistributed_modelparallel_amd CDNA4 (gfx950) kernels";
  m.def("fused_adam", &fused_adam);
  m.def("fused_sgd", &fused_sgd);
  m.def("fused_adagrad", &fused_adagrad);
  m.def("lamb_stage1", &lamb_stage1);
  m.def("lamb_stage2", &lamb_stage2);
  m.def("sumsq_", &sumsq_);
  m.def("nonfinite_", &nonfinite_);
  m.def("axpby_", &axpby_);
  m.def("cast_copy_", &cast_copy_);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("layernorm_apply_stats", &layernorm_apply_stats);
  m.def("bias_gelu_fwd", &bias_gelu_fwd);
  m.def("bias_gelu_bwd", &bias_gelu_bwd);
  m.def("col_sum", &col_sum);
  m.def("scaled_masked_softmax_fwd", &scaled_masked_softmax_fwd);
  m.def("scaled_upper_triang_softmax_fwd", &scaled_upper_triang_softmax_fwd);
  m.def("scaled_softmax_bwd", &scaled_softmax_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
}
