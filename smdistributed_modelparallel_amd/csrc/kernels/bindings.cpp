// torch bindings of the gfx950 kernels (module `_C`).  Validates shapes/dtypes/devices,
// allocates outputs and launches on the current HIP stream.  No fallbacks: a failing
// launch raises.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include "kernels.h"
#include "../torchrt/torchrt.h"

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

// ---------------------------------------------------------- multi-tensor apply
// meta: int64 GPU tensor = 6 x nt role pointers + nchunks x 3 chunk ranges (ops/multi_tensor.py
// MTMeta); g0 / p0: first grad / param of the list (their dtypes select the kernel)
const int64_t* mt_meta(const at::Tensor& meta, int64_t nt, int64_t nchunks) {
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous(), "mt: meta must be int64 GPU");
  TORCH_CHECK(meta.numel() == 6 * nt + 3 * nchunks, "mt: meta size mismatch");
  return meta.data_ptr<int64_t>();
}

void mt_adam(at::Tensor meta, int64_t nt, int64_t nchunks, at::Tensor g0, at::Tensor p0, bool master, double lr,
             double b1, double b2, double eps, double wd, double bc1, double bc2, double gscale, bool adamw) {
  check(smpk::mt_adam(mt_meta(meta, nt, nchunks), nt, nchunks, dt_code(p0), dt_code(g0), master ? 1 : 0, lr, b1, b2,
                      eps, wd, bc1, bc2, gscale, adamw ? 1 : 0, stream()),
        "mt_adam");
}

void mt_norm(at::Tensor meta, int64_t nt, int64_t nchunks, int64_t role, at::Tensor sample, at::Tensor out,
             double scale, bool maxabs) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() >= nt, "mt_norm: bad out");
  check(smpk::mt_norm(mt_meta(meta, nt, nchunks), nt, nchunks, static_cast<int>(role), dt_code(sample), scale,
                      maxabs ? 1 : 0, out.data_ptr<float>(), stream()),
        "mt_norm");
}

void mt_lamb1(at::Tensor meta, int64_t nt, int64_t nchunks, at::Tensor g0, at::Tensor p0, bool master, double b1,
              double b2, double b3, double bc1, double bc2, double eps, double wd, bool decoupled, at::Tensor gnorm,
              double max_gnorm, double gscale) {
  TORCH_CHECK(gnorm.is_cuda() && gnorm.scalar_type() == at::kFloat, "mt_lamb1: gnorm must be a float GPU tensor");
  check(smpk::mt_lamb1(mt_meta(meta, nt, nchunks), nt, nchunks, dt_code(p0), dt_code(g0), master ? 1 : 0, b1, b2, b3,
                       bc1, bc2, eps, wd, decoupled ? 1 : 0, gnorm.data_ptr<float>(), max_gnorm, gscale, stream()),
        "mt_lamb1");
}

void mt_lamb2(at::Tensor meta, int64_t nt, int64_t nchunks, at::Tensor p0, bool master, at::Tensor pn2, at::Tensor un2,
              double lr, bool use_trust) {
  check(smpk::mt_lamb2(mt_meta(meta, nt, nchunks), nt, nchunks, dt_code(p0), master ? 1 : 0, pn2.data_ptr<float>(),
                       un2.data_ptr<float>(), lr, use_trust ? 1 : 0, stream()),
        "mt_lamb2");
}

void mt_novograd(at::Tensor meta, int64_t nt, int64_t nchunks, at::Tensor g0, at::Tensor p0, bool master,
                 at::Tensor norms, double b1, double b3, double bc1, double bc2, double eps, double lr, double wd,
                 bool decoupled, double gscale) {
  check(smpk::mt_novograd(mt_meta(meta, nt, nchunks), nt, nchunks, dt_code(p0), dt_code(g0), master ? 1 : 0,
                          norms.data_ptr<float>(), b1, b3, bc1, bc2, eps, lr, wd, decoupled ? 1 : 0, gscale, stream()),
        "mt_novograd");
}

void novograd_blend(at::Tensor norms, at::Tensor fresh, double b2, bool l2, bool first, bool init_zero) {
  TORCH_CHECK(norms.is_cuda() && fresh.is_cuda() && norms.numel() == fresh.numel(), "novograd_blend: bad tensors");
  check(smpk::novograd_blend(norms.data_ptr<float>(), fresh.data_ptr<float>(), norms.numel(), b2, l2 ? 1 : 0,
                             first ? 1 : 0, init_zero ? 1 : 0, stream()),
        "novograd_blend");
}

void lamb_stage1(at::Tensor grad, at::Tensor master, at::Tensor m, at::Tensor v, at::Tensor update, double beta1,
                 double beta2, double eps, double wd, double bc1, double bc2, double grad_scale) {
  check_gpu(grad, "grad");
  check(smpk::lamb_stage1(dt_code(grad), grad.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                          v.data_ptr<float>(), update.data_ptr<float>(), master.numel(), beta1, beta2, eps, wd, bc1,
                          bc2, grad_scale, stream()),
        "lamb_stage1");
}

// Whole-domain LAMB stage 2: per-segment norms then the trust-scaled update, two launches.
void lamb_chunked(c10::optional<at::Tensor> param, at::Tensor master, at::Tensor update, at::Tensor chunks,
                  int64_t nseg, double lr, bool use_trust) {
  check_gpu(master, "master");
  check_gpu(update, "update");
  check_gpu(chunks, "chunks");
  TORCH_CHECK(chunks.scalar_type() == at::kLong && chunks.dim() == 2 && chunks.size(1) == 3, "chunks: [n, 3] int64");
  TORCH_CHECK(master.scalar_type() == at::kFloat && update.scalar_type() == at::kFloat, "master/update fp32");
  TORCH_CHECK(update.numel() == master.numel(), "update size");
  if (param.has_value()) TORCH_CHECK(param->numel() == master.numel() && param->is_contiguous(), "param size");
  auto norms = at::zeros({nseg, 2}, master.options());
  const int64_t n = chunks.size(0);
  check(smpk::lamb_norms_chunked(master.data_ptr<float>(), update.data_ptr<float>(), chunks.data_ptr<int64_t>(), n,
                                 norms.data_ptr<float>(), stream()),
        "lamb_norms_chunked");
  check(smpk::lamb_stage2_chunked(param.has_value() ? dt_code(*param) : 0, param.has_value() ? param->data_ptr() : nullptr,
                                  master.data_ptr<float>(), update.data_ptr<float>(), chunks.data_ptr<int64_t>(), n,
                                  norms.data_ptr<float>(), static_cast<float>(lr), use_trust ? 1 : 0, stream()),
        "lamb_stage2_chunked");
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

at::Tensor add3(at::Tensor a, at::Tensor b, at::Tensor c) {
  check_gpu(a, "a");
  check_gpu(b, "b");
  check_gpu(c, "c");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && c.is_contiguous(), "add3: contiguous inputs required");
  TORCH_CHECK(a.sizes() == b.sizes() && a.sizes() == c.sizes(), "add3: shape mismatch");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.scalar_type() == c.scalar_type(), "add3: dtype mismatch");
  for (const at::Tensor* t : {&a, &b, &c})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "add3: 16-B aligned inputs required");
  auto out = at::empty_like(a, at::MemoryFormat::Contiguous);
  check(smpk::add3(dt_code(a), a.data_ptr(), b.data_ptr(), c.data_ptr(), out.data_ptr(), a.numel(), stream()), "add3");
  return out;
}

void cast_copy_(at::Tensor src, at::Tensor dst, double scale) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "cast_copy: size mismatch");
  check(smpk::cast_copy(dt_code(src), src.data_ptr(), dt_code(dst), dst.data_ptr(), src.numel(), scale, stream()),
        "cast_copy");
}

// ------------------------------------------------------------------- layernorm
smpk::DropoutArgs dropout_args(double p, int64_t seed, int64_t offset) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  smpk::DropoutArgs d;
  if (p > 0.0) {
    uint32_t thr = static_cast<uint32_t>(p * 65536.0 + 0.5);
    d.thr = thr < 1 ? 1 : (thr > 65535 ? 65535 : thr);
    d.rs = static_cast<float>(1.0 / (1.0 - p));
    d.seed = static_cast<uint64_t>(seed);
    d.offset = static_cast<uint64_t>(offset);
  }
  return d;
}

bool aligned16(const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// y = residual + dropout(x)
at::Tensor dropout_add(at::Tensor x, c10::optional<at::Tensor> residual, double p, int64_t seed, int64_t offset) {
  check_gpu(x, "x");
  TORCH_CHECK(aligned16(x), "dropout_add: x must be 16-byte aligned");
  if (residual.has_value()) {
    check_gpu(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type() && aligned16(*residual),
                "dropout_add: residual mismatch");
  }
  auto y = at::empty_like(x);
  check(smpk::dropout_add(dt_code(x), x.data_ptr(), opt_ptr(residual), y.data_ptr(), x.numel(),
                          dropout_args(p, seed, offset), stream()),
        "dropout_add");
  return y;
}

at::Tensor dropout_bwd(at::Tensor dy, double p, int64_t seed, int64_t offset) {
  check_gpu(dy, "dy");
  TORCH_CHECK(aligned16(dy), "dropout_bwd: dy must be 16-byte aligned");
  auto dx = at::empty_like(dy);
  check(smpk::dropout_bwd(dt_code(dy), dy.data_ptr(), dx.data_ptr(), dy.numel(), dropout_args(p, seed, offset),
                          stream()),
        "dropout_bwd");
  return dx;
}

std::vector<at::Tensor> layernorm_fwd(at::Tensor x, c10::optional<at::Tensor> residual,
                                      c10::optional<at::Tensor> w, c10::optional<at::Tensor> b, double eps,
                                      double dropout_p, int64_t seed, int64_t offset, bool mixed_output) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  // mixed_output: y in the affine parameters' dtype (MixedFusedLayerNorm)
  TORCH_CHECK(!mixed_output || w.has_value(), "mixed-dtype LayerNorm needs a weight");
  auto y = mixed_output ? at::empty(x.sizes(), x.options().dtype(w->scalar_type())) : at::empty_like(x);
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
                            rows, cols, eps, stream(), dropout_args(residual.has_value() ? dropout_p : 0.0, seed, offset),
                            mixed_output ? wdt : -1),
        "layernorm_fwd");
  if (residual.has_value()) return {y, mean, rstd, xo};
  return {y, mean, rstd};
}

// dw_out/db_out given (both): dgamma/dbeta accumulated into them in place (flat-buffer
// grad views) and returned; otherwise fresh tensors.
std::vector<at::Tensor> layernorm_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> w, at::Tensor mean,
                                      at::Tensor rstd, bool need_wgrad, bool need_bgrad,
                                      c10::optional<at::Tensor> dres, c10::optional<at::Tensor> dw_out,
                                      c10::optional<at::Tensor> db_out, c10::optional<at::Tensor> ext_sums,
                                      double ext_n, double dropout_p, int64_t seed, int64_t offset) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  auto dx = at::empty_like(x);
  // dropout_p > 0: also dxd = dropout backward of dx (the residual-branch dropout of a fused
  // add + LayerNorm) from the same kernel when the block kernels serve this width
  at::Tensor dxd;
  smpk::DropoutArgs drop = dropout_args(dropout_p, seed, offset);
  const bool aligned = ((reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(dy.data_ptr()) |
                         reinterpret_cast<uintptr_t>(dx.data_ptr()) |
                         (dres.has_value() ? reinterpret_cast<uintptr_t>(dres->data_ptr()) : 0) |
                         (w.has_value() ? reinterpret_cast<uintptr_t>(w->data_ptr()) : 0)) &
                        15) == 0;
  const int parts = smpk::layernorm_bwd_num_parts(dt_code(x), rows, cols, aligned);
  if (drop.thr != 0 && !ext_sums.has_value() && smpk::layernorm_bwd_dropout_fusable(dt_code(x), cols, aligned))
    dxd = at::empty_like(x);
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
                            stream(), ext_sums.has_value() ? ext_sums->data_ptr<float>() : nullptr,
                            static_cast<float>(ext_n), dxd.defined() ? dxd.data_ptr() : nullptr, &drop),
        "layernorm_bwd");
  if (dwp.defined()) {
    auto wo = w.has_value() ? w->options() : x.options();
    const bool acc = dw_out.has_value() && db_out.has_value();
    if (acc) {
      for (const at::Tensor* t : {&*dw_out, &*db_out})
        TORCH_CHECK(t->is_contiguous() && t->numel() == cols && dt_code(*t) == wdt,
                    "layernorm_bwd: dw_out/db_out must be contiguous [cols] tensors of the weight dtype");
      dw = *dw_out;
      db = *db_out;
    } else {
      dw = at::empty({cols}, wo);
      db = at::empty({cols}, wo);
    }
    auto work = at::empty({smpk::kLnReduceSlices, 2, cols}, x.options().dtype(at::kFloat));
    check(smpk::layernorm_bwd_reduce(wdt, dwp.data_ptr<float>(), dbp.data_ptr<float>(), dw.data_ptr(), db.data_ptr(),
                                     parts, cols, work.data_ptr<float>(), stream(), acc),
          "layernorm_bwd_reduce");
  }
  if (dxd.defined()) return {dx, dw, db, dxd};
  return {dx, dw, db};
}

// dst (view) <- src (view), same shape, <= 4 dims after the caller's collapsing, any strides
void strided_copy_(at::Tensor dst, at::Tensor src) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda() && dst.device() == src.device(), "strided_copy_: GPU tensors required");
  TORCH_CHECK(dst.sizes() == src.sizes() && dst.scalar_type() == src.scalar_type(), "strided_copy_: shape/dtype mismatch");
  TORCH_CHECK(dst.dim() <= 4, "strided_copy_: at most 4 dims (collapse first)");
  int64_t sz[4] = {1, 1, 1, 1}, ss[4] = {0, 0, 0, 0}, ds[4] = {0, 0, 0, 0};
  const int off = 4 - static_cast<int>(dst.dim());
  for (int i = 0; i < dst.dim(); ++i) {
    sz[off + i] = dst.size(i);
    ss[off + i] = src.stride(i);
    ds[off + i] = dst.stride(i);
  }
  check(smpk::strided_copy4(static_cast<int>(dst.element_size()), src.data_ptr(), dst.data_ptr(), sz, ss, ds, stream()),
        "strided_copy4");
}

at::Tensor layernorm_local_stats(at::Tensor x) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  auto out = at::empty({rows, 3}, x.options().dtype(at::kFloat));
  check(smpk::layernorm_local_stats(dt_code(x), x.data_ptr(), out.data_ptr<float>(), rows, cols, stream()),
        "layernorm_local_stats");
  return out;
}

at::Tensor layernorm_bwd_local_sums(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> w, at::Tensor mean,
                                    at::Tensor rstd) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd_local_sums: stats mismatch");
  auto out = at::empty({rows, 2}, x.options().dtype(at::kFloat));
  int wdt = w.has_value() ? dt_code(*w) : dt_code(x);
  check(smpk::layernorm_bwd_local_sums(dt_code(x), dy.data_ptr(), x.data_ptr(), wdt, opt_ptr(w),
                                       mean.data_ptr<float>(), rstd.data_ptr<float>(), out.data_ptr<float>(), rows,
                                       cols, stream()),
        "layernorm_bwd_local_sums");
  return out;
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
at::Tensor bias_gelu_fwd(at::Tensor x, c10::optional<at::Tensor> bias, bool exact) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  if (bias.has_value()) TORCH_CHECK(bias->numel() == cols && bias->scalar_type() == x.scalar_type(), "bias mismatch");
  auto y = at::empty_like(x);
  check(smpk::bias_gelu_fwd(dt_code(x), x.data_ptr(), opt_ptr(bias), y.data_ptr(), x.numel() / cols, cols, stream(),
                            exact),
        "bias_gelu_fwd");
  return y;
}

at::Tensor bias_gelu_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> bias, bool exact) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  auto dx = at::empty_like(x);
  check(smpk::bias_gelu_bwd(dt_code(x), dy.data_ptr(), x.data_ptr(), opt_ptr(bias), dx.data_ptr(), x.numel() / cols,
                            cols, stream(), exact),
        "bias_gelu_bwd");
  return dx;
}

// Weight gradient: c (+)= dy^T x with dy [tokens, n], x [tokens, k] (rows may be strided,
// elements contiguous), c contiguous [n, k] (bf16/f16/f32 -- the bound .grad view or an fp32
// main grad).  splits = 0: chosen for the device's CU count.
// dbias given (bf16 operands): dbias (+)= sum over tokens of dy from the same kernel pass
// (dbias_accumulate: add into it, else overwrite).
void wgrad_(at::Tensor c, at::Tensor dy, at::Tensor x, bool accumulate, int64_t splits,
            c10::optional<at::Tensor> dbias_opt, bool dbias_accumulate, int64_t impl) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && c.is_cuda(), "wgrad_: GPU tensors required");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && c.dim() == 2, "wgrad_: 2-D operands required");
  TORCH_CHECK(dy.size(0) == x.size(0), "wgrad_: token counts differ");
  TORCH_CHECK(c.size(0) == dy.size(1) && c.size(1) == x.size(1) && c.is_contiguous(), "wgrad_: c must be [n, k]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1, "wgrad_: operand rows must be contiguous");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "wgrad_: operand dtypes differ");
  const int64_t tokens = dy.size(0), n = dy.size(1), k = x.size(1);
  TORCH_CHECK(n % 8 == 0 && k % 8 == 0 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0,
              "wgrad_: n, k and row strides must be multiples of 8");
  TORCH_CHECK(n < (1LL << 31) && k < (1LL << 31), "wgrad_: dims too large");
  if (splits <= 0) {
    const int cus = at::cuda::getCurrentDeviceProperties()->multiProcessorCount;
    splits = smpk::wgrad_splits(tokens, static_cast<int>(n), static_cast<int>(k), cus);
  }
  // the kernel takes whole 64-token tiles; the remainder rows go through the library GEMM
  const int64_t main_t = tokens / 64 * 64, tail = tokens - main_t;
  at::Tensor dbias;
  if (dbias_opt.has_value() && dbias_opt->defined()) {
    dbias = *dbias_opt;
    TORCH_CHECK(dbias.is_cuda() && dbias.is_contiguous() && dbias.numel() == n, "wgrad_: dbias must be [n]");
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16, "wgrad_: fused bias gradient needs bf16 operands");
    TORCH_CHECK(dbias.scalar_type() == at::kBFloat16 || dbias.scalar_type() == at::kFloat,
                "wgrad_: dbias must be bf16 or fp32");
  }
  if (main_t == 0) {
    if (!accumulate) c.zero_();
    if (dbias.defined() && !dbias_accumulate) dbias.zero_();
  } else {
    const int64_t cs_rows = splits * ((k + 255) / 256);  // column-sum partials (wgrad.hip)
    auto ws = at::empty({splits * n * k + (dbias.defined() ? cs_rows * n : 0)}, dy.options().dtype(at::kFloat));
    float* cs = dbias.defined() ? ws.data_ptr<float>() + splits * n * k : nullptr;
    check(smpk::wgrad(dt_code(dy), dy.data_ptr(), x.data_ptr(), dt_code(c), c.data_ptr(), ws.data_ptr<float>(), main_t,
                      static_cast<int>(n), static_cast<int>(k), dy.stride(0), x.stride(0), static_cast<int>(splits),
                      accumulate ? 1 : 0, stream(), dbias.defined() ? dt_code(dbias) : 0,
                      dbias.defined() ? dbias.data_ptr() : nullptr, cs, dbias_accumulate ? 1 : 0,
                      static_cast<int>(impl)),
          "wgrad");
  }
  if (tail > 0) {
    // < 64 rows: fp32 (no bf16 rounding of the partial product)
    auto part = at::mm(dy.narrow(0, main_t, tail).to(at::kFloat).t(), x.narrow(0, main_t, tail).to(at::kFloat));
    c.add_(part.to(c.scalar_type()));
    if (dbias.defined()) dbias.add_(dy.narrow(0, main_t, tail).to(at::kFloat).sum(0).to(dbias.scalar_type()));
  }
}

int64_t wgrad_splits(int64_t tokens, int64_t n, int64_t k, int64_t cus) {
  return smpk::wgrad_splits(tokens, static_cast<int>(n), static_cast<int>(k), static_cast<int>(cus));
}

// out=None: fresh [cols] tensor; out given: out += colsum(x) in place (bias .grad views).
at::Tensor col_sum(at::Tensor x, c10::optional<at::Tensor> out_opt) {
  check_gpu(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  const int64_t parts = smpk::col_sum_parts(rows);
  auto ws = at::empty({parts + 32, cols}, x.options().dtype(at::kFloat));
  const bool acc = out_opt.has_value();
  at::Tensor out = acc ? *out_opt : at::empty({cols}, x.options());
  if (acc)
    TORCH_CHECK(out.is_contiguous() && out.numel() == cols && out.scalar_type() == x.scalar_type(),
                "col_sum: out must be a contiguous [cols] tensor of x's dtype");
  check(smpk::col_sum(dt_code(x), x.data_ptr(), out.data_ptr(), ws.data_ptr<float>(), rows, cols, stream(), acc),
        "col_sum");
  return out;
}

// (dx, dbias) of gelu(x + bias) in one pass; falls back to bwd + col_sum for odd shapes.
// dbias_out given: dbias accumulated into it in place (and returned).
std::vector<at::Tensor> bias_gelu_bwd_dbias(at::Tensor dy, at::Tensor x, at::Tensor bias,
                                            c10::optional<at::Tensor> dbias_out, bool exact) {
  check_gpu(dy, "dy");
  check_gpu(x, "x");
  check_gpu(bias, "bias");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  TORCH_CHECK(bias.numel() == cols && bias.scalar_type() == x.scalar_type(), "bias mismatch");
  auto dx = at::empty_like(x);
  const bool acc = dbias_out.has_value();
  at::Tensor db = acc ? *dbias_out : at::empty({cols}, x.options());
  if (acc)
    TORCH_CHECK(db.is_contiguous() && db.numel() == cols && db.scalar_type() == x.scalar_type(),
                "bias_gelu_bwd_dbias: dbias_out must be a contiguous [cols] tensor of x's dtype");
  const int64_t parts = smpk::gelu_dbias_parts(rows);
  auto ws = at::empty({parts + 32, cols}, x.options().dtype(at::kFloat));
  const int rc = smpk::bias_gelu_bwd_dbias(dt_code(x), dy.data_ptr(), x.data_ptr(), bias.data_ptr(), dx.data_ptr(),
                                           db.data_ptr(), ws.data_ptr<float>(), rows, cols, stream(), acc, exact);
  if (rc == -2) {
    dx = bias_gelu_bwd(dy, x, bias, exact);
    return {dx, col_sum(dx.view({rows, cols}), dbias_out)};
  }
  check(rc, "bias_gelu_bwd_dbias");
  return {dx, db};
}

// -------------------------------------------------------------------- transpose
// dst <- src^T for a contiguous 2-D src; dst must be a contiguous [cols, rows] tensor.
at::Tensor transpose_into(at::Tensor src, at::Tensor dst) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && src.is_contiguous() && dst.is_contiguous(), "transpose_into: contiguous 2-D tensors");
  TORCH_CHECK(dst.size(0) == src.size(1) && dst.size(1) == src.size(0) && dst.scalar_type() == src.scalar_type(),
              "transpose_into: dst must be [cols, rows] of src's dtype");
  check(smpk::transpose2d(dt_code(src), src.data_ptr(), dst.data_ptr(), src.size(0), src.size(1), stream()),
        "transpose2d");
  return dst;
}

// ------------------------------------------------------------------------ rope
static void rope_launch(at::Tensor x, at::Tensor y, at::Tensor cos_t, at::Tensor sin_t, int64_t rotary_dim, bool neox,
                        bool inverse, int64_t pos_offset, bool copy_rest) {
  TORCH_CHECK(x.is_cuda(), "x must be a GPU tensor");  // strided (b, s, h) views are fine
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "x must be [b, s, h, d] with contiguous d");
  TORCH_CHECK(y.is_cuda() && y.dim() == 4 && y.stride(3) == 1 && y.sizes() == x.sizes() &&
                  y.scalar_type() == x.scalar_type(), "y must be [b, s, h, d] like x, contiguous d");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat, "cos/sin tables must be fp32");
  TORCH_CHECK(cos_t.is_contiguous() && sin_t.is_contiguous(), "cos/sin tables must be contiguous");
  TORCH_CHECK(cos_t.size(0) >= x.size(1) + pos_offset && cos_t.size(1) == rotary_dim / 2, "cos/sin table shape");
  check(smpk::rope_apply(dt_code(x), x.data_ptr(), y.data_ptr(), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(),
                         x.size(0), x.size(1), x.size(2), x.size(3), rotary_dim, x.stride(0), x.stride(1), x.stride(2),
                         y.stride(0), y.stride(1), y.stride(2), neox ? 1 : 0, inverse ? 1 : 0, pos_offset,
                         copy_rest ? 1 : 0, stream()),
        "rope_apply");
}

at::Tensor rope_apply(at::Tensor x, at::Tensor cos_t, at::Tensor sin_t, int64_t rotary_dim, bool neox, bool inverse,
                      int64_t pos_offset) {
  auto y = at::empty({x.size(0), x.size(1), x.size(2), x.size(3)}, x.options());
  rope_launch(x, y, cos_t, sin_t, rotary_dim, neox, inverse, pos_offset, true);
  return y;
}

// y = rope(x) into a caller-given [b, s, h, d] view (e.g. the q / k slices of a packed QKV
// buffer); y may be x itself (in-place rotation, with copy_rest = false touching only the
// rotary channels)
void rope_apply_into(at::Tensor x, at::Tensor y, at::Tensor cos_t, at::Tensor sin_t, int64_t rotary_dim, bool neox,
                     bool inverse, int64_t pos_offset, bool copy_rest) {
  TORCH_CHECK(copy_rest || x.data_ptr() == y.data_ptr(), "copy_rest = false needs y to be x (in place)");
  rope_launch(x, y, cos_t, sin_t, rotary_dim, neox, inverse, pos_offset, copy_rest);
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
// vocab in (0, logits.size(1)): rows of stride logits.size(1) whose first `vocab` columns
// are valid (64-padded LM head); the backward then zero-fills the padding columns.
std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor target, int64_t vocab_start, int64_t ignore_index,
                                 int64_t vocab) {
  check_gpu(logits, "logits");
  check_gpu(target, "target");
  TORCH_CHECK(logits.dim() == 2 && target.dim() == 1 && target.size(0) == logits.size(0), "xent_fwd: shapes");
  TORCH_CHECK(logits.is_contiguous(), "xent_fwd: logits must be contiguous");
  TORCH_CHECK(target.scalar_type() == at::kLong, "target must be int64");
  const int64_t rows = logits.size(0), ld = logits.size(1);
  if (vocab <= 0) vocab = ld;
  TORCH_CHECK(vocab <= ld, "xent_fwd: vocab exceeds the row length");
  auto fo = logits.options().dtype(at::kFloat);
  auto mx = at::empty({rows}, fo), se = at::empty({rows}, fo), tl = at::empty({rows}, fo);
  check(smpk::xent_fwd_stats(dt_code(logits), logits.data_ptr(), target.data_ptr<int64_t>(), rows, vocab, vocab_start,
                             mx.data_ptr<float>(), se.data_ptr<float>(), tl.data_ptr<float>(), ignore_index, stream(),
                             ld),
        "xent_fwd");
  return {mx, se, tl};
}

at::Tensor xent_bwd(at::Tensor logits, at::Tensor target, at::Tensor lse, at::Tensor grad_rows, int64_t vocab_start,
                    int64_t ignore_index, int64_t vocab) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "xent_bwd: logits must be a contiguous 2-D tensor");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && grad_rows.scalar_type() == at::kFloat, "lse/grad must be fp32");
  TORCH_CHECK(grad_rows.is_contiguous() && lse.is_contiguous(), "lse/grad contiguous");
  const int64_t ld = logits.size(1);
  if (vocab <= 0) vocab = ld;
  TORCH_CHECK(vocab <= ld, "xent_bwd: vocab exceeds the row length");
  auto d = at::empty_like(logits);
  check(smpk::xent_bwd(dt_code(logits), logits.data_ptr(), target.data_ptr<int64_t>(), lse.data_ptr<float>(),
                       grad_rows.data_ptr<float>(), d.data_ptr(), logits.size(0), vocab, vocab_start, ignore_index,
                       stream(), ld),
        "xent_bwd");
  return d;
}

// ------------------------------------------------------------------- attention
// q, k, v: [b, s, h, d] with the last dim contiguous (other strides arbitrary, e.g. views
// of a fused [b, s, 3, h, d] QKV projection).
void check_bshd(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.stride(3) == 1, n, " must be a GPU [b, s, h, d] tensor with contiguous d");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, n, " must be bf16/fp16");
}

void set_dropout(smpk::AttnParams& p, double dropout_p, int64_t seed, int64_t offset);

smpk::AttnParams attn_params(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale, bool causal,
                             int64_t window, const c10::optional<at::Tensor>& kbias,
                             double dropout_p, int64_t seed,
                             int64_t offset) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(2) == k.size(2) && q.size(3) == k.size(3),
              "attention: q/k/v shape mismatch");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "attention: dtype mismatch");
  TORCH_CHECK(smpk::attention_head_dim_supported(q.size(3)), "attention kernel supports head_dim 64, 96, 128, 256");
  for (const at::Tensor* t : {&q, &k, &v})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0 && t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                    t->stride(0) % 8 == 0,
                "attention: operands must be 16-byte aligned");
  TORCH_CHECK(q.size(1) < (1 << 24) && k.size(1) < (1 << 24), "attention: sequence too long");
  smpk::AttnParams p{};
  p.q = q.data_ptr();
  p.k = k.data_ptr();
  p.v = v.data_ptr();
  p.b = q.size(0);
  p.sq = q.size(1);
  p.h = q.size(2);
  p.d = q.size(3);
  p.sk = k.size(1);
  p.q_sb = q.stride(0), p.q_ss = q.stride(1), p.q_sh = q.stride(2);
  p.k_sb = k.stride(0), p.k_ss = k.stride(1), p.k_sh = k.stride(2);
  p.v_sb = v.stride(0), p.v_ss = v.stride(1), p.v_sh = v.stride(2);
  p.scale = static_cast<float>(scale);
  p.causal = causal ? 1 : 0;
  p.window = static_cast<int>(window);
  if (kbias.has_value() && kbias->defined()) {
    const at::Tensor& kb = *kbias;
    TORCH_CHECK(kb.is_cuda() && kb.scalar_type() == at::kFloat && kb.dim() == 2 && kb.stride(1) == 1 &&
                    kb.size(1) == p.sk && (kb.size(0) == p.b || kb.size(0) == 1),
                "attention: key bias must be a float32 [b or 1, sk] GPU tensor with contiguous rows");
    p.kbias = kb.data_ptr<float>();
    p.kbias_sb = kb.size(0) == 1 ? 0 : kb.stride(0);
  }
  set_dropout(p, dropout_p, seed, offset);
  return p;
}

// dropout fields of the attention parameters (the keep-bits kernel needs only these and the
// sizes)
void set_dropout(smpk::AttnParams& p, double dropout_p, int64_t seed, int64_t offset) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "attention: dropout_p must be in [0, 1)");
  if (dropout_p > 0.0) {
    // dropped iff the element's 8-bit uniform < thr, where each 32x32 block draws thr from
    // {lo, lo + 1} with P(lo + 1) = frac / 65536 (attention_impl.h drop_block_thr): the drop
    // probability of every element is (lo + frac / 65536) / 256 = dropout_p to 2^-24, and kept
    // values are scaled by 1 / (1 - dropout_p)
    const double x = dropout_p * 256.0;
    uint32_t lo = static_cast<uint32_t>(x);
    uint32_t frac = static_cast<uint32_t>((x - lo) * 65536.0 + 0.5);
    if (frac >= 65536u) lo += 1, frac = 0;
    const double p_eff = (lo + frac / 65536.0) / 256.0;
    auto consts = [](uint32_t thr, uint32_t& xr, uint32_t& c) {
      const uint32_t t7 = thr <= 128 ? thr : 256 - thr;  // 0..128
      xr = thr <= 128 ? 0u : 0xffffffffu;
      c = (128u - t7) * 0x01010101u;
    };
    p.drop_on = 1;
    p.drop_thr = lo;
    p.drop_frac = frac;
    p.drop_rs = static_cast<float>(1.0 / (1.0 - p_eff));
    consts(lo, p.drop_xr, p.drop_c);
    consts(lo + 1, p.drop_xr1, p.drop_c1);
    p.seed = static_cast<uint64_t>(seed);
    p.offset = static_cast<uint64_t>(offset);
  }
}

std::vector<at::Tensor> attention_fwd(at::Tensor q, at::Tensor k, at::Tensor v, double scale, bool causal,
                                      int64_t window, c10::optional<at::Tensor> kbias,
                                      double dropout_p, int64_t seed,
                                      int64_t offset, bool store_bits, c10::optional<at::Tensor> bits_in) {
  auto p = attn_params(q, k, v, scale, causal, window, kbias, dropout_p, seed, offset);
  auto o = at::empty({p.b, p.sq, p.h, p.d}, q.options());
  auto lse = at::empty({p.b, p.h, p.sq}, q.options().dtype(at::kFloat));
  p.o = o.data_ptr();
  p.o_sb = o.stride(0), p.o_ss = o.stride(1), p.o_sh = o.stride(2);
  p.lse = lse.data_ptr<float>();
  // dropout: the keep bits (1 bit per score: b h sq sk / 8 bytes) are generated first by the
  // keep-bits kernel and read by the forward (no hash in the MFMA loop); kept for the backward
  // when store_bits, else dropped here and regenerated before the backward
  // (bits_in: the same words, generated earlier by attention_keep_bits_for on a side stream)
  at::Tensor bits;
  if (p.drop_on && bits_in.has_value() && bits_in->defined()) {
    bits = *bits_in;
    TORCH_CHECK(bits.is_cuda() && bits.scalar_type() == at::kInt && bits.is_contiguous() &&
                    bits.numel() == p.b * p.h * ((p.sk + 63) / 64) * p.sq * 2,
                "attention_fwd: bits_in must be the int32 [b h, ceil(sk / 64), sq, 2] keep bits");
    p.drop_bits = reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>());
  } else if (p.drop_on) {
    bits = at::empty({p.b * p.h, (p.sk + 63) / 64, p.sq, 2}, q.options().dtype(at::kInt));
    p.drop_bits = reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>());
    check(smpk::attention_keep_bits(p, p.drop_bits, stream()), "attention_keep_bits");
  }
  check(smpk::attention_fwd(dt_code(q), p, stream()), "attention_fwd");
  if (!p.drop_on || !store_bits) bits = at::empty({0}, q.options().dtype(at::kInt));
  return {o, lse, bits};
}

// The keep bits a dropout forward with these arguments stores, regenerated from the hash (for a
// forward called with store_bits = false).
// The keep bits of a (b, h, sq, sk) attention from the sizes alone, on the current stream (the
// caller's side stream: launched before the QKV projection, the hash runs beside that GEMM)
at::Tensor attention_keep_bits_for(int64_t b, int64_t h, int64_t sq, int64_t sk, bool causal, double dropout_p,
                                   int64_t seed, int64_t offset, at::Tensor like) {
  TORCH_CHECK(dropout_p > 0.0, "attention_keep_bits_for: dropout_p must be > 0");
  TORCH_CHECK(like.is_cuda(), "attention_keep_bits_for: like must be a GPU tensor");
  TORCH_CHECK(b >= 0 && h >= 0 && sq >= 0 && sk >= 0 && sq < (1 << 24) && sk < (1 << 24), "attention_keep_bits_for: sizes");
  smpk::AttnParams p{};
  p.b = b, p.h = h, p.sq = sq, p.sk = sk;
  p.causal = causal ? 1 : 0;
  set_dropout(p, dropout_p, seed, offset);
  auto bits = at::empty({b * h, (sk + 63) / 64, sq, 2}, like.options().dtype(at::kInt));
  check(smpk::attention_keep_bits(p, reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>()), stream()),
        "attention_keep_bits");
  return bits;
}

at::Tensor attention_keep_bits(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, int64_t window,
                               double dropout_p, int64_t seed, int64_t offset) {
  TORCH_CHECK(dropout_p > 0.0, "attention_keep_bits: dropout_p must be > 0");
  auto p = attn_params(q, k, v, 1.0, causal, window, c10::nullopt, dropout_p, seed, offset);
  auto bits = at::empty({p.b * p.h, (p.sk + 63) / 64, p.sq, 2}, q.options().dtype(at::kInt));
  check(smpk::attention_keep_bits(p, reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>()), stream()),
        "attention_keep_bits");
  return bits;
}

// Writes into the provided dq/dk/dv (may be views of one packed gradient buffer).
void attention_bwd_into(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                        at::Tensor dq, at::Tensor dk, at::Tensor dv, double scale, bool causal, int64_t window,
                        c10::optional<at::Tensor> kbias, double dropout_p,
                        int64_t seed, int64_t offset, c10::optional<at::Tensor> drop_bits) {
  smpk::AttnBwdParams P{};
  P.f = attn_params(q, k, v, scale, causal, window, kbias, dropout_p, seed, offset);
  if (P.f.drop_on) {
    TORCH_CHECK(drop_bits.has_value() && drop_bits->defined(), "attention_bwd: dropout needs the forward's keep bits");
    const at::Tensor& bt = *drop_bits;
    TORCH_CHECK(bt.is_cuda() && bt.scalar_type() == at::kInt && bt.is_contiguous() &&
                    bt.numel() == P.f.b * P.f.h * ((P.f.sk + 63) / 64) * P.f.sq * 2,
                "attention_bwd: keep bits must be the forward's int32 [b h, ceil(sk / 64), sq, 2] tensor");
    P.f.drop_bits = reinterpret_cast<uint32_t*>(bt.data_ptr<int32_t>());
  }
  check_bshd(dout, "dout");
  check_bshd(o, "o");
  check_bshd(dq, "dq");
  check_bshd(dk, "dk");
  check_bshd(dv, "dv");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes() &&
                  dk.sizes() == k.sizes() && dv.sizes() == v.sizes(),
              "attention_bwd: shape mismatch");
  P.f.o = o.data_ptr();
  P.f.o_sb = o.stride(0), P.f.o_ss = o.stride(1), P.f.o_sh = o.stride(2);
  P.f.lse = lse.data_ptr<float>();
  P.dout = dout.data_ptr();
  P.do_sb = dout.stride(0), P.do_ss = dout.stride(1), P.do_sh = dout.stride(2);
  P.dq = dq.data_ptr();
  P.dk = dk.data_ptr();
  P.dv = dv.data_ptr();
  P.dq_sb = dq.stride(0), P.dq_ss = dq.stride(1), P.dq_sh = dq.stride(2);
  P.dk_sb = dk.stride(0), P.dk_ss = dk.stride(1), P.dk_sh = dk.stride(2);
  P.dv_sb = dv.stride(0), P.dv_ss = dv.stride(1), P.dv_sh = dv.stride(2);
  auto delta = at::empty({P.f.b, P.f.h, P.f.sq}, q.options().dtype(at::kFloat));
  P.delta = delta.data_ptr<float>();
  check(smpk::attention_bwd(dt_code(q), P, stream()), "attention_bwd");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "smdistributed_modelparallel_amd CDNA4 (gfx950) kernels + torch-aware runtime";
  smprt_torch::register_bindings(m);
  m.def("fused_adam", &fused_adam);
  m.def("fused_sgd", &fused_sgd);
  m.def("fused_adagrad", &fused_adagrad);
  m.def("mt_adam", &mt_adam);
  m.def("mt_norm", &mt_norm);
  m.def("mt_lamb1", &mt_lamb1);
  m.def("mt_lamb2", &mt_lamb2);
  m.def("mt_novograd", &mt_novograd);
  m.def("novograd_blend", &novograd_blend);
  m.def("lamb_stage1", &lamb_stage1);
  m.def("lamb_stage2", &lamb_stage2);
  m.def("lamb_chunked_", &lamb_chunked);
  m.def("sumsq_", &sumsq_);
  m.def("nonfinite_", &nonfinite_);
  m.def("axpby_", &axpby_);
  m.def("cast_copy_", &cast_copy_);
  m.def("layernorm_fwd", &layernorm_fwd, py::arg("x"), py::arg("residual"), py::arg("w"), py::arg("b"),
        py::arg("eps"), py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0,
        py::arg("mixed_output") = false);
  m.def("dropout_add", &dropout_add, py::arg("x"), py::arg("residual"), py::arg("p"), py::arg("seed"),
        py::arg("offset"));
  m.def("dropout_bwd", &dropout_bwd, py::arg("dy"), py::arg("p"), py::arg("seed"), py::arg("offset"));
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"), py::arg("rstd"),
        py::arg("need_wgrad"), py::arg("need_bgrad"), py::arg("dres"), py::arg("dw_out") = py::none(),
        py::arg("db_out") = py::none(), py::arg("ext_sums") = py::none(), py::arg("ext_n") = 0.0,
        py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0);
  m.def("layernorm_local_stats", &layernorm_local_stats);
  m.def("strided_copy_", &strided_copy_);
  m.def("add3", &add3);
  m.def("layernorm_bwd_local_sums", &layernorm_bwd_local_sums);
  m.def("layernorm_apply_stats", &layernorm_apply_stats);
  m.def("bias_gelu_fwd", &bias_gelu_fwd, py::arg("x"), py::arg("bias"), py::arg("exact") = false);
  m.def("bias_gelu_bwd", &bias_gelu_bwd, py::arg("dy"), py::arg("x"), py::arg("bias"), py::arg("exact") = false);
  m.def("transpose_into", &transpose_into);
  m.def("col_sum", &col_sum, py::arg("x"), py::arg("out") = py::none());
  m.def("wgrad_", &wgrad_, py::arg("c"), py::arg("dy"), py::arg("x"), py::arg("accumulate") = true,
        py::arg("splits") = 0, py::arg("dbias") = py::none(), py::arg("dbias_accumulate") = true,
        py::arg("impl") = -1);
  m.def("wgrad_splits", &wgrad_splits);
  m.def("rope_apply", &rope_apply);
  m.def("rope_apply_into", &rope_apply_into, py::arg("x"), py::arg("y"), py::arg("cos"), py::arg("sin"),
        py::arg("rotary_dim"), py::arg("neox"), py::arg("inverse"), py::arg("pos_offset"), py::arg("copy_rest") = true);
  m.def("bias_gelu_bwd_dbias", &bias_gelu_bwd_dbias, py::arg("dy"), py::arg("x"), py::arg("bias"),
        py::arg("dbias_out") = py::none(), py::arg("exact") = false);
  m.def("scaled_masked_softmax_fwd", &scaled_masked_softmax_fwd);
  m.def("scaled_upper_triang_softmax_fwd", &scaled_upper_triang_softmax_fwd);
  m.def("scaled_softmax_bwd", &scaled_softmax_bwd);
  m.def("xent_fwd", &xent_fwd, py::arg("logits"), py::arg("target"), py::arg("vocab_start"),
        py::arg("ignore_index"), py::arg("vocab") = -1);
  m.def("xent_bwd", &xent_bwd, py::arg("logits"), py::arg("target"), py::arg("lse"), py::arg("grad_rows"),
        py::arg("vocab_start"), py::arg("ignore_index"), py::arg("vocab") = -1);
  m.def("attention_fwd", &attention_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("scale"),
        py::arg("causal"), py::arg("window"), py::arg("kbias") = py::none(),
        py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0, py::arg("store_bits") = true,
        py::arg("bits_in") = py::none());
  m.def("attention_keep_bits_for", &attention_keep_bits_for, py::arg("b"), py::arg("h"), py::arg("sq"), py::arg("sk"),
        py::arg("causal"), py::arg("dropout_p"), py::arg("seed"), py::arg("offset"), py::arg("like"));
  m.def("attention_keep_bits", &attention_keep_bits, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"),
        py::arg("window"), py::arg("dropout_p"), py::arg("seed"), py::arg("offset"));
  m.def("attention_bwd_into", &attention_bwd_into, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("o"), py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("scale"),
        py::arg("causal"), py::arg("window"), py::arg("kbias") = py::none(),
        py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0, py::arg("drop_bits") = py::none());
}
