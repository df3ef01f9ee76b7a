// Host-side launcher API of the gfx950 kernels.  Pure C++ (no torch types) so the
// kernels are reusable and their translation units compile quickly; the torch binding
// layer (bindings.cpp) validates tensors and forwards raw pointers + the current stream.
// Every launcher returns 0 on success or a hipError_t / negative code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smpk {

enum DType : int { F32 = 0, F16 = 1, BF16 = 2 };

// ---------------------------------------------------------------- optimizers (optim.hip)
// Fused Adam/AdamW over one contiguous range. param may be null (master is the param).
int fused_adam(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* exp_avg,
               float* exp_avg_sq, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
               float bias_c1, float bias_c2, float grad_scale, int adamw_mode, hipStream_t s);
int fused_sgd(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* mom, int64_t n,
              float lr, float momentum, float dampening, float weight_decay, int nesterov, int first_run,
              float grad_scale, hipStream_t s);
int fused_adagrad(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* sum, int64_t n,
                  float lr, float eps, float weight_decay, float grad_scale, hipStream_t s);
// LAMB stage 1: update = adam_direction + wd * p  (written into `update`), m/v updated.
int lamb_stage1(int grad_dt, const void* grad, const float* master, float* exp_avg, float* exp_avg_sq,
                float* update, int64_t n, float beta1, float beta2, float eps, float weight_decay, float bias_c1,
                float bias_c2, float grad_scale, hipStream_t s);
// LAMB stage 2: p -= lr * trust * update, trust from per-range norms (device scalars).
int lamb_stage2(int param_dt, void* param, float* master, const float* update, int64_t n, float lr,
                const float* p_norm_sq, const float* u_norm_sq, int use_trust, hipStream_t s);
// LAMB over a domain with per-parameter trust ratios in two launches: chunks [nchunks][3] =
// (segment, start, end) element ranges (<= 64K elements, each inside one segment = one
// parameter's piece); norms [nsegments][2] fp32 (zeroed by the caller) receive
// (|p|^2, |update|^2) per segment; stage 2 applies p -= lr * trust(segment) * update.
int lamb_norms_chunked(const float* master, const float* update, const int64_t* chunks, int64_t nchunks,
                       float* norms, hipStream_t s);
int lamb_stage2_chunked(int param_dt, void* param, float* master, const float* update, const int64_t* chunks,
                        int64_t nchunks, const float* norms, float lr, int use_trust, hipStream_t s);
// sum of squares of x (any dtype) * scale^2 accumulated into *out (fp32, atomic).
int sumsq(int dt, const void* x, int64_t n, float scale, float* out, hipStream_t s);
// multi-tensor apply over tensor lists (optim.hip: meta = role pointer table + chunk table)
int mt_adam(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master, float lr,
            float b1, float b2, float eps, float wd, float bc1, float bc2, float gscale, int adamw, hipStream_t s);
int mt_norm(const int64_t* meta, int64_t nt, int64_t nchunks, int role, int dt, float scale, int maxabs, float* out,
            hipStream_t s);
int mt_lamb1(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master, float b1,
             float b2, float b3, float bc1, float bc2, float eps, float wd, int decoupled, const float* gnorm,
             float max_gnorm, float gscale, hipStream_t s);
int mt_lamb2(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int master, const float* pn2,
             const float* un2, float lr, int use_trust, hipStream_t s);
int mt_novograd(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master,
                const float* norms, float b1, float b3, float bc1, float bc2, float eps, float lr, float wd,
                int decoupled, float gscale, hipStream_t s);
int novograd_blend(float* norms, const float* fresh, int64_t nt, float b2, int l2, int first, int init_zero,
                   hipStream_t s);
// *out = max(*out, 1 if any element non-finite).
int nonfinite(int dt, const void* x, int64_t n, float* out, hipStream_t s);
// y = a * x + b * y (elementwise, same dtype) ; y may equal x.
int axpby(int dt, const void* x, void* y, int64_t n, float a, float b, hipStream_t s);
int add3(int dt, const void* a, const void* b, const void* c, void* out, int64_t n, hipStream_t s);
// copy with cast: dst(dt_dst) = src(dt_src) * scale
int cast_copy(int dt_src, const void* src, int dt_dst, void* dst, int64_t n, float scale, hipStream_t s);

// ------------------------------------------------------------------ norms (layernorm.hip)
// y = (x - mean) * rstd * w + b ; optional residual add: x = x + r written to x_out first.
// Element-wise dropout decided by a counter hash of (seed, offset, element index): no mask
// tensor is stored, the backward regenerates the decisions.  thr = 0 disables dropout.
struct DropoutArgs {
  uint32_t thr = 0;  // element dropped iff its 16-bit uniform < thr
  float rs = 1.f;    // 1 / (1 - p)
  uint64_t seed = 0, offset = 0;
};
// y = residual + dropout(x)  (residual may be null); x, residual, y same dtype, contiguous
int dropout_add(int dt, const void* x, const void* residual, void* y, int64_t n, const DropoutArgs& d, hipStream_t s);
// dx = dy * keep * rs  (the backward of dropout)
int dropout_bwd(int dt, const void* dy, void* dx, int64_t n, const DropoutArgs& d, hipStream_t s);

// residual != null: x_out = residual + dropout(x) is written and normalised (pre-LN block)
int layernorm_fwd(int dt, const void* x, const void* residual, void* x_out, int wdt, const void* w, const void* b,
                  void* y, float* mean, float* rstd, int64_t rows, int64_t cols, float eps, hipStream_t s,
                  const DropoutArgs& drop = DropoutArgs(), int out_dt = -1);
// out_dt: -1 = y in the input dtype; the parameter dtype = mixed-dtype LayerNorm (K10, apex
// MixedFusedLayerNorm: output takes the affine parameters' dtype).
int layernorm_bwd(int dt, const void* dy, const void* x, int wdt, const void* w, const float* mean,
                  const float* rstd, void* dx, float* dw_part, float* db_part, int64_t rows, int64_t cols,
                  int part_rows, const void* dres, hipStream_t s,
                  const float* ext_sums = nullptr, float ext_n = 0.f, void* dxd = nullptr,
                  const DropoutArgs* drop = nullptr);
// dxd (the dropout branch's gradient dx * keep / (1 - p), one pass with dx) is available for
// these widths / alignment (the block-per-rows backward kernels)
bool layernorm_bwd_dropout_fusable(int dt, int64_t cols, bool aligned);
// dgamma/dbeta from the per-block partials; work = [kLnReduceSlices][2][cols] fp32 scratch.
constexpr int kLnReduceSlices = 32;
int layernorm_bwd_reduce(int wdt, const float* dw_part, const float* db_part, void* dw, void* db, int parts,
                         int64_t cols, float* work, hipStream_t s, bool accumulate = false);
// Distributed-LN pieces (hidden sharded across TP): apply with global stats, local sums.
int layernorm_apply_stats(int dt, const void* x, int wdt, const void* w, const void* b, const float* mean,
                          const float* var, void* y, float* rstd, int64_t rows, int64_t cols, float eps, hipStream_t s);
// Distributed LayerNorm over a TP-sharded hidden dim (K6-K8; reference
// smp/torch/nn/layer_norm.py:24-102):
//  * layernorm_local_stats: per row of the local shard (n*m, M2, n*m*m) with m the local
//    mean and M2 = sum (x - m)^2 -- summed over the TP group they give the exact global
//    mean and variance (Chan's parallel combination, no E[x^2] - E[x]^2 cancellation);
//  * layernorm_apply_stats (K6): y from the global mean / var;
//  * layernorm_bwd_local_sums (K7): per row (sum dy*w, sum dy*w*xhat) over the local shard;
//  * layernorm_bwd with ext_sums (K8): dx from the TP-summed row sums over ext_n columns,
//    plus this shard's dgamma / dbeta partials.
int layernorm_local_stats(int dt, const void* x, float* stats3, int64_t rows, int64_t cols, hipStream_t s);
int layernorm_bwd_local_sums(int dt, const void* dy, const void* x, int wdt, const void* w, const float* mean,
                             const float* rstd, float* sums2, int64_t rows, int64_t cols, hipStream_t s);
int layernorm_bwd_num_parts(int dt, int64_t rows, int64_t cols, bool aligned);

// ------------------------------------------------------------- elementwise (gelu.hip)
// y = gelu_tanh(x + bias) ; bias broadcast over the last dim (may be null).
// exact: erf GeLU (F.gelu) instead of the tanh approximation.
int bias_gelu_fwd(int dt, const void* x, const void* bias, void* y, int64_t rows, int64_t cols, hipStream_t s,
                  bool exact = false);
// dx = dy * gelu'(x + bias) ; dbias partial sums per row-chunk (fp32) when dbias_part != null.
int bias_gelu_bwd(int dt, const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int64_t cols,
                  hipStream_t s, bool exact = false);
// Column sums of a [rows, cols] matrix into fp32 partials then final (for bias grads).
// accumulate: out += colsum(x) (bias gradients bound into the flat grad buffer).
int col_sum(int dt, const void* x, void* out, float* workspace, int64_t rows, int64_t cols, hipStream_t s,
            bool accumulate = false);
int col_sum_parts(int64_t rows);
int gelu_dbias_parts(int64_t rows);  // workspace partial rows for bias_gelu_bwd_dbias
int bias_gelu_bwd_dbias(int dt, const void* dy, const void* x, const void* bias, void* dx, void* dbias,
                        float* workspace, int64_t rows, int64_t cols, hipStream_t s, bool accumulate = false,
                        bool exact = false);

// ------------------------------------------------------------- transpose (transpose.hip)
// dst[cols][rows] = src[rows][cols] (row-major, contiguous).
int transpose2d(int dt, const void* src, void* dst, int64_t rows, int64_t cols, hipStream_t s);

// --------------------------------------------------------------- softmax (softmax.hip)
int scaled_masked_softmax_fwd(int dt, const void* x, const uint8_t* mask, void* y, int64_t batch, int64_t heads,
                              int64_t sq, int64_t sk, int64_t mask_batch, float scale, hipStream_t s);
int scaled_upper_triang_softmax_fwd(int dt, const void* x, void* y, int64_t attn_batches, int64_t sq, int64_t sk,
                                    float scale, hipStream_t s);
int scaled_softmax_bwd(int dt, const void* dy, const void* y, void* dx, int64_t rows, int64_t cols, float scale,
                       hipStream_t s);

// ------------------------------------------------------------------------ rope (rope.hip)
// y = rope(x): x and y [b, s, h, d] with their own (b, s, h) strides and contiguous d (y may
// alias x); rotary_dim channels rotate (the rest are copied unless copy_rest = 0), style 0 = GPT-J (interleaved pairs), 1 = NeoX (half
// rotation), inverse = rotate by -theta (backward).  cos/sin tables [positions, rotary_dim/2] fp32.
int rope_apply(int dt, const void* x, void* y, const float* cos_t, const float* sin_t, int64_t b, int64_t s_len,
               int64_t h, int64_t d, int64_t rotary_dim, int64_t stride_b, int64_t stride_s, int64_t stride_h,
               int64_t y_b, int64_t y_s, int64_t y_h, int style, int inverse, int64_t pos_offset, int copy_rest,
               hipStream_t s);

// -------------------------------------------------------------- attention (attention.hip)
// Flash-style attention, bf16/fp16 in, fp32 softmax stats. q,k,v,o: [b, h, s, d] with
// explicit strides (elements); lse: [b, h, sq] fp32.
struct AttnParams {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  int64_t b, h, sq, sk, d;
  int64_t q_sb, q_sh, q_ss;
  int64_t k_sb, k_sh, k_ss;
  int64_t v_sb, v_sh, v_ss;
  int64_t o_sb, o_sh, o_ss;
  float scale;
  int causal;
  int window;  // >0: local attention window (GPT-Neo)
  const float* kbias;  // optional additive key bias [b, sk] (padding mask); nullptr = none
  int64_t kbias_sb;    // its batch stride (0: one row shared by the batch)
  uint32_t drop_on;    // dropout enabled
  uint32_t drop_thr;   // element dropped iff its 8-bit uniform < thr, thr = drop_thr or drop_thr + 1
  uint32_t drop_frac;  //   per 32x32 block, thr = drop_thr + 1 with probability drop_frac / 65536
  float drop_rs;       // 1 / keep probability = 1 / (1 - dropout_p)
  uint32_t drop_xr;    // per-byte keep test constants for thr = drop_thr (attention_impl.h keep_flags):
  uint32_t drop_c;     //   xr = 0 / ~0 for thr <= / > 128, c = per-byte add constant
  uint32_t drop_xr1;   // ... and for thr = drop_thr + 1
  uint32_t drop_c1;
  // keep bits [b * h][ceil(sk / 64)][sq][2] (one uint32 per (row, 64-key tile, half-wave)):
  // written by the forward, read by dQ / dK-dV (attention_impl.h drop_bit layout)
  uint32_t* drop_bits;
  uint64_t seed, offset;
};
struct AttnBwdParams {
  AttnParams f;
  const void* dout;
  int64_t do_sb, do_sh, do_ss;
  void* dq;
  void* dk;
  void* dv;
  int64_t dq_sb, dq_sh, dq_ss;
  int64_t dk_sb, dk_sh, dk_ss;
  int64_t dv_sb, dv_sh, dv_ss;
  float* delta;  // [b, h, sq] workspace
};
int attention_fwd(int dt, const AttnParams& p, hipStream_t s);
// the dropout keep bits from the hash into `bits` ([b h, ceil(sk / 64), sq, 2] uint32): before
// every dropout forward (which reads them), and before a backward whose forward kept none
int attention_keep_bits(const AttnParams& p, uint32_t* bits, hipStream_t s);
bool attention_head_dim_supported(int64_t d);
int attention_bwd(int dt, const AttnBwdParams& p, hipStream_t s);

// ------------------------------------------------------- cross entropy (cross_entropy.hip)
// Per-row: lse over [vocab_start, vocab_end) local shard; returns local max / sumexp /
// target logit (target may be outside the shard -> 0). Fused fwd writes softmax stats;
// bwd writes dlogits = (softmax - onehot) * grad.
int xent_fwd_stats(int dt, const void* logits, const int64_t* target, int64_t rows, int64_t vocab, int64_t vocab_start,
                   float* row_max, float* row_sumexp, float* row_target_logit, int64_t ignore_index, hipStream_t s,
                   int64_t ld = 0);
int xent_bwd(int dt, const void* logits, const int64_t* target, const float* row_lse, const float* grad_rows,
             void* dlogits, int64_t rows, int64_t vocab, int64_t vocab_start, int64_t ignore_index, hipStream_t s,
             int64_t ld = 0);

// ------------------------------------------------------------ weight gradient (wgrad.hip)
// C[n][k] (+)= sum_t A[t][n] B[t][k]  (A = dY [tokens, n], B = X [tokens, k], row-major with
// row strides lda / ldb; C contiguous [n, k] of c_dt).  Split-K over tokens into the fp32
// workspace ws [splits][n][k], then reduced into C.  n, k, lda, ldb multiples of 8.
int wgrad_splits(int64_t tokens, int n, int k, int num_cus);
// bias != nullptr (bf16 operands): bias (+)= sum over tokens of A, computed by the same kernel
// from its staged A tiles (cs: [splits * ceil(k / 256)][n] fp32 workspace, wgrad.hip).
// impl: 1 = ping-pong kernel, 0 = one-barrier-per-tile kernel, -1 = SMP_WGRAD_IMPL / default.
int wgrad(int dt, const void* a, const void* b, int c_dt, void* c, float* ws, int64_t tokens, int n, int k,
          int64_t lda, int64_t ldb, int splits, int accumulate, hipStream_t s, int bias_dt = 0, void* bias = nullptr,
          float* cs = nullptr, int bias_accumulate = 1, int impl = -1);

// ---------------------------------------------------------------- pack / unpack (pack.hip)
// Generic strided 4-D copy: dst[i0,i1,i2,i3] = src[...] with element strides (for the
// split/merge-axis all-to-all and allgatherv packing).
int strided_copy4(int elem_bytes, const void* src, void* dst, const int64_t* sizes, const int64_t* src_strides,
                  const int64_t* dst_strides, hipStream_t s);
// Flat byte copy by a kernel on `s` (16-byte vectors when both ends are 16-byte aligned): the
// pipeline's IPC pulls use it instead of hipMemcpyAsync, so a pull is an ordinary compute-queue
// kernel of the pull stream (no copy-engine queue shared with the process's other streams).
int device_copy(void* dst, const void* src, int64_t nbytes, hipStream_t s);

}  // namespace smpk
