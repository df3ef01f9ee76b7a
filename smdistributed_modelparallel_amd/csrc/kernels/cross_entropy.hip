// Vocab-parallel cross entropy (K19 of SURVEY §2.6; reference
// `smp/torch/nn/cross_entropy.py:28-112`, which materialises fp32 softmax copies).
//
// Forward: one 256-thread block per row streams the (local-shard) logits ONCE in
// low precision and keeps an online (max, sum-exp) pair per thread in fp32, merged by a
// block reduction; it also picks the target logit if the target falls in this shard.
// The caller combines shards (max all-reduce, rescaled sum-exp all-reduce).
// Backward: dlogits = (exp(x - lse) - onehot(target)) * g_row, written in the logits
// dtype in one pass -- no fp32 [tokens, vocab] tensor is ever materialised.
// Rows of an odd vocabulary are not 16-byte aligned, so each row is split into a scalar
// head, a 16-byte-vector body and a scalar tail.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

struct MaxSum {
  float m, s;
};

__device__ __forceinline__ MaxSum merge(MaxSum a, MaxSum b) {
  if (a.m == -INFINITY) return b;
  if (b.m == -INFINITY) return a;
  const float m = fmaxf(a.m, b.m);
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}

__device__ __forceinline__ void add(MaxSum& a, float x) {
  if (x > a.m) {
    a.s = a.s * __expf(a.m - x) + 1.f;
    a.m = x;
  } else {
    a.s += __expf(x - a.m);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       int64_t vocab, int64_t vstart, float* __restrict__ rmax,
                                                       float* __restrict__ rsum, float* __restrict__ rtgt,
                                                       int64_t ignore, int64_t ld) {
  constexpr int N = Vec16<T>::N;
  __shared__ float sm[8], ss[8];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  MaxSum acc{-INFINITY, 0.f};
  // head until 16-byte aligned
  const int64_t mis = (reinterpret_cast<uintptr_t>(x) & 15) / sizeof(T);
  const int64_t head = mis ? ((N - mis) < vocab ? (N - mis) : vocab) : 0;
  for (int64_t c = threadIdx.x; c < head; c += 256) add(acc, to_f32(x[c]));
  const int64_t nvec = (vocab - head) / N;
  const T* xb = x + head;
  for (int64_t v = threadIdx.x; v < nvec; v += 256) {
    Vec16<T> a = load16(xb + v * N);
#pragma unroll
    for (int j = 0; j < N; ++j) add(acc, to_f32(a.v[j]));
  }
  for (int64_t c = head + nvec * N + threadIdx.x; c < vocab; c += 256) add(acc, to_f32(x[c]));
  // wave reduce
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MaxSum other{__shfl_xor(acc.m, o, 64), __shfl_xor(acc.s, o, 64)};
    acc = merge(acc, other);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = acc.m;
    ss[wid] = acc.s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MaxSum r{sm[0], ss[0]};
    for (int w = 1; w < 4; ++w) r = merge(r, MaxSum{sm[w], ss[w]});
    rmax[row] = r.m;
    rsum[row] = r.s;
    const int64_t t = tgt[row];
    float tl = 0.f;
    if (t != ignore && t >= vstart && t < vstart + vocab) tl = to_f32(x[t - vstart]);
    rtgt[row] = tl;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse, const float* __restrict__ g,
                                                       T* __restrict__ dl, int64_t vocab, int64_t vstart,
                                                       int64_t ignore, int64_t ld) {
  constexpr int N = Vec16<T>::N;
  const int64_t row = blockIdx.x;
  const int64_t t = tgt[row];
  const float gr = (t == ignore) ? 0.f : g[row];
  const float l = lse[row];
  const int64_t tl = t - vstart;  // local target column (may be out of range)
  const T* x = logits + row * ld;
  T* d = dl + row * ld;
  // padding columns of a row stride ld > vocab (64-padded LM head): zero gradient
  for (int64_t c = vocab + threadIdx.x; c < ld; c += 256) d[c] = from_f32<T>(0.f);
  const int64_t mis = (reinterpret_cast<uintptr_t>(x) & 15) / sizeof(T);
  const bool same_align = ((reinterpret_cast<uintptr_t>(x) ^ reinterpret_cast<uintptr_t>(d)) & 15) == 0;
  auto one = [&](int64_t c) {
    const float p = __expf(to_f32(x[c]) - l);
    d[c] = from_f32<T>((p - (c == tl ? 1.f : 0.f)) * gr);
  };
  if (!same_align) {
    for (int64_t c = threadIdx.x; c < vocab; c += 256) one(c);
    return;
  }
  const int64_t head = mis ? ((N - mis) < vocab ? (N - mis) : vocab) : 0;
  for (int64_t c = threadIdx.x; c < head; c += 256) one(c);
  const int64_t nvec = (vocab - head) / N;
  for (int64_t v = threadIdx.x; v < nvec; v += 256) {
    const int64_t c0 = head + v * N;
    Vec16<T> a = load16(x + c0);
    Vec16<T> o;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float p = __expf(to_f32(a.v[j]) - l);
      o.v[j] = from_f32<T>((p - (c0 + j == tl ? 1.f : 0.f)) * gr);
    }
    store16(d + c0, o);
  }
  for (int64_t c = head + nvec * N + threadIdx.x; c < vocab; c += 256) one(c);
}

}  // namespace

// ld: row stride in elements (>= vocab; 0 = vocab).  Rows beyond `vocab` are padding that
// the forward ignores and the backward zero-fills (64-padded LM head, ops/lm_head.py).
int xent_fwd_stats(int dt, const void* logits, const int64_t* target, int64_t rows, int64_t vocab, int64_t vocab_start,
                   float* row_max, float* row_sumexp, float* row_target_logit, int64_t ignore_index, hipStream_t s,
                   int64_t ld) {
  if (rows <= 0) return 0;
  if (ld < vocab) ld = vocab;
  SMPK_DISPATCH(dt, T, {
    xent_fwd_kernel<T><<<static_cast<unsigned>(rows), 256, 0, s>>>(static_cast<const T*>(logits), target, vocab,
                                                                   vocab_start, row_max, row_sumexp,
                                                                   row_target_logit, ignore_index, ld);
  });
  return static_cast<int>(hipGetLastError());
}

int xent_bwd(int dt, const void* logits, const int64_t* target, const float* row_lse, const float* grad_rows,
             void* dlogits, int64_t rows, int64_t vocab, int64_t vocab_start, int64_t ignore_index, hipStream_t s,
             int64_t ld) {
  if (rows <= 0) return 0;
  if (ld < vocab) ld = vocab;
  SMPK_DISPATCH(dt, T, {
    xent_bwd_kernel<T><<<static_cast<unsigned>(rows), 256, 0, s>>>(static_cast<const T*>(logits), target, row_lse,
                                                                   grad_rows, static_cast<T*>(dlogits), vocab,
                                                                   vocab_start, ignore_index, ld);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
