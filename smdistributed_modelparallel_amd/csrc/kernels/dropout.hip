// Fused dropout for the transformer's residual branches (reference: `F.dropout` after the
// attention / MLP output and on the embeddings, `smp/torch/nn/transformer.py:1143,1524`,
// `:449`): y = residual + dropout(x) in one pass, decisions from the element-index hash
// (common.h), so no mask tensor is written in the forward nor read in the backward.
// Forward: 2 reads + 1 write (torch: dropout 1 read + 2 writes, then add 2 reads + 1 write).
// Backward of the x branch: dx = dy * keep * rs, 1 read + 1 write.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

template <typename T>
__global__ void __launch_bounds__(256) dropout_add_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                          T* __restrict__ y, int64_t n, DropoutArgs d) {
  constexpr int N = Vec16<T>::N;
  const uint32_t key = dropout_key(d);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * N;
  for (int64_t e = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * N; e < n; e += stride) {
    if (e + N <= n) {
      Vec16<T> a = load16(x + e);
      float f[8];
      if constexpr (N == 8) {
        dropout_factors8(key, e, d, f);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) f[j] = dropout_factor1(key, e + j, d);
      }
      if (r != nullptr) {
        Vec16<T> b = load16(r + e);
#pragma unroll
        for (int j = 0; j < N; ++j) a.v[j] = from_f32<T>(fmaf(to_f32(a.v[j]), f[j], to_f32(b.v[j])));
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) a.v[j] = from_f32<T>(to_f32(a.v[j]) * f[j]);
      }
      store16(y + e, a);
    } else {
      for (int64_t i = e; i < n; ++i) {
        const float f = dropout_factor1(key, i, d);
        y[i] = from_f32<T>(to_f32(x[i]) * f + (r != nullptr ? to_f32(r[i]) : 0.f));
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int64_t n,
                                                          DropoutArgs d) {
  constexpr int N = Vec16<T>::N;
  const uint32_t key = dropout_key(d);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * N;
  for (int64_t e = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * N; e < n; e += stride) {
    if (e + N <= n) {
      Vec16<T> a = load16(dy + e);
      float f[8];
      if constexpr (N == 8) {
        dropout_factors8(key, e, d, f);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) f[j] = dropout_factor1(key, e + j, d);
      }
#pragma unroll
      for (int j = 0; j < N; ++j) a.v[j] = from_f32<T>(to_f32(a.v[j]) * f[j]);
      store16(dx + e, a);
    } else {
      for (int64_t i = e; i < n; ++i) dx[i] = from_f32<T>(to_f32(dy[i]) * dropout_factor1(key, i, d));
    }
  }
}

int grid_for(int64_t n, int per_thread) {
  const int64_t blocks = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  return static_cast<int>(blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks));  // grid-stride beyond 8192
}

}  // namespace

int dropout_add(int dt, const void* x, const void* residual, void* y, int64_t n, const DropoutArgs& d, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    dropout_add_kernel<T><<<grid_for(n, Vec16<T>::N), 256, 0, s>>>(
        static_cast<const T*>(x), static_cast<const T*>(residual), static_cast<T*>(y), n, d);
  });
  return static_cast<int>(hipGetLastError());
}

int dropout_bwd(int dt, const void* dy, void* dx, int64_t n, const DropoutArgs& d, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    dropout_bwd_kernel<T><<<grid_for(n, Vec16<T>::N), 256, 0, s>>>(static_cast<const T*>(dy), static_cast<T*>(dx), n,
                                                                    d);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
