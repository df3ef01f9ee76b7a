// Fused optimizer kernels over contiguous flat ranges (K12-K16, K20 in SURVEY §2.6).
//
// Memory-bound: Adam on bf16 params / bf16 grads / fp32 master+m+v moves 28 B per
// element.  Each thread handles 4 consecutive elements (16-B fp32 vectors, 8-B bf16
// vectors); the grid is capped at 256 CUs x 8 blocks and grid-strides the rest
// (Guideline 11).  Math is fp32; the low-precision param copy is written in the same
// pass so no separate master->model cast kernel is needed.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 4;

inline int grid_for(int64_t n) {
  int64_t blocks = (n / kVec + kThreads - 1) / kThreads;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  return static_cast<int>(blocks);
}

template <typename T>
struct Vec4 {
  T v[4];
};

template <typename T>
__device__ __forceinline__ void load4(const T* p, int64_t i, int64_t n, float (&out)[4]) {
  if (i + 4 <= n && (reinterpret_cast<uintptr_t>(p + i) % (4 * sizeof(T)) == 0)) {
    Vec4<T> r = *reinterpret_cast<const Vec4<T>*>(p + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = to_f32(r.v[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = (i + j < n) ? to_f32(p[i + j]) : 0.f;
  }
}

template <typename T>
__device__ __forceinline__ void store4(T* p, int64_t i, int64_t n, const float (&in)[4]) {
  if (i + 4 <= n && (reinterpret_cast<uintptr_t>(p + i) % (4 * sizeof(T)) == 0)) {
    Vec4<T> r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.v[j] = from_f32<T>(in[j]);
    *reinterpret_cast<Vec4<T>*>(p + i) = r;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < n) p[i + j] = from_f32<T>(in[j]);
  }
}

template <typename P, typename G, bool HAS_P>
__global__ void __launch_bounds__(kThreads) adam_kernel(P* __restrict__ param, const G* __restrict__ grad,
                                                        float* __restrict__ master, float* __restrict__ m,
                                                        float* __restrict__ v, int64_t n, float lr, float b1,
                                                        float b2, float eps, float wd, float bc1, float bc2,
                                                        float gscale, int adamw) {
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float g[4], p[4], mm[4], vv[4];
    load4(grad, i, n, g);
    load4(master, i, n, p);
    load4(m, i, n, mm);
    load4(v, i, n, vv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * gscale;
      if (adamw) {
        p[j] -= lr * wd * p[j];
      } else {
        gj += wd * p[j];
      }
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      const float denom = sqrtf(vv[j]) * inv_sqrt_bc2 + eps;
      p[j] -= step_size * mm[j] / denom;
    }
    store4(master, i, n, p);
    store4(m, i, n, mm);
    store4(v, i, n, vv);
    if (HAS_P) store4(param, i, n, p);
  }
}

template <typename P, typename G, bool HAS_P>
__global__ void __launch_bounds__(kThreads) sgd_kernel(P* __restrict__ param, const G* __restrict__ grad,
                                                       float* __restrict__ master, float* __restrict__ mom,
                                                       int64_t n, float lr, float momentum, float damp, float wd,
                                                       int nesterov, int first, float gscale) {
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float g[4], p[4], b[4];
    load4(grad, i, n, g);
    load4(master, i, n, p);
    if (momentum != 0.f) load4(mom, i, n, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * gscale + wd * p[j];
      if (momentum != 0.f) {
        b[j] = first ? gj : momentum * b[j] + (1.f - damp) * gj;
        gj = nesterov ? gj + momentum * b[j] : b[j];
      }
      p[j] -= lr * gj;
    }
    store4(master, i, n, p);
    if (momentum != 0.f) store4(mom, i, n, b);
    if (HAS_P) store4(param, i, n, p);
  }
}

template <typename P, typename G, bool HAS_P>
__global__ void __launch_bounds__(kThreads) adagrad_kernel(P* __restrict__ param, const G* __restrict__ grad,
                                                           float* __restrict__ master, float* __restrict__ sum,
                                                           int64_t n, float lr, float eps, float wd, float gscale) {
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float g[4], p[4], h[4];
    load4(grad, i, n, g);
    load4(master, i, n, p);
    load4(sum, i, n, h);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * gscale + wd * p[j];
      h[j] += gj * gj;
      p[j] -= lr * gj / (sqrtf(h[j]) + eps);
    }
    store4(master, i, n, p);
    store4(sum, i, n, h);
    if (HAS_P) store4(param, i, n, p);
  }
}

template <typename G>
__global__ void __launch_bounds__(kThreads) lamb1_kernel(const G* __restrict__ grad, const float* __restrict__ master,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         float* __restrict__ upd, int64_t n, float b1, float b2,
                                                         float eps, float wd, float bc1, float bc2, float gscale) {
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float g[4], p[4], mm[4], vv[4], u[4];
    load4(grad, i, n, g);
    load4(master, i, n, p);
    load4(m, i, n, mm);
    load4(v, i, n, vv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * gscale;
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      u[j] = (mm[j] / bc1) / (sqrtf(vv[j] / bc2) + eps) + wd * p[j];
    }
    store4(m, i, n, mm);
    store4(v, i, n, vv);
    store4(upd, i, n, u);
  }
}

template <typename P, bool HAS_P>
__global__ void __launch_bounds__(kThreads) lamb2_kernel(P* __restrict__ param, float* __restrict__ master,
                                                         const float* __restrict__ upd, int64_t n, float lr,
                                                         const float* pn, const float* un, int use_trust) {
  float trust = 1.f;
  if (use_trust) {
    const float a = sqrtf(*pn), b = sqrtf(*un);
    trust = (a > 0.f && b > 0.f) ? a / b : 1.f;
  }
  const float s = lr * trust;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float p[4], u[4];
    load4(master, i, n, p);
    load4(upd, i, n, u);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] -= s * u[j];
    store4(master, i, n, p);
    if (HAS_P) store4(param, i, n, p);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) sumsq_kernel(const T* __restrict__ x, int64_t n, float scale,
                                                         float* __restrict__ out) {
  __shared__ float smem[16];
  float acc = 0.f;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float a[4];
    load4(x, i, n, a);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += a[j] * a[j];
  }
  acc = block_sum(acc, smem);
  if (threadIdx.x == 0) atomicAdd(out, acc * scale * scale);
}

template <typename T>
__global__ void __launch_bounds__(kThreads) nonfinite_kernel(const T* __restrict__ x, int64_t n,
                                                             float* __restrict__ out) {
  int bad = 0;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float a[4];
    load4(x, i, n, a);
#pragma unroll
    for (int j = 0; j < 4; ++j) bad |= !isfinite(a[j]);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<int*>(out), 0x3f800000);  // 1.0f
}

template <typename T>
__global__ void __launch_bounds__(kThreads) axpby_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                         float a, float b) {
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float xv[4], yv[4];
    load4(x, i, n, xv);
    load4(y, i, n, yv);
#pragma unroll
    for (int j = 0; j < 4; ++j) yv[j] = a * xv[j] + b * yv[j];
    store4(y, i, n, yv);
  }
}

template <typename S, typename D>
__global__ void __launch_bounds__(kThreads) cast_kernel(const S* __restrict__ x, D* __restrict__ y, int64_t n,
                                                        float scale) {
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec; i < n;
       i += static_cast<int64_t>(gridDim.x) * kThreads * kVec) {
    float v[4];
    load4(x, i, n, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= scale;
    store4(y, i, n, v);
  }
}

// ---- LAMB over a whole domain in two launches (no per-parameter host loop) ----------------
// chunks [nchunks][3] = (segment, start, end): element ranges of <= kLambChunk elements, each
// inside one parameter's piece; a block per chunk.
template <typename P>
__device__ __forceinline__ void lamb_chunk(const int64_t* chunks, int64_t& seg, int64_t& s, int64_t& e) {
  const int64_t* c = chunks + 3 * static_cast<int64_t>(blockIdx.x);
  seg = c[0];
  s = c[1];
  e = c[2];
}

__global__ void __launch_bounds__(kThreads) lamb_norms_kernel(const float* __restrict__ master,
                                                              const float* __restrict__ upd,
                                                              const int64_t* __restrict__ chunks,
                                                              float* __restrict__ norms) {
  __shared__ float smem[16];
  int64_t seg, s, e;
  lamb_chunk<float>(chunks, seg, s, e);
  float a = 0.f, b = 0.f;
  for (int64_t i = s + threadIdx.x; i < e; i += kThreads) {
    const float p = master[i], u = upd[i];
    a += p * p;
    b += u * u;
  }
  a = block_sum(a, smem);
  __syncthreads();
  b = block_sum(b, smem);
  if (threadIdx.x == 0) {
    atomicAdd(norms + 2 * seg, a);
    atomicAdd(norms + 2 * seg + 1, b);
  }
}

template <typename P, bool HAS_P>
__global__ void __launch_bounds__(kThreads) lamb2_chunked_kernel(P* __restrict__ param, float* __restrict__ master,
                                                                 const float* __restrict__ upd,
                                                                 const int64_t* __restrict__ chunks,
                                                                 const float* __restrict__ norms, float lr,
                                                                 int use_trust) {
  int64_t seg, s, e;
  lamb_chunk<P>(chunks, seg, s, e);
  float trust = 1.f;
  if (use_trust) {
    const float a = sqrtf(norms[2 * seg]), b = sqrtf(norms[2 * seg + 1]);
    trust = (a > 0.f && b > 0.f) ? a / b : 1.f;
  }
  const float st = lr * trust;
  for (int64_t i = s + threadIdx.x; i < e; i += kThreads) {
    const float p = master[i] - st * upd[i];
    master[i] = p;
    if (HAS_P) param[i] = from_f32<P>(p);
  }
}

}  // namespace

int lamb_norms_chunked(const float* master, const float* update, const int64_t* chunks, int64_t nchunks,
                       float* norms, hipStream_t s) {
  if (nchunks <= 0) return 0;
  lamb_norms_kernel<<<static_cast<unsigned>(nchunks), kThreads, 0, s>>>(master, update, chunks, norms);
  return static_cast<int>(hipGetLastError());
}

int lamb_stage2_chunked(int param_dt, void* param, float* master, const float* update, const int64_t* chunks,
                        int64_t nchunks, const float* norms, float lr, int use_trust, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  if (param == nullptr) {
    lamb2_chunked_kernel<float, false><<<grid, kThreads, 0, s>>>(nullptr, master, update, chunks, norms, lr,
                                                                 use_trust);
  } else {
    SMPK_DISPATCH(param_dt, P, {
      lamb2_chunked_kernel<P, true><<<grid, kThreads, 0, s>>>(static_cast<P*>(param), master, update, chunks, norms,
                                                              lr, use_trust);
    });
  }
  return static_cast<int>(hipGetLastError());
}

int fused_adam(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* exp_avg,
               float* exp_avg_sq, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
               float bias_c1, float bias_c2, float grad_scale, int adamw_mode, hipStream_t s) {
  if (n <= 0) return 0;
  const int grid = grid_for(n);
  SMPK_DISPATCH(grad_dt, G, {
    if (param == nullptr) {
      adam_kernel<float, G, false><<<grid, kThreads, 0, s>>>(nullptr, static_cast<const G*>(grad), master, exp_avg,
                                                            exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay,
                                                            bias_c1, bias_c2, grad_scale, adamw_mode);
    } else {
      SMPK_DISPATCH(param_dt, P, {
        adam_kernel<P, G, true><<<grid, kThreads, 0, s>>>(static_cast<P*>(param), static_cast<const G*>(grad),
                                                          master, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps,
                                                          weight_decay, bias_c1, bias_c2, grad_scale, adamw_mode);
      });
    }
  });
  return static_cast<int>(hipGetLastError());
}

int fused_sgd(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* mom, int64_t n,
              float lr, float momentum, float dampening, float weight_decay, int nesterov, int first_run,
              float grad_scale, hipStream_t s) {
  if (n <= 0) return 0;
  const int grid = grid_for(n);
  SMPK_DISPATCH(grad_dt, G, {
    if (param == nullptr) {
      sgd_kernel<float, G, false><<<grid, kThreads, 0, s>>>(nullptr, static_cast<const G*>(grad), master, mom, n, lr,
                                                           momentum, dampening, weight_decay, nesterov, first_run,
                                                           grad_scale);
    } else {
      SMPK_DISPATCH(param_dt, P, {
        sgd_kernel<P, G, true><<<grid, kThreads, 0, s>>>(static_cast<P*>(param), static_cast<const G*>(grad), master,
                                                         mom, n, lr, momentum, dampening, weight_decay, nesterov,
                                                         first_run, grad_scale);
      });
    }
  });
  return static_cast<int>(hipGetLastError());
}

int fused_adagrad(int param_dt, void* param, int grad_dt, const void* grad, float* master, float* sum, int64_t n,
                  float lr, float eps, float weight_decay, float grad_scale, hipStream_t s) {
  if (n <= 0) return 0;
  const int grid = grid_for(n);
  SMPK_DISPATCH(grad_dt, G, {
    if (param == nullptr) {
      adagrad_kernel<float, G, false><<<grid, kThreads, 0, s>>>(nullptr, static_cast<const G*>(grad), master, sum, n,
                                                               lr, eps, weight_decay, grad_scale);
    } else {
      SMPK_DISPATCH(param_dt, P, {
        adagrad_kernel<P, G, true><<<grid, kThreads, 0, s>>>(static_cast<P*>(param), static_cast<const G*>(grad),
                                                             master, sum, n, lr, eps, weight_decay, grad_scale);
      });
    }
  });
  return static_cast<int>(hipGetLastError());
}

int lamb_stage1(int grad_dt, const void* grad, const float* master, float* exp_avg, float* exp_avg_sq, float* update,
                int64_t n, float beta1, float beta2, float eps, float weight_decay, float bias_c1, float bias_c2,
                float grad_scale, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(grad_dt, G, {
    lamb1_kernel<G><<<grid_for(n), kThreads, 0, s>>>(static_cast<const G*>(grad), master, exp_avg, exp_avg_sq,
                                                     update, n, beta1, beta2, eps, weight_decay, bias_c1, bias_c2,
                                                     grad_scale);
  });
  return static_cast<int>(hipGetLastError());
}

int lamb_stage2(int param_dt, void* param, float* master, const float* update, int64_t n, float lr,
                const float* p_norm_sq, const float* u_norm_sq, int use_trust, hipStream_t s) {
  if (n <= 0) return 0;
  if (param == nullptr) {
    lamb2_kernel<float, false><<<grid_for(n), kThreads, 0, s>>>(nullptr, master, update, n, lr, p_norm_sq, u_norm_sq,
                                                                use_trust);
  } else {
    SMPK_DISPATCH(param_dt, P, {
      lamb2_kernel<P, true><<<grid_for(n), kThreads, 0, s>>>(static_cast<P*>(param), master, update, n, lr,
                                                             p_norm_sq, u_norm_sq, use_trust);
    });
  }
  return static_cast<int>(hipGetLastError());
}

int sumsq(int dt, const void* x, int64_t n, float scale, float* out, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, { sumsq_kernel<T><<<grid_for(n), kThreads, 0, s>>>(static_cast<const T*>(x), n, scale, out); });
  return static_cast<int>(hipGetLastError());
}

int nonfinite(int dt, const void* x, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, { nonfinite_kernel<T><<<grid_for(n), kThreads, 0, s>>>(static_cast<const T*>(x), n, out); });
  return static_cast<int>(hipGetLastError());
}

int axpby(int dt, const void* x, void* y, int64_t n, float a, float b, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    axpby_kernel<T><<<grid_for(n), kThreads, 0, s>>>(static_cast<const T*>(x), static_cast<T*>(y), n, a, b);
  });
  return static_cast<int>(hipGetLastError());
}

int cast_copy(int dt_src, const void* src, int dt_dst, void* dst, int64_t n, float scale, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt_src, S, {
    SMPK_DISPATCH(dt_dst, D, {
      cast_kernel<S, D><<<grid_for(n), kThreads, 0, s>>>(static_cast<const S*>(src), static_cast<D*>(dst), n, scale);
    });
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
