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

// out = a + b + c (the parallel-attention residual sum hidden + attn + mlp in one pass):
// 16 B per operand per lane (8 bf16 / f16, 4 fp32) -- all four pointers 16-B aligned, checked
// by the caller -- and a scalar tail
template <typename T>
__global__ void __launch_bounds__(kThreads) add3_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                        const T* __restrict__ c, T* __restrict__ out, int64_t n) {
  constexpr int V = 16 / sizeof(T);
  struct alignas(16) Pack {
    T v[V];
  };
  const int64_t nv = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < nv; i += stride) {
    const Pack x = reinterpret_cast<const Pack*>(a)[i];
    const Pack y = reinterpret_cast<const Pack*>(b)[i];
    const Pack z = reinterpret_cast<const Pack*>(c)[i];
    Pack o;
#pragma unroll
    for (int j = 0; j < V; ++j) o.v[j] = from_f32<T>((to_f32(x.v[j]) + to_f32(y.v[j])) + to_f32(z.v[j]));
    reinterpret_cast<Pack*>(out)[i] = o;
  }
  for (int64_t i = nv * V + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride)
    out[i] = from_f32<T>((to_f32(a[i]) + to_f32(b[i])) + to_f32(c[i]));
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

// ---- multi-tensor apply (amp_C multi_tensor_* equivalents, N4 / K12-K16) ------------------
// One launch updates a whole LIST of separately allocated tensors (the standalone FusedAdam /
// FusedLAMB / FusedNovoGrad path; the DistributedOptimizer path runs on flat buffers instead).
// meta (int64, device): kRoles x nt tensor pointers (role-major; 0 = absent) followed by
// nchunks x 3 (tensor, start, end) element ranges of <= 65536 elements; one block per chunk.
// Roles: 0 grad (G), 1 param (P), 2 fp32 master (MASTER) -- without it P is fp32 and is its own
// master --, 3 first moment, 4 second moment, 5 fp32 update scratch (LAMB).
constexpr int kRoles = 6;

struct MTChunk {
  int t;
  int64_t s, e;
};

__device__ __forceinline__ MTChunk mt_chunk(const int64_t* meta, int64_t nt) {
  const int64_t* c = meta + kRoles * nt + 3 * static_cast<int64_t>(blockIdx.x);
  return MTChunk{static_cast<int>(c[0]), c[1], c[2]};
}

template <typename T>
__device__ __forceinline__ T* mt_ptr(const int64_t* meta, int64_t nt, int role, int t) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(meta[role * nt + t]));
}

// elements [s, e) of one chunk, 4 per thread per step (chunk bases are 4-aligned; load4 /
// store4 fall back to scalar accesses at a tensor's tail or an unaligned base)
#define SMPK_MT_LOOP(i) for (int64_t i = ch.s + threadIdx.x * kVec; i < ch.e; i += kThreads * kVec)

template <typename P, typename G, bool MASTER>
__global__ void __launch_bounds__(kThreads) mt_adam_kernel(const int64_t* __restrict__ meta, int64_t nt, float lr,
                                                           float b1, float b2, float eps, float wd, float bc1,
                                                           float bc2, float gscale, int adamw) {
  const MTChunk ch = mt_chunk(meta, nt);
  const G* g = mt_ptr<const G>(meta, nt, 0, ch.t);
  P* prm = mt_ptr<P>(meta, nt, 1, ch.t);
  float* mst = MASTER ? mt_ptr<float>(meta, nt, 2, ch.t) : reinterpret_cast<float*>(prm);
  float* m = mt_ptr<float>(meta, nt, 3, ch.t);
  float* v = mt_ptr<float>(meta, nt, 4, ch.t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  SMPK_MT_LOOP(i) {
    float gg[4], p[4], mm[4], vv[4];
    load4(g, i, ch.e, gg);
    load4(mst, i, ch.e, p);
    load4(m, i, ch.e, mm);
    load4(v, i, ch.e, vv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * gscale;
      if (adamw) {
        p[j] -= lr * wd * p[j];
      } else {
        gj += wd * p[j];
      }
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      p[j] -= step_size * mm[j] / (sqrtf(vv[j]) * inv_sqrt_bc2 + eps);
    }
    store4(mst, i, ch.e, p);
    store4(m, i, ch.e, mm);
    store4(v, i, ch.e, vv);
    if (MASTER) store4(prm, i, ch.e, p);
  }
}

// per-tensor sum of squares (MAXABS: max |x|) of role `role`, accumulated into out[t]
template <typename T, bool MAXABS>
__global__ void __launch_bounds__(kThreads) mt_norm_kernel(const int64_t* __restrict__ meta, int64_t nt, int role,
                                                           float scale, float* __restrict__ out) {
  __shared__ float smem[16];
  const MTChunk ch = mt_chunk(meta, nt);
  const T* x = mt_ptr<const T>(meta, nt, role, ch.t);
  float a = 0.f;
  SMPK_MT_LOOP(i) {
    float xv[4];
    load4(x, i, ch.e, xv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float y = xv[j] * scale;
      a = MAXABS ? fmaxf(a, fabsf(y)) : fmaf(y, y, a);
    }
  }
  a = MAXABS ? block_max(a, smem) : block_sum(a, smem);
  if (threadIdx.x == 0) {
    if (MAXABS) {
      atomicMax(reinterpret_cast<int*>(out + ch.t), __float_as_int(a));  // a >= 0: int order = float order
    } else {
      atomicAdd(out + ch.t, a);
    }
  }
}

// LAMB stage 1 (apex LAMBStage1Functor): update = m_hat / (sqrt(v_hat) + eps) [+ wd * p], with
// the gradient divided by the clipped global gradient norm; the update goes to the scratch role
template <typename P, typename G, bool MASTER>
__global__ void __launch_bounds__(kThreads) mt_lamb1_kernel(const int64_t* __restrict__ meta, int64_t nt, float b1,
                                                            float b2, float b3, float bc1, float bc2, float eps,
                                                            float wd, int decoupled, const float* __restrict__ gnorm,
                                                            float max_gnorm, float gscale) {
  const MTChunk ch = mt_chunk(meta, nt);
  const G* g = mt_ptr<const G>(meta, nt, 0, ch.t);
  const float* mst = MASTER ? mt_ptr<const float>(meta, nt, 2, ch.t) : mt_ptr<const float>(meta, nt, 1, ch.t);
  float* m = mt_ptr<float>(meta, nt, 3, ch.t);
  float* v = mt_ptr<float>(meta, nt, 4, ch.t);
  float* u = mt_ptr<float>(meta, nt, 5, ch.t);
  const float gn = *gnorm;
  const float clip = (max_gnorm > 0.f && gn > max_gnorm) ? gn / max_gnorm : 1.f;
  const float gmul = gscale / clip;
  SMPK_MT_LOOP(i) {
    float gg[4], p[4], mm[4], vv[4], uu[4];
    load4(g, i, ch.e, gg);
    load4(mst, i, ch.e, p);
    load4(m, i, ch.e, mm);
    load4(v, i, ch.e, vv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sg = gg[j] * gmul;
      if (!decoupled) sg += wd * p[j];
      mm[j] = mm[j] * b1 + b3 * sg;
      vv[j] = vv[j] * b2 + (1.f - b2) * sg * sg;
      uu[j] = (mm[j] / bc1) / (sqrtf(vv[j] / bc2) + eps);
      if (decoupled) uu[j] += wd * p[j];
    }
    store4(m, i, ch.e, mm);
    store4(v, i, ch.e, vv);
    store4(u, i, ch.e, uu);
  }
}

// LAMB stage 2 (apex LAMBStage2Functor): p -= lr * trust * update, trust = ||p|| / ||u|| per
// tensor (when use_nvlamb or weight decay is on)
template <typename P, bool MASTER>
__global__ void __launch_bounds__(kThreads) mt_lamb2_kernel(const int64_t* __restrict__ meta, int64_t nt,
                                                            const float* __restrict__ pn2,
                                                            const float* __restrict__ un2, float lr, int use_trust) {
  const MTChunk ch = mt_chunk(meta, nt);
  P* prm = mt_ptr<P>(meta, nt, 1, ch.t);
  float* mst = MASTER ? mt_ptr<float>(meta, nt, 2, ch.t) : reinterpret_cast<float*>(prm);
  const float* u = mt_ptr<const float>(meta, nt, 5, ch.t);
  float ratio = lr;
  if (use_trust) {
    const float a = sqrtf(pn2[ch.t]), b = sqrtf(un2[ch.t]);
    ratio = (a != 0.f && b != 0.f) ? lr * (a / b) : lr;
  }
  SMPK_MT_LOOP(i) {
    float p[4], uu[4];
    load4(mst, i, ch.e, p);
    load4(u, i, ch.e, uu);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] -= ratio * uu[j];
    store4(mst, i, ch.e, p);
    if (MASTER) store4(prm, i, ch.e, p);
  }
}

// NovoGrad (apex NovoGradFunctor): per-tensor second moment = blended gradient NORM (not its
// square); moment mode 0 = regularisation inside the moment, 1 = decoupled weight decay
template <typename P, typename G, bool MASTER>
__global__ void __launch_bounds__(kThreads) mt_novograd_kernel(const int64_t* __restrict__ meta, int64_t nt,
                                                               const float* __restrict__ norms, float b1, float b3,
                                                               float bc1, float bc2, float eps, float lr, float wd,
                                                               int decoupled, float gscale) {
  const MTChunk ch = mt_chunk(meta, nt);
  const G* g = mt_ptr<const G>(meta, nt, 0, ch.t);
  P* prm = mt_ptr<P>(meta, nt, 1, ch.t);
  float* mst = MASTER ? mt_ptr<float>(meta, nt, 2, ch.t) : reinterpret_cast<float*>(prm);
  float* m = mt_ptr<float>(meta, nt, 3, ch.t);
  const float denom = norms[ch.t] / bc2 + eps;
  SMPK_MT_LOOP(i) {
    float gg[4], p[4], mm[4];
    load4(g, i, ch.e, gg);
    load4(mst, i, ch.e, p);
    load4(m, i, ch.e, mm);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = gg[j] * gscale;
      if (!decoupled) {
        mm[j] = b1 * mm[j] + b3 * (gj / denom + wd * p[j]);
        p[j] -= lr * (mm[j] / bc1);
      } else {
        mm[j] = b1 * mm[j] + b3 * gj;
        p[j] -= lr * ((mm[j] / bc1) / denom + wd * p[j]);
      }
    }
    store4(mst, i, ch.e, p);
    store4(m, i, ch.e, mm);
    if (MASTER) store4(prm, i, ch.e, p);
  }
}

// blended per-tensor NovoGrad norms (apex multi_tensor_norm_out with a = b2, b = 1 - b2):
// L2 gn = sqrt(b2 gn^2 + (1 - b2) n^2) from the new sum of squares; L-inf gn = b2 gn + (1 - b2) n.
// First step: gn starts at n (or at 0 with init_zero).
__global__ void __launch_bounds__(kThreads) novograd_blend_kernel(float* __restrict__ norms,
                                                                  const float* __restrict__ fresh, int64_t nt, float b2,
                                                                  int l2, int first, int init_zero) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t >= nt) return;
  const float n = l2 ? sqrtf(fresh[t]) : fresh[t];
  const float old = first ? (init_zero ? 0.f : n) : norms[t];
  norms[t] = l2 ? sqrtf(b2 * old * old + (1.f - b2) * n * n) : b2 * old + (1.f - b2) * n;
}
#undef SMPK_MT_LOOP

}  // namespace

int mt_adam(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master, float lr,
            float b1, float b2, float eps, float wd, float bc1, float bc2, float gscale, int adamw, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  SMPK_DISPATCH(grad_dt, G, {
    if (!master) {
      if (param_dt != F32) return -2;
      mt_adam_kernel<float, G, false><<<grid, kThreads, 0, s>>>(meta, nt, lr, b1, b2, eps, wd, bc1, bc2, gscale, adamw);
    } else {
      SMPK_DISPATCH(param_dt, P, {
        mt_adam_kernel<P, G, true><<<grid, kThreads, 0, s>>>(meta, nt, lr, b1, b2, eps, wd, bc1, bc2, gscale, adamw);
      });
    }
  });
  return static_cast<int>(hipGetLastError());
}

int mt_norm(const int64_t* meta, int64_t nt, int64_t nchunks, int role, int dt, float scale, int maxabs, float* out,
            hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  SMPK_DISPATCH(dt, T, {
    if (maxabs) {
      mt_norm_kernel<T, true><<<grid, kThreads, 0, s>>>(meta, nt, role, scale, out);
    } else {
      mt_norm_kernel<T, false><<<grid, kThreads, 0, s>>>(meta, nt, role, scale, out);
    }
  });
  return static_cast<int>(hipGetLastError());
}

int mt_lamb1(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master, float b1,
             float b2, float b3, float bc1, float bc2, float eps, float wd, int decoupled, const float* gnorm,
             float max_gnorm, float gscale, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  SMPK_DISPATCH(grad_dt, G, {
    if (!master) {
      if (param_dt != F32) return -2;
      mt_lamb1_kernel<float, G, false><<<grid, kThreads, 0, s>>>(meta, nt, b1, b2, b3, bc1, bc2, eps, wd, decoupled,
                                                                  gnorm, max_gnorm, gscale);
    } else {
      mt_lamb1_kernel<float, G, true><<<grid, kThreads, 0, s>>>(meta, nt, b1, b2, b3, bc1, bc2, eps, wd, decoupled,
                                                                 gnorm, max_gnorm, gscale);
    }
  });
  return static_cast<int>(hipGetLastError());
}

int mt_lamb2(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int master, const float* pn2,
             const float* un2, float lr, int use_trust, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  if (!master) {
    if (param_dt != F32) return -2;
    mt_lamb2_kernel<float, false><<<grid, kThreads, 0, s>>>(meta, nt, pn2, un2, lr, use_trust);
  } else {
    SMPK_DISPATCH(param_dt, P, { mt_lamb2_kernel<P, true><<<grid, kThreads, 0, s>>>(meta, nt, pn2, un2, lr, use_trust); });
  }
  return static_cast<int>(hipGetLastError());
}

int mt_novograd(const int64_t* meta, int64_t nt, int64_t nchunks, int param_dt, int grad_dt, int master,
                const float* norms, float b1, float b3, float bc1, float bc2, float eps, float lr, float wd,
                int decoupled, float gscale, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const unsigned grid = static_cast<unsigned>(nchunks);
  SMPK_DISPATCH(grad_dt, G, {
    if (!master) {
      if (param_dt != F32) return -2;
      mt_novograd_kernel<float, G, false><<<grid, kThreads, 0, s>>>(meta, nt, norms, b1, b3, bc1, bc2, eps, lr, wd,
                                                                     decoupled, gscale);
    } else {
      SMPK_DISPATCH(param_dt, P, {
        mt_novograd_kernel<P, G, true><<<grid, kThreads, 0, s>>>(meta, nt, norms, b1, b3, bc1, bc2, eps, lr, wd,
                                                                  decoupled, gscale);
      });
    }
  });
  return static_cast<int>(hipGetLastError());
}

int novograd_blend(float* norms, const float* fresh, int64_t nt, float b2, int l2, int first, int init_zero,
                   hipStream_t s) {
  if (nt <= 0) return 0;
  novograd_blend_kernel<<<static_cast<unsigned>((nt + kThreads - 1) / kThreads), kThreads, 0, s>>>(
      norms, fresh, nt, b2, l2, first, init_zero);
  return static_cast<int>(hipGetLastError());
}


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

int add3(int dt, const void* a, const void* b, const void* c, void* out, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    int64_t blocks = (n / (16 / static_cast<int64_t>(sizeof(T))) + kThreads - 1) / kThreads;
    blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
    add3_kernel<T><<<static_cast<int>(blocks), kThreads, 0, s>>>(static_cast<const T*>(a), static_cast<const T*>(b),
                                                    static_cast<const T*>(c), static_cast<T*>(out), n);
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
