// Fused bias + tanh-GeLU forward/backward (K17 of SURVEY §2.6; the reference runs this
// as TorchScript, `smp/torch/nn/gelu.py:29-64`) and a column-sum kernel for bias grads.
//
// Elementwise and HBM-bound: 16-byte vectors (8 bf16) per lane, bias broadcast over the
// last dim, fp32 math.  The backward recomputes tanh from the saved pre-activation
// (x + bias is never materialised).
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

constexpr float kC0 = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kC1 = 0.044715f;

__device__ __forceinline__ float gelu_f(float x) {
  const float u = kC0 * (x + kC1 * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

__device__ __forceinline__ float gelu_grad(float x) {
  const float u = kC0 * (x + kC1 * x * x * x);
  const float t = tanhf(u);
  const float du = kC0 * (1.f + 3.f * kC1 * x * x);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
}

// tanh-GeLU in sigmoid form: 0.5 x (1 + tanh(u)) = x * sigmoid(2u), 2u = x (A + B x^2).
// sigmoid(z) = rcp(1 + 2^(-z log2 e)) on the transcendental unit (v_exp_f32, v_rcp_f32):
// 5 VALU + 2 transcendental ops per element forward, 8 + 2 backward (vs 12 / 15 for the
// tanh form) -- these elementwise passes over [tokens, 4h] are VALU-heavy enough for the
// instruction count to matter next to HBM time.  Saturates correctly at +-inf.
constexpr float kA = 2.f * kC0;                                 // d(2u)/dx at x = 0
constexpr float kB = 2.f * kC0 * kC1;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kAn = -kA * kLog2e, kBn = -kB * kLog2e;        // exponent of 2^(-2u log2 e)

__device__ __forceinline__ float gelu_sig(float x, float& x2) {
  x2 = x * x;
  const float z = x * fmaf(kBn, x2, kAn);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));  // sigmoid(2u)
}

__device__ __forceinline__ float gelu_fast(float x) {
  float x2;
  return x * gelu_sig(x, x2);
}

__device__ __forceinline__ float gelu_grad_fast(float x) {
  float x2;
  const float sg = gelu_sig(x, x2);
  const float ds = fmaf(-sg, sg, sg);         // sigmoid' = s (1 - s)
  const float du = fmaf(3.f * kB, x2, kA);    // d(2u)/dx
  return fmaf(x * ds, du, sg);
}

// Exact (erf) GeLU: F.gelu's default, which the reference uses unless fused_bias_gelu or
// SMP_USE_HF_GELU selects the tanh form (`smp/torch/nn/transformer.py:994,1106-1127`).
constexpr float kInvSqrt2 = 0.7071067811865476f;
constexpr float kInvSqrt2Pi = 0.3989422804014327f;

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * kInvSqrt2)); }

__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * kInvSqrt2)) + x * kInvSqrt2Pi * __expf(-0.5f * x * x);
}

// ACT 0: tanh approximation, ACT 1: exact erf.
template <int ACT>
__device__ __forceinline__ float act_fwd(float x) {
  return ACT == 1 ? gelu_erf(x) : gelu_fast(x);
}
template <int ACT>
__device__ __forceinline__ float act_grad(float x) {
  return ACT == 1 ? gelu_erf_grad(x) : gelu_grad_fast(x);
}

template <typename T, bool VEC, int ACT>
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                            T* __restrict__ y, int64_t rows, int64_t cols) {
  constexpr int N = Vec16<T>::N;
  const int64_t total = rows * cols;
  if (VEC) {
    for (int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * N; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256 * N) {
      Vec16<T> a = load16(x + i);
      const int64_t c = i % cols;
      Vec16<T> bb;
      if (bias) bb = load16(bias + c);
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        float v = to_f32(a.v[j]) + (bias ? to_f32(bb.v[j]) : 0.f);
        o.v[j] = from_f32<T>(act_fwd<ACT>(v));
      }
      store16(y + i, o);
    }
  } else {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256) {
      float v = to_f32(x[i]) + (bias ? to_f32(bias[i % cols]) : 0.f);
      y[i] = from_f32<T>(act_fwd<ACT>(v));
    }
  }
}

template <typename T, bool VEC, int ACT>
__global__ void __launch_bounds__(256) bias_gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const T* __restrict__ bias, T* __restrict__ dx,
                                                            int64_t rows, int64_t cols) {
  constexpr int N = Vec16<T>::N;
  const int64_t total = rows * cols;
  if (VEC) {
    for (int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * N; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256 * N) {
      Vec16<T> a = load16(x + i);
      Vec16<T> d = load16(dy + i);
      const int64_t c = i % cols;
      Vec16<T> bb;
      if (bias) bb = load16(bias + c);
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        float v = to_f32(a.v[j]) + (bias ? to_f32(bb.v[j]) : 0.f);
        o.v[j] = from_f32<T>(to_f32(d.v[j]) * act_grad<ACT>(v));
      }
      store16(dx + i, o);
    }
  } else {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256) {
      float v = to_f32(x[i]) + (bias ? to_f32(bias[i % cols]) : 0.f);
      dx[i] = from_f32<T>(to_f32(dy[i]) * act_grad<ACT>(v));
    }
  }
}

// ---------------------------------------------------------------- column walker
// Layout shared by the column-reduction kernels: each lane owns one 16-byte column
// vector (8 bf16) and walks rows; a 256-thread block is CVB column vectors x RL row
// lanes (CVB divides the column-vector count when possible, so no lanes idle on e.g.
// 1600 / 4800 / 6400 columns); grid = (column-vector groups, row parts).  The bias stays
// in registers, no per-element index division, and U independent 16-byte loads per lane
// are in flight before any arithmetic (HBM latency hiding at 4+ waves/SIMD).
struct ColWalk {
  int cvb, rl;
  int64_t groups;
};

inline ColWalk col_walk(int64_t cv) {
  ColWalk w{64, 4, (cv + 63) / 64};
  if (cv < 64) {
    w.cvb = static_cast<int>(cv);
    w.rl = 256 / w.cvb;
    w.groups = 1;
    return w;
  }
  for (int d = 64; d >= 32; --d)
    if (cv % d == 0) {
      w.cvb = d;
      w.rl = 256 / d;
      w.groups = cv / d;
      return w;
    }
  return w;
}

constexpr int kUnroll = 4;

// Column partial sums of x [rows, cols] -> part[blockIdx.y][cols] (fp32).
template <typename T>
__global__ void __launch_bounds__(256) col_sum_vec(const T* __restrict__ x, float* __restrict__ part, int64_t rows,
                                                   int64_t cols, int64_t rows_per_part, int cvb, int rl) {
  constexpr int N = Vec16<T>::N;
  __shared__ float s[256 * N];
  const int cvl = threadIdx.x % cvb, r_l = threadIdx.x / cvb;
  const int64_t c = (static_cast<int64_t>(blockIdx.x) * cvb + cvl) * N;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_part;
  const int64_t r1 = r0 + rows_per_part < rows ? r0 + rows_per_part : rows;
  float acc[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = 0.f;
  const bool active = r_l < rl && c < cols;
  if (active) {
    int64_t r = r0 + r_l;
    for (; r + (kUnroll - 1) * rl < r1; r += kUnroll * rl) {
      Vec16<T> v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = load16(x + (r + u * rl) * cols + c);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int j = 0; j < N; ++j) acc[j] += to_f32(v[u].v[j]);
    }
    for (; r < r1; r += rl) {
      Vec16<T> v = load16(x + r * cols + c);
#pragma unroll
      for (int j = 0; j < N; ++j) acc[j] += to_f32(v.v[j]);
    }
  }
  // combine the row lanes through LDS: s[r_l][cvl*N + j]
  const int width = cvb * N;
  if (r_l < rl)
#pragma unroll
    for (int j = 0; j < N; ++j) s[r_l * width + cvl * N + j] = acc[j];
  __syncthreads();
  for (int k = threadIdx.x; k < width; k += 256) {
    const int64_t col = static_cast<int64_t>(blockIdx.x) * width + k;
    if (col >= cols) continue;
    float a = 0.f;
    for (int q = 0; q < rl; ++q) a += s[q * width + k];
    part[static_cast<int64_t>(blockIdx.y) * cols + col] = a;
  }
}

// Scalar fallback (odd column counts / unaligned): 64 columns x 4 row lanes per block.
template <typename T>
__global__ void __launch_bounds__(256) col_sum_partial(const T* __restrict__ x, float* __restrict__ part,
                                                       int64_t rows, int64_t cols, int64_t rows_per_part) {
  __shared__ float s[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + cl;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_part;
  const int64_t r1 = r0 + rows_per_part < rows ? r0 + rows_per_part : rows;
  float a = 0.f;
  if (c < cols)
    for (int64_t r = r0 + rl; r < r1; r += 4) a += to_f32(x[r * cols + c]);
  s[rl][cl] = a;
  __syncthreads();
  if (rl == 0 && c < cols) part[static_cast<int64_t>(blockIdx.y) * cols + c] = s[0][cl] + s[1][cl] + s[2][cl] + s[3][cl];
}

// Fused backward + bias gradient over the column walker: dx = dy * gelu'(x + b) is
// written once and its column sums (dbias partials) never re-read dx.
template <typename T, int ACT>
__global__ void __launch_bounds__(256) bias_gelu_bwd_dbias_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                  const T* __restrict__ bias, T* __restrict__ dx,
                                                                  float* __restrict__ part, int64_t rows, int64_t cols,
                                                                  int64_t rows_per_part, int cvb, int rl) {
  constexpr int N = Vec16<T>::N;
  constexpr int U = 2;
  __shared__ float s[256 * N];
  const int cvl = threadIdx.x % cvb, r_l = threadIdx.x / cvb;
  const int64_t c = (static_cast<int64_t>(blockIdx.x) * cvb + cvl) * N;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_part;
  const int64_t r1 = r0 + rows_per_part < rows ? r0 + rows_per_part : rows;
  float acc[N], bb[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = 0.f;
  const bool active = r_l < rl && c < cols;
  if (active) {
    Vec16<T> bv = load16(bias + c);
#pragma unroll
    for (int j = 0; j < N; ++j) bb[j] = to_f32(bv.v[j]);
    int64_t r = r0 + r_l;
    for (; r + (U - 1) * rl < r1; r += U * rl) {
      Vec16<T> a[U], d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = load16(x + (r + u * rl) * cols + c);
        d[u] = load16(dy + (r + u * rl) * cols + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        Vec16<T> o;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          o.v[j] = from_f32<T>(to_f32(d[u].v[j]) * act_grad<ACT>(to_f32(a[u].v[j]) + bb[j]));
          acc[j] += to_f32(o.v[j]);
        }
        store16(dx + (r + u * rl) * cols + c, o);
      }
    }
    for (; r < r1; r += rl) {
      Vec16<T> a = load16(x + r * cols + c);
      Vec16<T> d = load16(dy + r * cols + c);
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        o.v[j] = from_f32<T>(to_f32(d.v[j]) * act_grad<ACT>(to_f32(a.v[j]) + bb[j]));
        acc[j] += to_f32(o.v[j]);
      }
      store16(dx + r * cols + c, o);
    }
  }
  const int width = cvb * N;
  if (r_l < rl)
#pragma unroll
    for (int j = 0; j < N; ++j) s[r_l * width + cvl * N + j] = acc[j];
  __syncthreads();
  for (int k = threadIdx.x; k < width; k += 256) {
    const int64_t col = static_cast<int64_t>(blockIdx.x) * width + k;
    if (col >= cols) continue;
    float a = 0.f;
    for (int q = 0; q < rl; ++q) a += s[q * width + k];
    part[static_cast<int64_t>(blockIdx.y) * cols + col] = a;
  }
}

// ---------------------------------------------------------------- one-pass streaming
// One 16-byte vector per lane, one pass (grid = vectors / 256, no grid-stride loop): each
// block streams 4 KB of consecutive memory once.  tools/membw/stream_variants.hip on MI355X
// ([65536, 6400] bf16 read + write): 6.18 TB/s for this shape of access against 4.4-4.6 TB/s
// for grid-stride loops of 1024-4096 blocks (any unroll), which is what the flat / walker
// kernels were.  The bias column comes from L1/L2 (a 12.8 KB row); 32-bit index math.
template <typename T, int ACT, bool BWD>
__global__ void __launch_bounds__(256) bias_gelu_once(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const T* __restrict__ bias, T* __restrict__ y, uint32_t nvec,
                                                      uint32_t cv) {
  constexpr int N = Vec16<T>::N;
  const uint32_t v = blockIdx.x * 256u + threadIdx.x;
  if (v >= nvec) return;
  const Vec16<T> a = load16(x + static_cast<int64_t>(v) * N);
  Vec16<T> bv;
  if (bias != nullptr) {
    bv = load16(bias + (v % cv) * N);
  } else {
    bv.raw = make_uint4(0, 0, 0, 0);
  }
  Vec16<T> o;
  if constexpr (BWD) {
    const Vec16<T> d = load16(dy + static_cast<int64_t>(v) * N);
#pragma unroll
    for (int j = 0; j < N; ++j) o.v[j] = from_f32<T>(to_f32(d.v[j]) * act_grad<ACT>(to_f32(a.v[j]) + to_f32(bv.v[j])));
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) o.v[j] = from_f32<T>(act_fwd<ACT>(to_f32(a.v[j]) + to_f32(bv.v[j])));
  }
  store16(y + static_cast<int64_t>(v) * N, o);
}

template <typename T, bool BWD>
void launch_once(const void* dy, const void* x, const void* bias, void* y, int64_t nvec, int64_t cv, bool exact,
                 hipStream_t s) {
  const unsigned g = static_cast<unsigned>((nvec + 255) / 256);
  if (exact)
    bias_gelu_once<T, 1, BWD><<<g, 256, 0, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                                static_cast<const T*>(bias), static_cast<T*>(y),
                                                static_cast<uint32_t>(nvec), static_cast<uint32_t>(cv));
  else
    bias_gelu_once<T, 0, BWD><<<g, 256, 0, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                                static_cast<const T*>(bias), static_cast<T*>(y),
                                                static_cast<uint32_t>(nvec), static_cast<uint32_t>(cv));
}
// [parts, cols] fp32 -> [cols] in two deterministic stages (slices of parts, then slices).
__global__ void __launch_bounds__(256) parts_reduce_stage1(const float* __restrict__ part, float* __restrict__ out,
                                                           int parts, int64_t cols, int slices) {
  __shared__ float s[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + cl;
  const int per = (parts + slices - 1) / slices;
  const int p0 = blockIdx.y * per, p1 = min(parts, p0 + per);
  float a = 0.f;
  if (c < cols)
    for (int p = p0 + pl; p < p1; p += 4) a += part[static_cast<int64_t>(p) * cols + c];
  s[pl][cl] = a;
  __syncthreads();
  if (pl == 0 && c < cols) out[static_cast<int64_t>(blockIdx.y) * cols + c] = s[0][cl] + s[1][cl] + s[2][cl] + s[3][cl];
}

template <typename T>
__global__ void __launch_bounds__(256) parts_reduce_stage2(const float* __restrict__ part, T* __restrict__ out,
                                                           int slices, int64_t cols, bool accumulate) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= cols) return;
  float a = accumulate ? to_f32(out[c]) : 0.f;
  // eight slice loads in flight at a time, added in slice order (deterministic)
  for (int p = 0; p < slices; p += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p + j < slices ? part[static_cast<int64_t>(p + j) * cols + c] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) a += v[j];
  }
  out[c] = from_f32<T>(a);
}

constexpr int kReduceSlices = 32;

template <typename T>
void reduce_parts(const float* part, int parts, int64_t cols, float* work, T* out, hipStream_t s,
                  bool accumulate = false) {
  const int slices = parts < kReduceSlices ? parts : kReduceSlices;
  dim3 g(static_cast<unsigned>((cols + 63) / 64), static_cast<unsigned>(slices));
  parts_reduce_stage1<<<g, 256, 0, s>>>(part, work, parts, cols, slices);
  parts_reduce_stage2<T><<<static_cast<unsigned>((cols + 255) / 256), 256, 0, s>>>(work, out, slices, cols,
                                                                                   accumulate);
}

inline int elt_grid(int64_t total, int per_thread) {
  int64_t b = (total / per_thread + 255) / 256;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return static_cast<int>(b);
}

template <typename T, bool V, int A>
void launch_gelu_bwd(const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int64_t cols,
                     hipStream_t s) {
  constexpr int N = Vec16<T>::N;
  bias_gelu_bwd_kernel<T, V, A><<<elt_grid(rows * cols, V ? N : 1), 256, 0, s>>>(
      static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(bias), static_cast<T*>(dx), rows,
      cols);
}

}  // namespace

int bias_gelu_fwd(int dt, const void* x, const void* bias, void* y, int64_t rows, int64_t cols, hipStream_t s,
                  bool exact) {
  const int64_t total = rows * cols;
  if (total <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool vec = (cols % N == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                                          reinterpret_cast<uintptr_t>(bias)) & 15) == 0;
    if (vec && total / N < (int64_t{1} << 31)) {
      launch_once<T, false>(nullptr, x, bias, y, total / N, cols / N, exact, s);
    } else {
      if (exact)
        bias_gelu_fwd_kernel<T, false, 1><<<elt_grid(total, 1), 256, 0, s>>>(
            static_cast<const T*>(x), static_cast<const T*>(bias), static_cast<T*>(y), rows, cols);
      else
        bias_gelu_fwd_kernel<T, false, 0><<<elt_grid(total, 1), 256, 0, s>>>(
            static_cast<const T*>(x), static_cast<const T*>(bias), static_cast<T*>(y), rows, cols);
    }
  });
  return static_cast<int>(hipGetLastError());
}

int bias_gelu_bwd(int dt, const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int64_t cols,
                  hipStream_t s, bool exact) {
  const int64_t total = rows * cols;
  if (total <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool vec = (cols % N == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
                                          reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(bias)) &
                                         15) == 0;
    if (vec && total / N < (int64_t{1} << 31))
      launch_once<T, true>(dy, x, bias, dx, total / N, cols / N, exact, s);
    else if (vec && exact)
      launch_gelu_bwd<T, true, 1>(dy, x, bias, dx, rows, cols, s);
    else if (vec)
      launch_gelu_bwd<T, true, 0>(dy, x, bias, dx, rows, cols, s);
    else if (exact)
      launch_gelu_bwd<T, false, 1>(dy, x, bias, dx, rows, cols, s);
    else
      launch_gelu_bwd<T, false, 0>(dy, x, bias, dx, rows, cols, s);
  });
  return static_cast<int>(hipGetLastError());
}

// workspace: (col_sum_parts(rows) + 32) * cols floats.
int col_sum_parts(int64_t rows) {
  int64_t parts = (rows + 63) / 64;
  if (parts > 256) parts = 256;
  return static_cast<int>(parts < 1 ? 1 : parts);
}

int col_sum(int dt, const void* x, void* out, float* workspace, int64_t rows, int64_t cols, hipStream_t s,
            bool accumulate) {
  if (rows <= 0 || cols <= 0) return 0;
  const int parts = col_sum_parts(rows);
  const int64_t rpp = (rows + parts - 1) / parts;
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool vec = (cols % N == 0) && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (vec) {
      const ColWalk w = col_walk(cols / N);
      dim3 g(static_cast<unsigned>(w.groups), static_cast<unsigned>(parts));
      col_sum_vec<T><<<g, 256, 0, s>>>(static_cast<const T*>(x), workspace, rows, cols, rpp, w.cvb, w.rl);
    } else {
      dim3 g(static_cast<unsigned>((cols + 63) / 64), static_cast<unsigned>(parts));
      col_sum_partial<T><<<g, 256, 0, s>>>(static_cast<const T*>(x), workspace, rows, cols, rpp);
    }
    reduce_parts<T>(workspace, parts, cols, workspace + static_cast<int64_t>(parts) * cols, static_cast<T*>(out), s,
                    accumulate);
  });
  return static_cast<int>(hipGetLastError());
}

// Workspace rows (partials) bias_gelu_bwd_dbias needs (col_sum_parts); the caller adds 32
// rows for the second reduction stage.
int gelu_dbias_parts(int64_t rows) { return col_sum_parts(rows); }

// dx = dy * gelu'(x + bias) and dbias = colsum(dx) in one pass over dy/x.
// Returns -2 when the shape/alignment needs the unfused path.  workspace as col_sum.
int bias_gelu_bwd_dbias(int dt, const void* dy, const void* x, const void* bias, void* dx, void* dbias,
                        float* workspace, int64_t rows, int64_t cols, hipStream_t s, bool accumulate,
                        bool exact) {
  if (rows <= 0 || cols <= 0) return 0;
  const int parts = col_sum_parts(rows);
  const int64_t rpp = (rows + parts - 1) / parts;
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool vec = bias != nullptr && (cols % N == 0) &&
                     ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
                       reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(bias)) & 15) == 0;
    if (!vec) return -2;
    const ColWalk w = col_walk(cols / N);
    dim3 g(static_cast<unsigned>(w.groups), static_cast<unsigned>(parts));
    if (exact)
      bias_gelu_bwd_dbias_kernel<T, 1><<<g, 256, 0, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                                         static_cast<const T*>(bias), static_cast<T*>(dx), workspace,
                                                         rows, cols, rpp, w.cvb, w.rl);
    else
      bias_gelu_bwd_dbias_kernel<T, 0><<<g, 256, 0, s>>>(static_cast<const T*>(dy), static_cast<const T*>(x),
                                                         static_cast<const T*>(bias), static_cast<T*>(dx), workspace,
                                                         rows, cols, rpp, w.cvb, w.rl);
    reduce_parts<T>(workspace, parts, cols, workspace + static_cast<int64_t>(parts) * cols, static_cast<T*>(dbias), s,
                    accumulate);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
