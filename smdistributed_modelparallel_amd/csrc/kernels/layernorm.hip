// Fused LayerNorm forward/backward (K9/K10/K11 of SURVEY §2.6) and the distributed-LN
// "apply with global statistics" piece (K6).
//
// One wave64 per row: every lane keeps VPT 16-byte vectors of its row in registers, so
// x is read once, mean/variance come from two wave reductions (exact two-pass variance
// on the register copy) and y is written once.  4 rows per 256-thread block.  An
// optional residual input is added in the same pass and the sum written out
// (pre-LN transformer: h = h + f(h); ln(h) in one kernel).
// Rows wider than the register budget fall back to a block-per-row streaming kernel.
//
// Backward: dx per row in registers; dgamma/dbeta accumulated per lane across the rows a
// block owns, combined across the block's waves in LDS and written as fp32 partials,
// then reduced by a column kernel (deterministic, no atomics).
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

constexpr int kRowsPerBlock = 4;

// N consecutive affine parameters (any W dtype) as fp32, with 16-byte loads when possible.
template <typename W, int N>
__device__ __forceinline__ void load_wn(const W* p, float (&o)[N]) {
  if constexpr (sizeof(W) * N == 16) {
    Vec16<W> a = load16(p);
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = to_f32(a.v[j]);
  } else if constexpr (sizeof(W) * N == 32) {
    constexpr int H = N / 2;
    Vec16<W> a = load16(p), b = load16(p + H);
#pragma unroll
    for (int j = 0; j < H; ++j) {
      o[j] = to_f32(a.v[j]);
      o[H + j] = to_f32(b.v[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = to_f32(p[j]);
  }
}

// TO: output dtype -- T, or W for the mixed-dtype LayerNorm (apex MixedFusedLayerNorm, K10:
// the output takes the parameters' dtype, computed from the fp32 statistics directly).
template <typename TO, typename T, int N>
__device__ __forceinline__ void store_out(TO* p, const float (&o)[N]) {
  if constexpr (sizeof(TO) * N == 16) {
    Vec16<TO> v;
#pragma unroll
    for (int j = 0; j < N; ++j) v.v[j] = from_f32<TO>(o[j]);
    store16(p, v);
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = from_f32<TO>(o[j]);
  }
}

template <typename T, typename W, int VPT, typename TO = T>
__global__ void __launch_bounds__(256) ln_fwd_reg(const T* __restrict__ x, const T* __restrict__ res,
                                                  T* __restrict__ x_out, const W* __restrict__ w,
                                                  const W* __restrict__ b, TO* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                  int64_t rows, int cols, float eps, DropoutArgs drop) {
  constexpr int N = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * cols;
  const uint32_t dkey = drop.thr ? dropout_key(drop) : 0u;
  float v[VPT][N];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = (k * 64 + lane) * N;
    if (c < cols) {
      Vec16<T> a = load16(xr + c);
      if (res != nullptr) {
        Vec16<T> r = load16(res + row * cols + c);
        float f[N];
        if (drop.thr) {  // x_out = residual + dropout(x)
          static_assert(N == 8 || N == 4, "dropout factors come in groups of 8");
          if constexpr (N == 8) {
            dropout_factors8(dkey, row * cols + c, drop, f);
          } else {
#pragma unroll
            for (int j = 0; j < N; ++j) f[j] = dropout_factor1(dkey, row * cols + c + j, drop);
          }
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) f[j] = 1.f;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
          v[k][j] = fmaf(to_f32(a.v[j]), f[j], to_f32(r.v[j]));
          a.v[j] = from_f32<T>(v[k][j]);
        }
        store16(x_out + row * cols + c, a);
#pragma unroll
        for (int j = 0; j < N; ++j) v[k][j] = to_f32(a.v[j]);  // normalise the rounded sum
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) v[k][j] = to_f32(a.v[j]);
      }
#pragma unroll
      for (int j = 0; j < N; ++j) sum += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) v[k][j] = 0.f;
    }
  }
  const float mean = wave_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = (k * 64 + lane) * N;
    if (c < cols) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float d = v[k][j] - mean;
        sq += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / cols + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = (k * 64 + lane) * N;
    if (c < cols) {
      float g[N], bb[N];
      if (w) {
        load_wn<W, N>(w + c, g);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) g[j] = 1.f;
      }
      if (b) {
        load_wn<W, N>(b + c, bb);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) bb[j] = 0.f;
      }
      float o[N];
#pragma unroll
      for (int j = 0; j < N; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + bb[j];
      store_out<TO, T, N>(y + row * cols + c, o);
    }
  }
}

// Generic fallback: one block per row, streaming (any width, any alignment).
template <typename T, typename W, typename TO = T>
__global__ void __launch_bounds__(256) ln_fwd_stream(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ x_out, const W* __restrict__ w,
                                                     const W* __restrict__ b, TO* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int cols, float eps, DropoutArgs drop) {
  __shared__ float smem[16];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  const uint32_t dkey = drop.thr ? dropout_key(drop) : 0u;
  float sum = 0.f;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float a = to_f32(xr[c]);
    if (res != nullptr) {
      const float f = drop.thr ? dropout_factor1(dkey, row * cols + c, drop) : 1.f;
      T s = from_f32<T>(fmaf(a, f, to_f32(res[row * cols + c])));
      x_out[row * cols + c] = s;
      a = to_f32(s);
    }
    sum += a;
  }
  const T* src = res != nullptr ? x_out + row * cols : xr;
  const float mean = block_sum(sum, smem) / cols;
  float sq = 0.f;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    const float d = to_f32(src[c]) - mean;
    sq += d * d;
  }
  const float rstd = rsqrtf(block_sum(sq, smem) / cols + eps);
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float g = w ? to_f32(w[c]) : 1.f;
    float bb = b ? to_f32(b[c]) : 0.f;
    y[row * cols + c] = from_f32<TO>((to_f32(src[c]) - mean) * rstd * g + bb);
  }
}

// Wide rows (more than 64 x 8 16-byte vectors: GPT-NeoX 6144, GPT-3 12288 in bf16): one
// 256-thread block per row, thread t holding vectors t, t + 256, .. (VB of them) in registers:
// x read once with 16-byte loads, two block reductions, y written once.  (The streaming
// fallback this replaces re-read the row three times with 2-byte accesses: ~1 TB/s at 6144.)
template <typename T, typename W, int VB, typename TO = T>
__global__ void __launch_bounds__(256) ln_fwd_wide(const T* __restrict__ x, const T* __restrict__ res,
                                                   T* __restrict__ x_out, const W* __restrict__ w,
                                                   const W* __restrict__ b, TO* __restrict__ y,
                                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                   int64_t rows, int cols, float eps, DropoutArgs drop) {
  constexpr int N = Vec16<T>::N;
  __shared__ float smem[16];
  const int t = threadIdx.x;
  const int64_t row = blockIdx.x;
  const int nvec = cols / N;
  const uint32_t dkey = drop.thr ? dropout_key(drop) : 0u;
  float v[VB][N];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    const int vi = t + 256 * k;
#pragma unroll
    for (int j = 0; j < N; ++j) v[k][j] = 0.f;
    if (vi < nvec) {
      const int64_t off = row * cols + static_cast<int64_t>(vi) * N;
      Vec16<T> a = load16(x + off);
      if (res != nullptr) {
        Vec16<T> r = load16(res + off);
        float f[N];
        if (drop.thr) {
          if constexpr (N == 8) {
            dropout_factors8(dkey, off, drop, f);
          } else {
#pragma unroll
            for (int j = 0; j < N; ++j) f[j] = dropout_factor1(dkey, off + j, drop);
          }
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) f[j] = 1.f;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) a.v[j] = from_f32<T>(fmaf(to_f32(a.v[j]), f[j], to_f32(r.v[j])));
        store16(x_out + off, a);
      }
#pragma unroll
      for (int j = 0; j < N; ++j) {
        v[k][j] = to_f32(a.v[j]);  // (the rounded sum is what is normalised)
        sum += v[k][j];
      }
    }
  }
  const float mean = block_sum(sum, smem) / cols;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    if (t + 256 * k < nvec) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float d = v[k][j] - mean;
        sq += d * d;
      }
    }
  }
  const float rstd = rsqrtf(block_sum(sq, smem) / cols + eps);
  if (t == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    const int vi = t + 256 * k;
    if (vi < nvec) {
      const int c = vi * N;
      float g[N], bb[N], o[N];
      if (w) {
        load_wn<W, N>(w + c, g);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) g[j] = 1.f;
      }
      if (b) {
        load_wn<W, N>(b + c, bb);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) bb[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < N; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + bb[j];
      store_out<TO, T, N>(y + row * cols + c, o);
    }
  }
}

// Wide-row backward: a block per `rows_per_block` rows, thread t owning vectors t + 256 k of
// every row; the row's x / dy (/ dres) stay in registers as packed 16-byte vectors between
// the reduction pass and the dx pass, gamma is re-read from L1/L2 per row (instead of VB x N
// more registers), and dgamma / dbeta accumulate per thread over the block's rows into one fp32
// partial row per block (parts = the register paths' count: no [rows, cols] partials).
// ext: the distributed LayerNorm's all-reduced row sums replace the local reduction.
template <typename T, typename W, int VB>
__global__ void __launch_bounds__(256) ln_bwd_wide(const T* __restrict__ dy, const T* __restrict__ x,
                                                   const W* __restrict__ w, const float* __restrict__ mean_in,
                                                   const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                   float* __restrict__ dw_part, float* __restrict__ db_part,
                                                   int64_t rows, int cols, const T* __restrict__ dres,
                                                   int64_t rows_per_block, const float* __restrict__ ext,
                                                   float ext_n) {
  constexpr int N = Vec16<T>::N;
  __shared__ float smem[2][16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int nvec = cols / N;
  float dwacc[VB][N], dbacc[VB][N];
#pragma unroll
  for (int k = 0; k < VB; ++k) {
#pragma unroll
    for (int j = 0; j < N; ++j) dwacc[k][j] = dbacc[k][j] = 0.f;
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  // a ring of two register rows (VB <= 4: the second set fits beside the dgamma / dbeta
  // accumulators): the next row's x / dy / dres loads are in flight while this row reduces,
  // crosses its barrier and writes dx -- one row at a time left each block waiting on HBM
  // (A/B against one row at a time: profiles/r5/shards_r5.md)
  constexpr bool RING = VB <= 4;
  constexpr int VR = RING ? VB : 1;
  Vec16<T> xa[VB], da[VB], ra[VB], xn[VR], dn[VR], rn[VR];
  auto load_row = [&](int64_t row, Vec16<T>* xx, Vec16<T>* dd, Vec16<T>* rr) {
#pragma unroll
    for (int k = 0; k < VB; ++k) {
      const int vi = t + 256 * k;
      if (vi < nvec) {
        const int64_t off = row * cols + static_cast<int64_t>(vi) * N;
        xx[k] = load16(x + off);
        dd[k] = load16(dy + off);
        if (dres != nullptr) rr[k] = load16(dres + off);
      }
    }
  };
  if (RING && r0 < r1) load_row(r0, xa, da, ra);
  for (int64_t row = r0; row < r1; ++row) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    if constexpr (RING) {
      if (row + 1 < r1) load_row(row + 1, xn, dn, rn);
    } else {
      load_row(row, xa, da, ra);
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VB; ++k) {
      const int vi = t + 256 * k;
      if (vi < nvec) {
        float g[N];
        if (w) {
          load_wn<W, N>(w + vi * N, g);
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) g[j] = 1.f;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const float dyv = to_f32(da[k].v[j]);
          const float xh = (to_f32(xa[k].v[j]) - mean) * rstd;
          const float gg = dyv * g[j];
          s1 += gg;
          s2 += gg * xh;
          dwacc[k][j] += dyv * xh;
          dbacc[k][j] += dyv;
        }
      }
    }
    // both row sums in one barrier pair (double-buffered by row parity)
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    float* red = smem[row & 1];
    if (lane == 0) {
      red[wid] = s1;
      red[8 + wid] = s2;
    }
    __syncthreads();
    if (ext != nullptr) {
      s1 = ext[2 * row] / ext_n;
      s2 = ext[2 * row + 1] / ext_n;
    } else {
      s1 = (red[0] + red[1] + red[2] + red[3]) / cols;
      s2 = (red[8] + red[9] + red[10] + red[11]) / cols;
    }
#pragma unroll
    for (int k = 0; k < VB; ++k) {
      const int vi = t + 256 * k;
      if (vi < nvec) {
        const int64_t off = row * cols + static_cast<int64_t>(vi) * N;
        float g[N];
        if (w) {
          load_wn<W, N>(w + vi * N, g);
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) g[j] = 1.f;
        }
        Vec16<T> o;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const float xh = (to_f32(xa[k].v[j]) - mean) * rstd;
          float vv = rstd * (to_f32(da[k].v[j]) * g[j] - s1 - xh * s2);
          if (dres != nullptr) vv += to_f32(ra[k].v[j]);
          o.v[j] = from_f32<T>(vv);
        }
        store16(dx + off, o);
      }
    }
    if constexpr (RING) {
#pragma unroll
      for (int k = 0; k < VB; ++k) {
        xa[k] = xn[k];
        da[k] = dn[k];
        ra[k] = rn[k];
      }
    }
  }
  if (dw_part == nullptr) return;
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    const int vi = t + 256 * k;
    if (vi >= nvec) continue;
    const int64_t c = static_cast<int64_t>(vi) * N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      dw_part[static_cast<int64_t>(blockIdx.x) * cols + c + j] = dwacc[k][j];
      if (db_part) db_part[static_cast<int64_t>(blockIdx.x) * cols + c + j] = dbacc[k][j];
    }
  }
}

// vectors per thread of the wide kernels (0: not a wide row): 3 / 4 / 6 x 256 16-byte vectors
constexpr int kLnWideMaxVB = 6;
__host__ __device__ inline int ln_wide_vb(int64_t nvec) {
  if (nvec <= 512 || nvec > 256 * kLnWideMaxVB) return 0;
  return nvec <= 768 ? 3 : (nvec <= 1024 ? 4 : 6);
}

template <typename T, typename W, int VPT>
__global__ void __launch_bounds__(256) ln_bwd_reg(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const W* __restrict__ w, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                  float* __restrict__ dw_part, float* __restrict__ db_part,
                                                  int64_t rows, int cols, const T* __restrict__ dres,
                                                  const float* __restrict__ ext, float ext_n) {
  constexpr int N = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float dwacc[VPT][N], dbacc[VPT][N], wv[VPT][N];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = (k * 64 + lane) * N;
    if (w != nullptr && c < cols) {
      load_wn<W, N>(w + c, wv[k]);
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) wv[k][j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) dwacc[k][j] = dbacc[k][j] = 0.f;
  }

  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock + wid; row < rows;
       row += static_cast<int64_t>(gridDim.x) * kRowsPerBlock) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[VPT][N], g[VPT][N];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int c = (k * 64 + lane) * N;
      if (c < cols) {
        Vec16<T> a = load16(x + row * cols + c);
        Vec16<T> d = load16(dy + row * cols + c);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const float dyv = to_f32(d.v[j]);
          xh[k][j] = (to_f32(a.v[j]) - mean) * rstd;
          g[k][j] = dyv * wv[k][j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
          dwacc[k][j] += dyv * xh[k][j];
          dbacc[k][j] += dyv;
        }
      }
    }
    if (ext != nullptr) {  // distributed LN: row sums over the whole TP-sharded row
      s1 = ext[2 * row] / ext_n;
      s2 = ext[2 * row + 1] / ext_n;
    } else {
      s1 = wave_sum(s1) / cols;
      s2 = wave_sum(s2) / cols;
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int c = (k * 64 + lane) * N;
      if (c < cols) {
        Vec16<T> o;
        Vec16<T> r;
        if (dres != nullptr) r = load16(dres + row * cols + c);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          float v = rstd * (g[k][j] - s1 - xh[k][j] * s2);
          if (dres != nullptr) v += to_f32(r.v[j]);
          o.v[j] = from_f32<T>(v);
        }
        store16(dx + row * cols + c, o);
      }
    }
  }
  // every wave parks its dgamma/dbeta sums in its own LDS slice, then the block adds the
  // 4 slices column-wise and writes one fp32 partial row
  extern __shared__ float lds[];  // [kRowsPerBlock][2][cols]
  if (dw_part == nullptr) return;
  float* mine = lds + static_cast<int64_t>(wid) * 2 * cols;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = (k * 64 + lane) * N;
    if (c < cols) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        mine[c + j] = dwacc[k][j];
        mine[cols + c + j] = dbacc[k][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * cols; c += blockDim.x) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < kRowsPerBlock; ++r) a += lds[r * 2 * cols + c];
    if (c < cols) {
      dw_part[static_cast<int64_t>(blockIdx.x) * cols + c] = a;
    } else if (db_part) {
      db_part[static_cast<int64_t>(blockIdx.x) * cols + c - cols] = a;
    }
  }
}

// Backward, block-per-row-group form for rows of <= 256 (VB=1) or 512 (VB=2) 16-byte
// vectors (e.g. hidden 1600 / 4096 in bf16): the 256 threads of a block share each row
// (thread t owns vectors t and t+256), so a thread's dgamma/dbeta accumulators cover only
// its own columns for all the block's rows -- 8*VB floats each instead of a wave's whole
// row -- and need no LDS combine: the block writes its fp32 partial row directly.  Row
// sums go through one LDS exchange per row (double-buffered: one barrier per row); x / dy /
// dres are loaded two rows ahead (a ring of two register sets).
// Low register use (high occupancy) is what the one-wave-per-row kernel lacked at 1600.
template <typename T, typename W, int VB>
__global__ void __launch_bounds__(256) ln_bwd_blk(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const W* __restrict__ w, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                  float* __restrict__ dw_part, float* __restrict__ db_part,
                                                  int64_t rows, int cols, const T* __restrict__ dres,
                                                  int64_t rows_per_block, T* __restrict__ dxd, DropoutArgs drop) {
  constexpr int N = Vec16<T>::N;
  __shared__ float red[2][2][4];  // [parity][s1|s2][wave]
  // dxd != null: also the dropout branch's gradient dxd = dx * keep / (1 - p), decisions from the
  // forward's element-index hash (the separate dropout_bwd pass re-read dx for this)
  const uint32_t dkey = dxd != nullptr ? dropout_key(drop) : 0u;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int nvec = cols / N;
  float wv[VB][N], dwacc[VB][N], dbacc[VB][N];
  bool act[VB];
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    const int v = t + 256 * k;
    act[k] = v < nvec;
    if (act[k] && w != nullptr) {
      load_wn<W, N>(w + v * N, wv[k]);
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) wv[k][j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) dwacc[k][j] = dbacc[k][j] = 0.f;
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  // two rows of x / dy / dres in flight (register ring of 2): the loads of row + 2 go out as
  // soon as row's values are in float registers, i.e. ahead of row's reduction and barrier
  Vec16<T> xa[2][VB], da[2][VB], ra[2][VB];
  auto load_row = [&](int64_t row, auto buf_c) {
    constexpr int B = decltype(buf_c)::value;
#pragma unroll
    for (int k = 0; k < VB; ++k) {
      if (act[k]) {
        const int64_t off = row * cols + static_cast<int64_t>(t + 256 * k) * N;
        xa[B][k] = load16(x + off);
        da[B][k] = load16(dy + off);
        if (dres != nullptr) ra[B][k] = load16(dres + off);
      }
    }
  };
  int parity = 0;
  auto body = [&](int64_t row, auto buf_c) {
    constexpr int B = decltype(buf_c)::value;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[VB][N], g[VB][N], rr[VB][N];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VB; ++k) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float dyv = act[k] ? to_f32(da[B][k].v[j]) : 0.f;
        xh[k][j] = act[k] ? (to_f32(xa[B][k].v[j]) - mean) * rstd : 0.f;
        rr[k][j] = (act[k] && dres != nullptr) ? to_f32(ra[B][k].v[j]) : 0.f;
        g[k][j] = dyv * wv[k][j];
        s1 += g[k][j];
        s2 += g[k][j] * xh[k][j];
        dwacc[k][j] += dyv * xh[k][j];
        dbacc[k][j] += dyv;
      }
    }
    if (row + 2 < r1) load_row(row + 2, buf_c);  // this buffer's next row, two ahead
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[parity][0][wid] = s1;
      red[parity][1][wid] = s2;
    }
    __syncthreads();
    s1 = (red[parity][0][0] + red[parity][0][1] + red[parity][0][2] + red[parity][0][3]) / cols;
    s2 = (red[parity][1][0] + red[parity][1][1] + red[parity][1][2] + red[parity][1][3]) / cols;
    parity ^= 1;
#pragma unroll
    for (int k = 0; k < VB; ++k) {
      if (!act[k]) continue;
      Vec16<T> o;
      float dv[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        dv[j] = rstd * (g[k][j] - s1 - xh[k][j] * s2) + rr[k][j];
        o.v[j] = from_f32<T>(dv[j]);
      }
      const int64_t off = row * cols + static_cast<int64_t>(t + 256 * k) * N;
      store16(dx + off, o);
      if (dxd != nullptr) {
        // the dropout factor multiplies the ROUNDED dx, exactly as dropout_bwd(dx) did
        float f[8];
        if constexpr (N == 8) {
          dropout_factors8(dkey, off, drop, f);
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) f[j] = dropout_factor1(dkey, off + j, drop);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) o.v[j] = from_f32<T>(to_f32(o.v[j]) * f[j]);
        store16(dxd + off, o);
      }
    }
  };
  if (r0 < r1) load_row(r0, std::integral_constant<int, 0>{});
  if (r0 + 1 < r1) load_row(r0 + 1, std::integral_constant<int, 1>{});
  for (int64_t row = r0; row < r1; row += 2) {
    body(row, std::integral_constant<int, 0>{});
    if (row + 1 < r1) body(row + 1, std::integral_constant<int, 1>{});
  }
  if (dw_part == nullptr) return;
#pragma unroll
  for (int k = 0; k < VB; ++k) {
    if (!act[k]) continue;
    const int64_t c = static_cast<int64_t>(t + 256 * k) * N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      dw_part[static_cast<int64_t>(blockIdx.x) * cols + c + j] = dwacc[k][j];
      if (db_part) db_part[static_cast<int64_t>(blockIdx.x) * cols + c + j] = dbacc[k][j];
    }
  }
}

template <typename T, typename W>
__global__ void __launch_bounds__(256) ln_bwd_stream(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                     float* __restrict__ dw_part, float* __restrict__ db_part,
                                                     int64_t rows, int cols, const T* __restrict__ dres,
                                                     const float* __restrict__ ext, float ext_n) {
  // one block per row; dw/db partial per row (parts == rows) -- only used for odd shapes
  __shared__ float smem[16];
  const int64_t row = blockIdx.x;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    const float dyv = to_f32(dy[row * cols + c]);
    const float xh = (to_f32(x[row * cols + c]) - mean) * rstd;
    const float gg = dyv * (w ? to_f32(w[c]) : 1.f);
    s1 += gg;
    s2 += gg * xh;
    if (dw_part) dw_part[row * cols + c] = dyv * xh;
    if (db_part) db_part[row * cols + c] = dyv;
  }
  s1 = block_sum(s1, smem) / cols;
  s2 = block_sum(s2, smem) / cols;
  if (ext != nullptr) {
    s1 = ext[2 * row] / ext_n;
    s2 = ext[2 * row + 1] / ext_n;
  }
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    const float dyv = to_f32(dy[row * cols + c]);
    const float xh = (to_f32(x[row * cols + c]) - mean) * rstd;
    const float gg = dyv * (w ? to_f32(w[c]) : 1.f);
    float v = rstd * (gg - s1 - xh * s2);
    if (dres) v += to_f32(dres[row * cols + c]);
    dx[row * cols + c] = from_f32<T>(v);
  }
}

// Stage 1: block (column chunk of 64, part slice) sums its slice of the partial rows.
__global__ void __launch_bounds__(256) ln_bwd_reduce_stage1(const float* __restrict__ dw_part,
                                                            const float* __restrict__ db_part, float* __restrict__ out,
                                                            int parts, int64_t cols, int slices) {
  __shared__ float sw[4][64], sb[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + cl;
  const int per = (parts + slices - 1) / slices;
  const int p0 = blockIdx.y * per, p1 = min(parts, p0 + per);
  float a = 0.f, b = 0.f;
  if (c < cols) {
    for (int p = p0 + pl; p < p1; p += 4) {
      a += dw_part[p * cols + c];
      if (db_part) b += db_part[p * cols + c];
    }
  }
  sw[pl][cl] = a;
  sb[pl][cl] = b;
  __syncthreads();
  if (pl == 0 && c < cols) {
    out[static_cast<int64_t>(blockIdx.y) * 2 * cols + c] = sw[0][cl] + sw[1][cl] + sw[2][cl] + sw[3][cl];
    out[static_cast<int64_t>(blockIdx.y) * 2 * cols + cols + c] = sb[0][cl] + sb[1][cl] + sb[2][cl] + sb[3][cl];
  }
}

// Stage 2: one thread per column adds the slice sums (fixed order: deterministic).
template <typename W>
__global__ void __launch_bounds__(256) ln_bwd_reduce_stage2(const float* __restrict__ part2, W* __restrict__ dw,
                                                            W* __restrict__ db, int64_t cols, int slices,
                                                            bool accumulate) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= cols) return;
  float a = (accumulate && dw) ? to_f32(dw[c]) : 0.f;
  float b = (accumulate && db) ? to_f32(db[c]) : 0.f;
  // the slice loads in flight together (the adds keep their fixed order): a rolled loop waited
  // for each load in turn, 12 us per call for 32 slices
  float va[kLnReduceSlices], vb[kLnReduceSlices];
#pragma unroll
  for (int s = 0; s < kLnReduceSlices; ++s) {
    va[s] = s < slices ? part2[static_cast<int64_t>(s) * 2 * cols + c] : 0.f;
    vb[s] = s < slices ? part2[static_cast<int64_t>(s) * 2 * cols + cols + c] : 0.f;
  }
#pragma unroll
  for (int s = 0; s < kLnReduceSlices; ++s) {
    a += va[s];
    b += vb[s];
  }
  if (dw) dw[c] = from_f32<W>(a);
  if (db) db[c] = from_f32<W>(b);
}

template <typename T, typename W>
__global__ void __launch_bounds__(256) ln_apply_stats(const T* __restrict__ x, const W* __restrict__ w,
                                                      const W* __restrict__ b, const float* __restrict__ mean,
                                                      const float* __restrict__ var, T* __restrict__ y,
                                                      float* __restrict__ rstd_out, int64_t rows, int cols,
                                                      float eps) {
  const int64_t row = blockIdx.x;
  const float m = mean[row];
  const float r = rsqrtf(var[row] + eps);
  if (threadIdx.x == 0 && rstd_out) rstd_out[row] = r;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    const float g = w ? to_f32(w[c]) : 1.f;
    const float bb = b ? to_f32(b[c]) : 0.f;
    y[row * cols + c] = from_f32<T>((to_f32(x[row * cols + c]) - m) * r * g + bb);
  }
}

template <typename T>
bool vec_ok(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

}  // namespace

namespace {
template <typename T, typename W, typename TO>
void launch_ln_fwd(const void* x, const void* residual, void* x_out, const void* w, const void* b, void* y,
                   float* mean, float* rstd, int64_t rows, int64_t cols, float eps, hipStream_t s,
                   const DropoutArgs& drop) {
  constexpr int N = Vec16<T>::N;
  const bool aligned = (cols % N == 0) && vec_ok<T>(x) && vec_ok<TO>(y) && vec_ok<W>(w) && vec_ok<W>(b) &&
                       (residual == nullptr || (vec_ok<T>(residual) && vec_ok<T>(x_out)));
  const int vpt = static_cast<int>((cols + 64 * N - 1) / (64 * N));
  const int grid = static_cast<int>((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  const T* xx = static_cast<const T*>(x);
  const T* rr = static_cast<const T*>(residual);
  T* xo = static_cast<T*>(x_out);
  const W* ww = static_cast<const W*>(w);
  const W* bb = static_cast<const W*>(b);
  TO* yy = static_cast<TO*>(y);
  const int c = static_cast<int>(cols);
  if (aligned && vpt <= 1) {
    ln_fwd_reg<T, W, 1, TO><<<grid, 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && vpt <= 2) {
    ln_fwd_reg<T, W, 2, TO><<<grid, 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && vpt <= 4) {
    ln_fwd_reg<T, W, 4, TO><<<grid, 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && vpt <= 8) {
    ln_fwd_reg<T, W, 8, TO><<<grid, 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && ln_wide_vb(cols / N) == 3) {
    ln_fwd_wide<T, W, 3, TO><<<static_cast<int>(rows), 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && ln_wide_vb(cols / N) == 4) {
    ln_fwd_wide<T, W, 4, TO><<<static_cast<int>(rows), 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else if (aligned && ln_wide_vb(cols / N) == 6) {
    ln_fwd_wide<T, W, 6, TO><<<static_cast<int>(rows), 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps, drop);
  } else {
    ln_fwd_stream<T, W, TO><<<static_cast<int>(rows), 256, 0, s>>>(xx, rr, xo, ww, bb, yy, mean, rstd, rows, c, eps,
                                                                   drop);
  }
}
}  // namespace

int layernorm_fwd(int dt, const void* x, const void* residual, void* x_out, int wdt, const void* w, const void* b,
                  void* y, float* mean, float* rstd, int64_t rows, int64_t cols, float eps, hipStream_t s,
                  const DropoutArgs& drop, int out_dt) {
  if (rows <= 0) return 0;
  if (out_dt >= 0 && out_dt != dt && out_dt != wdt) return -3;  // output: input or parameter dtype
  const bool mixed = out_dt >= 0 && out_dt != dt;
  SMPK_DISPATCH(dt, T, {
    SMPK_DISPATCH(wdt, W, {
      if (mixed)
        launch_ln_fwd<T, W, W>(x, residual, x_out, w, b, y, mean, rstd, rows, cols, eps, s, drop);
      else
        launch_ln_fwd<T, W, T>(x, residual, x_out, w, b, y, mean, rstd, rows, cols, eps, s, drop);
    });
  });
  return static_cast<int>(hipGetLastError());
}

// Number of partial rows the backward will produce for (rows, cols): callers size
// dw_part/db_part as [parts, cols] fp32.
// Cap on the partial rows (= backward workgroups) of the register paths; more workgroups keep
// more rows in flight per CU (the block-per-rows kernel streams its rows one at a time behind a
// barrier) at the price of a larger dgamma/dbeta partial reduction.  1024: in the GPT-2 XL
// step's kernel trace the block-per-rows kernel takes 176 us at 1024 partial rows and 191 us at
// 1792 (bench-level A/B of 1024 / 1792 / 3584 was within the box's +-1 % noise).
constexpr int64_t kLnBwdPartsCap = 1024;
static inline int64_t ln_bwd_parts_cap() { return kLnBwdPartsCap; }

static inline int ln_bwd_parts(int64_t rows, int64_t cols, bool reg_path) {
  if (!reg_path) return static_cast<int>(rows);
  int64_t blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  if (blocks > ln_bwd_parts_cap()) blocks = ln_bwd_parts_cap();
  return static_cast<int>(blocks);
}

int layernorm_bwd(int dt, const void* dy, const void* x, int wdt, const void* w, const float* mean, const float* rstd,
                  void* dx, float* dw_part, float* db_part, int64_t rows, int64_t cols, int part_rows,
                  const void* dres, hipStream_t s, const float* ext_sums, float ext_n, void* dxd,
                  const DropoutArgs* drop) {
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    SMPK_DISPATCH(wdt, W, {
      constexpr int N = Vec16<T>::N;
      const bool aligned = (cols % N == 0) && vec_ok<T>(x) && vec_ok<T>(dy) && vec_ok<T>(dx) && vec_ok<W>(w) &&
                           (dres == nullptr || vec_ok<T>(dres));
      const int vpt = static_cast<int>((cols + 64 * N - 1) / (64 * N));
      const bool reg = aligned && vpt <= 8;
      const int wide = aligned ? ln_wide_vb(cols / N) : 0;
      const int parts = ln_bwd_parts(rows, cols, reg || wide > 0);
      if (part_rows != parts) return -2;  // caller must size partials with layernorm_bwd_parts
      const T* dyy = static_cast<const T*>(dy);
      const T* xx = static_cast<const T*>(x);
      const W* ww = static_cast<const W*>(w);
      T* dxx = static_cast<T*>(dx);
      const T* dr = static_cast<const T*>(dres);
      const int c = static_cast<int>(cols);
      const size_t lds = static_cast<size_t>(2 * kRowsPerBlock) * cols * sizeof(float);
      const int64_t nvec = cols / N;
      const int64_t rpb = (rows + parts - 1) / parts;
      const bool blk_ok = ext_sums == nullptr;  // the block-per-rows form has no external-sum mode
      T* dxdd = static_cast<T*>(dxd);
      const DropoutArgs dd = drop != nullptr ? *drop : DropoutArgs{};
      const bool blk1 = blk_ok && reg && nvec <= 256 && nvec >= 128, blk2 = blk_ok && reg && nvec <= 512 && nvec > 256;
      if (dxd != nullptr && !(blk1 || blk2)) return -4;  // fused dropout output: block kernels only
      if (blk1) {
        ln_bwd_blk<T, W, 1><<<parts, 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, rpb, dxdd,
                                                  dd);
      } else if (blk2) {
        ln_bwd_blk<T, W, 2><<<parts, 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, rpb, dxdd,
                                                  dd);
      } else if (reg && vpt <= 1) {
        ln_bwd_reg<T, W, 1><<<parts, 256, lds, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, ext_sums, ext_n);
      } else if (reg && vpt <= 2) {
        ln_bwd_reg<T, W, 2><<<parts, 256, lds, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, ext_sums, ext_n);
      } else if (reg && vpt <= 4) {
        ln_bwd_reg<T, W, 4><<<parts, 256, lds, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, ext_sums, ext_n);
      } else if (reg) {
        ln_bwd_reg<T, W, 8><<<parts, 256, lds, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, ext_sums, ext_n);
      } else if (wide == 3) {
        ln_bwd_wide<T, W, 3><<<parts, 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, rpb,
                                                   ext_sums, ext_n);
      } else if (wide == 4) {
        ln_bwd_wide<T, W, 4><<<parts, 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, rpb,
                                                   ext_sums, ext_n);
      } else if (wide == 6) {
        ln_bwd_wide<T, W, 6><<<parts, 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part, rows, c, dr, rpb,
                                                   ext_sums, ext_n);
      } else {
        ln_bwd_stream<T, W><<<static_cast<int>(rows), 256, 0, s>>>(dyy, xx, ww, mean, rstd, dxx, dw_part, db_part,
                                                                   rows, c, dr, ext_sums, ext_n);
      }
    });
  });
  return static_cast<int>(hipGetLastError());
}

int layernorm_bwd_reduce(int wdt, const float* dw_part, const float* db_part, void* dw, void* db, int parts,
                         int64_t cols, float* work, hipStream_t s, bool accumulate) {
  // work: [kLnReduceSlices][2][cols] fp32
  const int slices = parts < kLnReduceSlices ? parts : kLnReduceSlices;
  dim3 g1(static_cast<unsigned>((cols + 63) / 64), static_cast<unsigned>(slices));
  ln_bwd_reduce_stage1<<<g1, 256, 0, s>>>(dw_part, db_part, work, parts, cols, slices);
  SMPK_DISPATCH(wdt, W, {
    ln_bwd_reduce_stage2<W><<<static_cast<int>((cols + 255) / 256), 256, 0, s>>>(
        work, static_cast<W*>(dw), static_cast<W*>(db), cols, slices, accumulate);
  });
  return static_cast<int>(hipGetLastError());
}

int layernorm_apply_stats(int dt, const void* x, int wdt, const void* w, const void* b, const float* mean,
                          const float* var, void* y, float* rstd, int64_t rows, int64_t cols, float eps,
                          hipStream_t s) {
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    SMPK_DISPATCH(wdt, W, {
      ln_apply_stats<T, W><<<static_cast<int>(rows), 256, 0, s>>>(
          static_cast<const T*>(x), static_cast<const W*>(w), static_cast<const W*>(b), mean, var, static_cast<T*>(y),
          rstd, rows, static_cast<int>(cols), eps);
    });
  });
  return static_cast<int>(hipGetLastError());
}

namespace {

// one wave per row, strided over the local shard (any width); two passes over x (local mean,
// then M2 about it) -- exact, and the values stay in L2 between the passes
template <typename T>
__global__ void __launch_bounds__(256) ln_local_stats_kernel(const T* __restrict__ x, float* __restrict__ out,
                                                             int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * cols;
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += to_f32(xr[c]);
  s = wave_sum(s);
  const float m = s / cols;
  float m2 = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float d = to_f32(xr[c]) - m;
    m2 += d * d;
  }
  m2 = wave_sum(m2);
  if (lane == 0) {
    out[3 * row] = s;
    out[3 * row + 1] = m2;
    out[3 * row + 2] = s * m;
  }
}

template <typename T, typename W>
__global__ void __launch_bounds__(256) ln_bwd_local_sums_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                const W* __restrict__ w,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                float* __restrict__ out, int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float mu = mean[row], rs = rstd[row];
  float a = 0.f, b = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float g = to_f32(dy[row * cols + c]) * (w ? to_f32(w[c]) : 1.f);
    a += g;
    b += g * (to_f32(x[row * cols + c]) - mu) * rs;
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    out[2 * row] = a;
    out[2 * row + 1] = b;
  }
}

}  // namespace

int layernorm_local_stats(int dt, const void* x, float* stats3, int64_t rows, int64_t cols, hipStream_t s) {
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    ln_local_stats_kernel<T><<<static_cast<int>((rows + kRowsPerBlock - 1) / kRowsPerBlock), 256, 0, s>>>(
        static_cast<const T*>(x), stats3, rows, static_cast<int>(cols));
  });
  return static_cast<int>(hipGetLastError());
}

int layernorm_bwd_local_sums(int dt, const void* dy, const void* x, int wdt, const void* w, const float* mean,
                             const float* rstd, float* sums2, int64_t rows, int64_t cols, hipStream_t s) {
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    SMPK_DISPATCH(wdt, W, {
      ln_bwd_local_sums_kernel<T, W><<<static_cast<int>((rows + kRowsPerBlock - 1) / kRowsPerBlock), 256, 0, s>>>(
          static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const W*>(w), mean, rstd, sums2, rows,
          static_cast<int>(cols));
    });
  });
  return static_cast<int>(hipGetLastError());
}

// exported helper so bindings can size partial buffers
bool layernorm_bwd_dropout_fusable(int dt, int64_t cols, bool aligned) {
  const int N = dt == F32 ? 4 : 8;
  if (!aligned || cols % N != 0) return false;
  const int64_t nvec = cols / N, vpt = (cols + 64 * N - 1) / (64 * N);
  return vpt <= 8 && nvec >= 128 && nvec <= 512;
}

int layernorm_bwd_num_parts(int dt, int64_t rows, int64_t cols, bool aligned) {
  const int N = dt == F32 ? 4 : 8;
  const int vpt = static_cast<int>((cols + 64 * N - 1) / (64 * N));
  const bool ok = aligned && (cols % N == 0);
  return ln_bwd_parts(rows, cols, ok && (vpt <= 8 || ln_wide_vb(cols / N) > 0));
}

}  // namespace smpk
