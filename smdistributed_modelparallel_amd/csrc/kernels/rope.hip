// Rotary position embeddings (K18 of SURVEY §2.6; the reference applies RoPE with torch
// ops, `smp/torch/nn/transformer.py:114-182,1565-1615`).
//
// y = rope(x) for x [b, s, h, d] with arbitrary (b, s, h) strides (e.g. q/k views into the
// packed QKV projection) and contiguous d; y is written contiguous [b, s, h, d].  Only the
// first rotary_dim channels rotate; the rest are copied.  style 0 = GPT-J (interleaved
// pairs 2i, 2i+1), 1 = GPT-NeoX (pairs i, i + rotary_dim/2).  `inverse` rotates by -theta
// (the backward).  cos/sin come from fp32 tables [positions, rotary_dim/2].
//
// Layout: one 64-lane wave per (b, s, h) row, 4 rows per 256-thread block; each lane
// handles channel pairs so every pair is read once and written once (HBM-bound).
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

template <typename T>
__global__ void __launch_bounds__(256) rope_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                   const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                   int64_t rows, int64_t s_len, int64_t h, int d, int rd,
                                                   int64_t sb, int64_t ss, int64_t sh, int style, int inverse,
                                                   int64_t pos_offset) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t hh = row % h, bs = row / h, pos = bs % s_len, bb = bs / s_len;
  const T* xr = x + bb * sb + pos * ss + hh * sh;
  T* yr = y + row * d;
  const float* cr = cos_t + (pos + pos_offset) * (rd / 2);
  const float* sr = sin_t + (pos + pos_offset) * (rd / 2);
  const float sgn = inverse ? -1.f : 1.f;
  const int half = rd / 2;
  for (int p = lane; p < half; p += 64) {
    const int i0 = style == 0 ? 2 * p : p;
    const int i1 = style == 0 ? 2 * p + 1 : p + half;
    const float a = to_f32(xr[i0]), b = to_f32(xr[i1]);
    const float c = cr[p], sn = sgn * sr[p];
    yr[i0] = from_f32<T>(a * c - b * sn);
    yr[i1] = from_f32<T>(b * c + a * sn);
  }
  for (int i = rd + lane; i < d; i += 64) yr[i] = xr[i];
}

}  // namespace

int rope_apply(int dt, const void* x, void* y, const float* cos_t, const float* sin_t, int64_t b, int64_t s_len,
               int64_t h, int64_t d, int64_t rotary_dim, int64_t stride_b, int64_t stride_s, int64_t stride_h,
               int style, int inverse, int64_t pos_offset, hipStream_t s) {
  const int64_t rows = b * s_len * h;
  if (rows <= 0) return 0;
  if (rotary_dim % 2 != 0 || rotary_dim > d) return -2;
  SMPK_DISPATCH(dt, T, {
    rope_kernel<T><<<static_cast<unsigned>((rows + 3) / 4), 256, 0, s>>>(
        static_cast<const T*>(x), static_cast<T*>(y), cos_t, sin_t, rows, s_len, h, static_cast<int>(d),
        static_cast<int>(rotary_dim), stride_b, stride_s, stride_h, style, inverse, pos_offset);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
