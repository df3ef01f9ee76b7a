// Rotary position embeddings (K18 of SURVEY §2.6; the reference applies RoPE with torch
// ops, `smp/torch/nn/transformer.py:114-182,1565-1615`).
//
// y = rope(x) for x [b, s, h, d] with arbitrary (b, s, h) strides (e.g. q/k views into the
// packed QKV projection) and contiguous d; y has its own (b, s, h) strides (contiguous, or a
// slice of a packed [b, s, 3, h, d] buffer; y may alias x: every element pair is read and
// written by one thread, so the rotation can run in place).  Only the
// first rotary_dim channels rotate; the rest are copied (copy_rest = 0 leaves them alone: the
// in-place form then reads and writes the rotary channels only).  style 0 = GPT-J (interleaved
// pairs 2i, 2i+1), 1 = GPT-NeoX (pairs i, i + rotary_dim/2).  `inverse` rotates by -theta
// (the backward).  cos/sin come from fp32 tables [positions, rotary_dim/2].
//
// Layout (general / fp32 fallback): one 64-lane wave per (b, s, h) row, 4 rows per 256-thread
// block; each lane handles channel pairs so every pair is read once and written once.  16-bit
// types with aligned rows take the vector kernel below.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

template <typename T>
__global__ void __launch_bounds__(256) rope_kernel(const T* x, T* y, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, int64_t rows, int64_t s_len,
                                                   int64_t h, int d, int rd, int64_t sb, int64_t ss, int64_t sh,
                                                   int64_t yb, int64_t ys, int64_t yh, int style, int inverse,
                                                   int64_t pos_offset, int copy_rest) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t hh = row % h, bs = row / h, pos = bs % s_len, bb = bs / s_len;
  const T* xr = x + bb * sb + pos * ss + hh * sh;
  T* yr = y + bb * yb + pos * ys + hh * yh;
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
  if (copy_rest)
    for (int i = rd + lane; i < d; i += 64) yr[i] = xr[i];
}

// Vector path: one thread per VEC-element chunk of a row (VEC = 8: 16-byte accesses, VEC = 4:
// 8-byte), consecutive threads on consecutive chunks, so a wave moves 512 / 256 contiguous bytes
// per access instead of the scalar kernel's 2-byte lanes (which ran the GPT-J shape at ~2.5 TB/s,
// profiles/r5/fused_ops_counters.md).  GPT-J pairs (2i, 2i + 1) lie inside a chunk; NeoX pairs
// (i, i + rd/2) pair chunk c with chunk c + rd/(2 VEC), so the first-half lanes do both and the
// second-half lanes return.  Needs d % VEC == 0, rd % (2 VEC) == 0, VEC-aligned rows.
template <int VEC>
struct VecT;
template <>
struct VecT<8> {
  typedef uint4 U;
};
template <>
struct VecT<4> {
  typedef uint2 U;
};

template <typename T, int VEC, int STYLE>
__global__ void __launch_bounds__(256) rope_vec_kernel(const T* x, T* y, const float* __restrict__ cos_t,
                                                       const float* __restrict__ sin_t, int64_t chunks, int cpr,
                                                       int64_t s_len, int64_t h, int rd, int64_t sb, int64_t ss,
                                                       int64_t sh, int64_t yb, int64_t ys, int64_t yh, int inverse,
                                                       int64_t pos_offset) {
  typedef typename VecT<VEC>::U U;
  union Pack {
    U u;
    T v[VEC];
  };
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (g >= chunks) return;
  const int64_t row = g / cpr;
  const int e0 = static_cast<int>(g - row * cpr) * VEC;
  const int64_t hh = row % h, bs = row / h, pos = bs % s_len, bb = bs / s_len;
  const T* xr = x + bb * sb + pos * ss + hh * sh;
  T* yr = y + bb * yb + pos * ys + hh * yh;
  if (e0 >= rd) {  // pass-through channels
    *reinterpret_cast<U*>(yr + e0) = *reinterpret_cast<const U*>(xr + e0);
    return;
  }
  const int half = rd / 2;
  if (STYLE == 1 && e0 >= half) return;  // done by the partner chunk's lane
  const float sgn = inverse ? -1.f : 1.f;
  const float* cr = cos_t + (pos + pos_offset) * half;
  const float* sr = sin_t + (pos + pos_offset) * half;
  if (STYLE == 0) {
    Pack a;
    a.u = *reinterpret_cast<const U*>(xr + e0);
    Pack o;
#pragma unroll
    for (int j = 0; j < VEC / 2; ++j) {
      const float c = cr[e0 / 2 + j], sn = sgn * sr[e0 / 2 + j];
      const float u0 = to_f32(a.v[2 * j]), u1 = to_f32(a.v[2 * j + 1]);
      o.v[2 * j] = from_f32<T>(u0 * c - u1 * sn);
      o.v[2 * j + 1] = from_f32<T>(u1 * c + u0 * sn);
    }
    *reinterpret_cast<U*>(yr + e0) = o.u;
  } else {
    Pack a, b2;
    a.u = *reinterpret_cast<const U*>(xr + e0);
    b2.u = *reinterpret_cast<const U*>(xr + e0 + half);
    Pack o1, o2;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float c = cr[e0 + j], sn = sgn * sr[e0 + j];
      const float u0 = to_f32(a.v[j]), u1 = to_f32(b2.v[j]);
      o1.v[j] = from_f32<T>(u0 * c - u1 * sn);
      o2.v[j] = from_f32<T>(u1 * c + u0 * sn);
    }
    *reinterpret_cast<U*>(yr + e0) = o1.u;
    *reinterpret_cast<U*>(yr + e0 + half) = o2.u;
  }
}

template <typename T, int VEC>
void launch_vec(const void* x, void* y, const float* cos_t, const float* sin_t, int64_t rows, int64_t s_len,
                int64_t h, int64_t d, int64_t rd, int64_t sb, int64_t ss, int64_t sh, int64_t yb, int64_t ys,
                int64_t yh, int style, int inverse, int64_t pos_offset, int copy_rest, hipStream_t s) {
  // without the pass-through copy (in-place rotation) only the rotary chunks get a thread
  const int cpr = static_cast<int>((copy_rest ? d : rd) / VEC);
  const int64_t chunks = rows * cpr;
  const unsigned grid = static_cast<unsigned>((chunks + 255) / 256);
  if (style == 0)
    rope_vec_kernel<T, VEC, 0><<<grid, 256, 0, s>>>(static_cast<const T*>(x), static_cast<T*>(y), cos_t, sin_t, chunks,
                                                    cpr, s_len, h, static_cast<int>(rd), sb, ss, sh, yb, ys, yh, inverse,
                                                    pos_offset);
  else
    rope_vec_kernel<T, VEC, 1><<<grid, 256, 0, s>>>(static_cast<const T*>(x), static_cast<T*>(y), cos_t, sin_t, chunks,
                                                    cpr, s_len, h, static_cast<int>(rd), sb, ss, sh, yb, ys, yh, inverse,
                                                    pos_offset);
}

// the vector path's conditions for VEC elements per access (element size 2)
bool rope_vec_ok(int vec, const void* x, const void* y, int64_t d, int64_t rd, int64_t sb, int64_t ss, int64_t sh,
                 int64_t yb, int64_t ys, int64_t yh) {
  return d % vec == 0 && rd % (2 * vec) == 0 && sb % vec == 0 && ss % vec == 0 && sh % vec == 0 && yb % vec == 0 &&
         ys % vec == 0 && yh % vec == 0 && reinterpret_cast<uintptr_t>(x) % (2 * vec) == 0 &&
         reinterpret_cast<uintptr_t>(y) % (2 * vec) == 0;
}

}  // namespace

int rope_apply(int dt, const void* x, void* y, const float* cos_t, const float* sin_t, int64_t b, int64_t s_len,
               int64_t h, int64_t d, int64_t rotary_dim, int64_t stride_b, int64_t stride_s, int64_t stride_h,
               int64_t y_b, int64_t y_s, int64_t y_h, int style, int inverse, int64_t pos_offset, int copy_rest,
               hipStream_t s) {
  const int64_t rows = b * s_len * h;
  if (rows <= 0) return 0;
  if (rotary_dim % 2 != 0 || rotary_dim > d) return -2;
  if (dt == BF16 || dt == F16) {
    for (int vec : {8, 4}) {
      if (!rope_vec_ok(vec, x, y, d, rotary_dim, stride_b, stride_s, stride_h, y_b, y_s, y_h)) continue;
      if (dt == BF16)
        vec == 8 ? launch_vec<bf16, 8>(x, y, cos_t, sin_t, rows, s_len, h, d, rotary_dim, stride_b, stride_s, stride_h,
                                       y_b, y_s, y_h, style, inverse, pos_offset, copy_rest, s)
                 : launch_vec<bf16, 4>(x, y, cos_t, sin_t, rows, s_len, h, d, rotary_dim, stride_b, stride_s, stride_h,
                                       y_b, y_s, y_h, style, inverse, pos_offset, copy_rest, s);
      else
        vec == 8 ? launch_vec<f16, 8>(x, y, cos_t, sin_t, rows, s_len, h, d, rotary_dim, stride_b, stride_s, stride_h,
                                      y_b, y_s, y_h, style, inverse, pos_offset, copy_rest, s)
                 : launch_vec<f16, 4>(x, y, cos_t, sin_t, rows, s_len, h, d, rotary_dim, stride_b, stride_s, stride_h,
                                      y_b, y_s, y_h, style, inverse, pos_offset, copy_rest, s);
      return static_cast<int>(hipGetLastError());
    }
  }
  SMPK_DISPATCH(dt, T, {
    rope_kernel<T><<<static_cast<unsigned>((rows + 3) / 4), 256, 0, s>>>(
        static_cast<const T*>(x), static_cast<T*>(y), cos_t, sin_t, rows, s_len, h, static_cast<int>(d),
        static_cast<int>(rotary_dim), stride_b, stride_s, stride_h, y_b, y_s, y_h, style, inverse, pos_offset, copy_rest);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
