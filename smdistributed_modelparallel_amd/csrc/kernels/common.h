// Shared device helpers for the CDNA4 (gfx950) kernels.
//
// * wave64 everywhere: reductions use 64-lane shuffles (__shfl_xor over width 64);
// * 16-byte vector loads/stores for bf16/fp16 (8 elements per lane) -- hipcc does not
//   auto-vectorise 16-bit loads (cdna_hip_programming.md Guideline 13);
// * all math in fp32, storage in the tensor dtype.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace smpk {

constexpr int kWave = 64;


typedef __hip_bfloat16 bf16;
typedef __half f16;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(f16 x) { return __half2float(x); }
__device__ __forceinline__ float to_f32(bf16 x) { return __bfloat162float(x); }

template <typename T>
__device__ __forceinline__ T from_f32(float x);
template <>
__device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <>
__device__ __forceinline__ f16 from_f32<f16>(float x) { return __float2half(x); }
template <>
__device__ __forceinline__ bf16 from_f32<bf16>(float x) { return __float2bfloat16(x); }

// 16-byte vector of N elements of T.
template <typename T>
struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  union {
    uint4 raw;
    T v[N];
  };
};

template <typename T>
__device__ __forceinline__ Vec16<T> load16(const T* p) {
  Vec16<T> r;
  r.raw = *reinterpret_cast<const uint4*>(p);
  return r;
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<uint4*>(p) = r.raw;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `smem` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? smem[lane] : 0.f;
  r = wave_sum(r);
  return r;
}
__device__ __forceinline__ float block_max(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? smem[lane] : -INFINITY;
  r = wave_max(r);
  return r;
}

}  // namespace smpk

#define SMPK_CHECK(expr)                                                      \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) return static_cast<int>(_e);                        \
  } while (0)

// Dispatch on the runtime dtype code into a templated launcher.
#define SMPK_DISPATCH(dt, T, ...)                 \
  switch (dt) {                                   \
    case smpk::F32: {                             \
      typedef float T;                            \
      __VA_ARGS__;                                \
      break;                                      \
    }                                             \
    case smpk::F16: {                             \
      typedef smpk::f16 T;                        \
      __VA_ARGS__;                                \
      break;                                      \
    }                                             \
    case smpk::BF16: {                            \
      typedef smpk::bf16 T;                       \
      __VA_ARGS__;                                \
      break;                                      \
    }                                             \
    default:                                      \
      return -1;                                  \
  }
