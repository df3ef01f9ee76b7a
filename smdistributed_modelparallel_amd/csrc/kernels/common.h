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

// ------------------------------------------------------------ element-wise dropout hash
// lowbias32 mixer; a 32-bit hash serves an element PAIR (16-bit uniform each), indexed by
// the flat element index, so any kernel that knows an element's index can regenerate the
// decision (forward fused into LayerNorm / residual add, backward fused into its consumer).
__device__ __forceinline__ uint32_t dmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t dropout_key(const DropoutArgs& d) {
  const uint32_t s0 = static_cast<uint32_t>(d.seed), s1 = static_cast<uint32_t>(d.seed >> 32);
  const uint32_t o0 = static_cast<uint32_t>(d.offset), o1 = static_cast<uint32_t>(d.offset >> 32);
  return dmix32(s0 ^ dmix32(s1 + 0x27d4eb2fu) ^ dmix32(o0 ^ dmix32(o1 + 0x165667b1u)));
}

// keep factors (0 or rs) of the 8 consecutive elements e0..e0+7 (e0 even)
__device__ __forceinline__ void dropout_factors8(uint32_t key, int64_t e0, const DropoutArgs& d, float (&f)[8]) {
  const uint32_t thr16 = d.thr << 16;
  const uint32_t hi = static_cast<uint32_t>(static_cast<uint64_t>(e0) >> 33) * 0x9e3779b1u;
  const uint32_t pr = static_cast<uint32_t>(static_cast<uint64_t>(e0) >> 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t h = dmix32(key ^ hi ^ (pr + j));
    f[2 * j] = (h << 16) >= thr16 ? d.rs : 0.f;
    f[2 * j + 1] = h >= thr16 ? d.rs : 0.f;
  }
}

__device__ __forceinline__ float dropout_factor1(uint32_t key, int64_t e, const DropoutArgs& d) {
  const uint32_t hi = static_cast<uint32_t>(static_cast<uint64_t>(e) >> 33) * 0x9e3779b1u;
  const uint32_t h = dmix32(key ^ hi ^ static_cast<uint32_t>(static_cast<uint64_t>(e) >> 1));
  const uint32_t u = (e & 1) ? (h >> 16) : (h & 0xffffu);
  return u >= d.thr ? d.rs : 0.f;
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

// LDS-DMA: 16 B per lane from `src` into LDS at lds_wave_base + 16 * lane (global_load_lds,
// lane-linear destination, base in M0).  Issued from inline asm: with the builtin, hipcc
// (ROCm 7.2) cannot tell the LDS buffer being filled from the one being read and drains
// vmcnt(0) before the next ds_read -- a prefetch would never overlap compute.  The caller
// waits for it with an explicit s_waitcnt vmcnt before the barrier that publishes the data.
__device__ __forceinline__ void lds_dma16(const void* src, const void* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)lds_wave_base)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

// One dword per lane (a wave writes 256 consecutive LDS bytes at lds_wave_base): small slabs
// that ride with a tile's 16-byte DMA pieces, e.g. the attention forward's dropout keep words.
__device__ __forceinline__ void lds_dma4(const void* src, const void* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)lds_wave_base)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

// Same, saddr form: scalar 64-bit base + 32-bit per-lane byte offset.  Interior tiles use
// this so the only per-lane address term is loop-invariant (no 64-bit row * stride multiply
// and add per load per tile).
__device__ __forceinline__ void lds_dma16_sv(const void* sbase, uint32_t voff_bytes, const void* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)lds_wave_base)));
  const uint64_t b = reinterpret_cast<uint64_t>(sbase);
  // (readfirstlane returns int: widen through uint32_t, or a low word >= 2^31 sign-extends
  // into the high word)
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b >> 32)));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b)));
  const uint64_t sb = (static_cast<uint64_t>(hi) << 32) | static_cast<uint64_t>(lo);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff_bytes), "s"(sb), "s"(lds)
               : "memory", "m0");
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
