// Throughput of the dropout-hash building blocks on one MI355X: v_mul_lo_u32 vs
// v_mul_u32_u24 / v_mul_hi_u32_u24 chains, and the full lowbias32 mixer vs a 24-bit-multiply
// mixer.  8 independent chains per lane, 2 waves per SIMD (grid = 256 CUs x 8 waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return (a & 0xffffffu) * (b & 0xffffffu); }
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
  return static_cast<uint32_t>((static_cast<uint64_t>(a & 0xffffffu) * (b & 0xffffffu)) >> 32);
}
__device__ __forceinline__ uint32_t mix24(uint32_t x) {
  x ^= x >> 16;
  x = mul24(x, 0x352d7fu) ^ mulhi24(x, 0xeb352du) ^ (x & 0xff000000u);
  x ^= x >> 15;
  x = mul24(x, 0x6ca68bu) ^ mulhi24(x, 0x846ca6u) ^ (x & 0xff000000u);
  x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(512) void k(uint32_t* out, int iters) {
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 8 + i + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (MODE == 0) v[i] = v[i] * 0x7feb352du;
      else if constexpr (MODE == 1) v[i] = mul24(v[i], 0x352d7fu);
      else if constexpr (MODE == 2) v[i] = v[i] ^ (v[i] >> 15);
      else if constexpr (MODE == 3) v[i] = mix32(v[i]);
      else v[i] = mix24(v[i]);
    }
  }
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a ^= v[i];
  out[blockIdx.x * 512 + threadIdx.x] = a;
}

template <int MODE>
float run(uint32_t* out, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  k<MODE><<<256 * 4, 512>>>(out, iters);
  hipEventRecord(a);
  k<MODE><<<256 * 4, 512>>>(out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  uint32_t* out; hipMalloc(&out, 256 * 4 * 512 * 4);
  const int iters = 4096;
  const char* names[] = {"v_mul_lo_u32", "v_mul_u32_u24", "xor-shift", "lowbias32 mix", "24-bit mix"};
  float t[5] = {run<0>(out, iters), run<1>(out, iters), run<2>(out, iters), run<3>(out, iters), run<4>(out, iters)};
  // per-op cost in SIMD cycles at ~2.1-2.4 GHz: waves per SIMD = 1024*8/(256*4) = 8
  for (int i = 0; i < 5; ++i) {
    const double ops = 256.0 * 4 * 512 * iters * 8;  // lane-ops
    printf("%-16s %.3f ms  %.1f Gops/s (lane)\n", names[i], t[i], ops / t[i] / 1e6);
  }
  hipFree(out);
  return 0;
}
