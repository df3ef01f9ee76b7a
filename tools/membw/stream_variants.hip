// HBM streaming micro-benchmark: which access pattern reaches the MI355X HBM rate for the
// elementwise kernels (y = x * a + b over bf16 [rows, cols]).  Variants:
//   gs     grid-stride loop, 2048 blocks x 256 threads, U 16-byte vectors in flight per lane
//   once   one pass: each lane handles U consecutive-stride vectors, grid = n / (256 U)
//   *_nt   same with non-temporal (streaming) stores
//   *_ntl  non-temporal loads and stores
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_variants stream_variants.hip
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 op(u32x4 v) {
  // bf16 pairs: x * 1.0078125 + 0 via float (keeps the VALU cost of a real elementwise op small)
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(v[i] << 16), hi = __uint_as_float(v[i] & 0xffff0000u);
    const float a = lo * 1.0078125f, b = hi * 1.0078125f;
    o[i] = (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xffff0000u);
  }
  return o;
}

template <int U, bool NTS, bool NTL>
__global__ void __launch_bounds__(256) k_gs(const u32x4* __restrict__ x, u32x4* __restrict__ y, long n) {
  const long stride = (long)gridDim.x * 256;
  long v = (long)blockIdx.x * 256 + threadIdx.x;
  for (; v + (U - 1) * stride < n; v += U * stride) {
    u32x4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = NTL ? __builtin_nontemporal_load(x + v + u * stride) : x[v + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS)
        __builtin_nontemporal_store(op(a[u]), y + v + u * stride);
      else
        y[v + u * stride] = op(a[u]);
    }
  }
  for (; v < n; v += stride) y[v] = op(x[v]);
}

template <int U, bool NTS, bool NTL>
__global__ void __launch_bounds__(256) k_once(const u32x4* __restrict__ x, u32x4* __restrict__ y, long n) {
  // block b covers vectors [b * 256 U, (b + 1) * 256 U): lane t takes t + 256 u
  const long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + 256 * u;
    if (i < n) a[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + 256 * u;
    if (i < n) {
      if (NTS)
        __builtin_nontemporal_store(op(a[u]), y + i);
      else
        y[i] = op(a[u]);
    }
  }
}

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("error %s at %d\n", hipGetErrorString(e), __LINE__);    \
      exit(1);                                                       \
    }                                                                \
  } while (0)

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a));
  const int it = 20;
  for (int i = 0; i < it; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / it;
}

int main() {
  const long shapes[2][2] = {{65536, 1600}, {65536, 6400}};
  for (auto& sh : shapes) {
    const long elems = sh[0] * sh[1];
    const long n = elems / 8;  // 16-byte vectors
    u32x4 *x, *y;
    CK(hipMalloc(&x, n * 16));
    CK(hipMalloc(&y, n * 16));
    CK(hipMemset(x, 0x3c, n * 16));
    const double bytes = 2.0 * n * 16;
    auto rep = [&](const char* name, float ms) {
      printf("{\"shape\": \"%ldx%ld\", \"variant\": \"%s\", \"us\": %.1f, \"TBps\": %.2f}\n", sh[0], sh[1], name, ms * 1e3,
             bytes / ms / 1e9);
    };
    rep("hipMemcpy", timeit([&] { CK(hipMemcpyAsync(y, x, n * 16, hipMemcpyDeviceToDevice, 0)); }));
    for (int g : {1024, 2048, 4096}) {
      char nm[64];
      snprintf(nm, sizeof nm, "gs_u4_g%d", g);
      rep(nm, timeit([&] { k_gs<4, false, false><<<g, 256>>>(x, y, n); }));
      snprintf(nm, sizeof nm, "gs_u4_g%d_nt", g);
      rep(nm, timeit([&] { k_gs<4, true, false><<<g, 256>>>(x, y, n); }));
    }
    rep("gs_u2_g2048", timeit([&] { k_gs<2, false, false><<<2048, 256>>>(x, y, n); }));
    rep("gs_u8_g2048", timeit([&] { k_gs<8, false, false><<<2048, 256>>>(x, y, n); }));
    rep("gs_u4_g2048_ntl", timeit([&] { k_gs<4, true, true><<<2048, 256>>>(x, y, n); }));
    for (int u : {1, 2, 4, 8}) {
      char nm[64];
      const unsigned grid = (unsigned)((n + 256L * u - 1) / (256L * u));
      snprintf(nm, sizeof nm, "once_u%d", u);
      switch (u) {
        case 1: rep(nm, timeit([&] { k_once<1, false, false><<<grid, 256>>>(x, y, n); })); break;
        case 2: rep(nm, timeit([&] { k_once<2, false, false><<<grid, 256>>>(x, y, n); })); break;
        case 4: rep(nm, timeit([&] { k_once<4, false, false><<<grid, 256>>>(x, y, n); })); break;
        default: rep(nm, timeit([&] { k_once<8, false, false><<<grid, 256>>>(x, y, n); })); break;
      }
      snprintf(nm, sizeof nm, "once_u%d_nt", u);
      switch (u) {
        case 1: rep(nm, timeit([&] { k_once<1, true, false><<<grid, 256>>>(x, y, n); })); break;
        case 2: rep(nm, timeit([&] { k_once<2, true, false><<<grid, 256>>>(x, y, n); })); break;
        case 4: rep(nm, timeit([&] { k_once<4, true, false><<<grid, 256>>>(x, y, n); })); break;
        default: rep(nm, timeit([&] { k_once<8, true, false><<<grid, 256>>>(x, y, n); })); break;
      }
    }
    CK(hipFree(x));
    CK(hipFree(y));
  }
  return 0;
}
