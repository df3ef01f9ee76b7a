// 2-D transpose through LDS (dst[C][R] = src[R][C]) for the cached W^T copies of
// `ops/linear.py` (input-gradient GEMMs in the forward layout).  A 64x64 tile per
// 256-thread block: 16-byte vector loads along the source rows into a padded LDS tile,
// 16-byte vector stores along the destination rows; the padding (+2 elements per row)
// spreads the column reads over the LDS banks.  Ragged edges fall back to scalar
// accesses.  Memory-bound: one read + one write of the matrix.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

constexpr int kTile = 64;

template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(const T* __restrict__ src, T* __restrict__ dst, int64_t R,
                                                        int64_t C, bool vec_ok) {
  constexpr int N = Vec16<T>::N;             // elements per 16-byte vector
  constexpr int VPR = kTile / N;             // vectors per tile row
  constexpr int RPP = 256 / VPR;             // tile rows per pass
  __shared__ T tile[kTile][kTile + 2];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kTile, c0 = static_cast<int64_t>(blockIdx.x) * kTile;
  const int tx = threadIdx.x % VPR, ty = threadIdx.x / VPR;
  const bool full = vec_ok && r0 + kTile <= R && c0 + kTile <= C;
#pragma unroll
  for (int i = 0; i < kTile / RPP; ++i) {
    const int r = ty + RPP * i;
    const int64_t gr = r0 + r, gc = c0 + tx * N;
    if (full) {
      Vec16<T> v = load16(src + gr * C + gc);
#pragma unroll
      for (int j = 0; j < N; ++j) tile[r][tx * N + j] = v.v[j];
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (gr < R && gc + j < C) tile[r][tx * N + j] = src[gr * C + gc + j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kTile / RPP; ++i) {
    const int c = ty + RPP * i;                    // destination row within the tile
    const int64_t dr = c0 + c, dc = r0 + tx * N;  // destination (row, first column)
    if (full) {
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) o.v[j] = tile[tx * N + j][c];
      store16(dst + dr * R + dc, o);
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (dr < C && dc + j < R) dst[dr * R + dc + j] = tile[tx * N + j][c];
    }
  }
}

}  // namespace

int transpose2d(int dt, const void* src, void* dst, int64_t rows, int64_t cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  dim3 g(static_cast<unsigned>((cols + kTile - 1) / kTile), static_cast<unsigned>((rows + kTile - 1) / kTile));
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool vec_ok = (cols % N == 0) && (rows % N == 0) &&
                        ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    transpose_kernel<T><<<g, 256, 0, s>>>(static_cast<const T*>(src), static_cast<T*>(dst), rows, cols, vec_ok);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
