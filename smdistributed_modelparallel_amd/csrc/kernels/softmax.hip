// Fused scaled (masked / causal) softmax forward and backward (K1-K4 of SURVEY §2.6;
// reference ops `scaled_masked_softmax_*`, `scaled_upper_triang_softmax_*`).
//
// One wave64 per row with the row held in registers (16-byte vectors), max and sum by
// wave reductions -- x is read once and y written once.  The reference kernel is capped
// at sk <= 2048 (`transformer.py:101`); the register path here covers sk <= 8192 and a
// block-per-row streaming kernel covers anything larger.  The causal variant never loads
// the masked upper triangle (half the reads).
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

constexpr int kRows = 4;  // rows (waves) per 256-thread block

template <typename T, int VPT, int MODE>  // MODE 0: mask, 1: causal, 2: none
__global__ void __launch_bounds__(256) softmax_fwd_reg(const T* __restrict__ x, const uint8_t* __restrict__ mask,
                                                       T* __restrict__ y, int64_t rows, int64_t heads, int64_t sq,
                                                       int64_t sk, int64_t mask_batch, float scale) {
  constexpr int N = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRows + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t i = row % sq;              // query index
  const int64_t bh = row / sq;             // b * heads + h
  const int64_t b = bh / heads;
  int64_t limit = sk;                      // causal: keys [0, i + sk - sq]
  if (MODE == 1) limit = i + (sk - sq) + 1;
  const T* xr = x + row * sk;
  const uint8_t* mr = (MODE == 0) ? mask + ((b % mask_batch) * sq + i) * sk : nullptr;
  float v[VPT][N];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t c = (static_cast<int64_t>(k) * 64 + lane) * N;
    if (c < limit) {
      Vec16<T> a = load16(xr + c);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        float t = to_f32(a.v[j]) * scale;
        if (MODE == 0 && mr[c + j]) t = -INFINITY;
        if (MODE == 1 && c + j >= limit) t = -INFINITY;
        v[k][j] = t;
        mx = fmaxf(mx, t);
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) v[k][j] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float e = (mx == -INFINITY) ? 0.f : __expf(v[k][j] - mx);
      v[k][j] = e;
      sum += e;
    }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t c = (static_cast<int64_t>(k) * 64 + lane) * N;
    if (c < sk) {
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) o.v[j] = from_f32<T>(v[k][j] * inv);
      store16(y + row * sk + c, o);
    }
  }
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) softmax_fwd_stream(const T* __restrict__ x, const uint8_t* __restrict__ mask,
                                                          T* __restrict__ y, int64_t rows, int64_t heads, int64_t sq,
                                                          int64_t sk, int64_t mask_batch, float scale) {
  __shared__ float smem[16];
  const int64_t row = blockIdx.x;
  const int64_t i = row % sq, b = (row / sq) / heads;
  int64_t limit = MODE == 1 ? i + (sk - sq) + 1 : sk;
  const T* xr = x + row * sk;
  const uint8_t* mr = (MODE == 0) ? mask + ((b % mask_batch) * sq + i) * sk : nullptr;
  auto val = [&](int64_t c) -> float {
    if (c >= limit) return -INFINITY;
    if (MODE == 0 && mr[c]) return -INFINITY;
    return to_f32(xr[c]) * scale;
  };
  float mx = -INFINITY;
  for (int64_t c = threadIdx.x; c < sk; c += blockDim.x) mx = fmaxf(mx, val(c));
  mx = block_max(mx, smem);
  float sum = 0.f;
  for (int64_t c = threadIdx.x; c < sk; c += blockDim.x) sum += mx == -INFINITY ? 0.f : __expf(val(c) - mx);
  sum = block_sum(sum, smem);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int64_t c = threadIdx.x; c < sk; c += blockDim.x)
    y[row * sk + c] = from_f32<T>(mx == -INFINITY ? 0.f : __expf(val(c) - mx) * inv);
}

template <typename T, int VPT>
__global__ void __launch_bounds__(256) softmax_bwd_reg(const T* __restrict__ dy, const T* __restrict__ y,
                                                       T* __restrict__ dx, int64_t rows, int64_t cols, float scale) {
  constexpr int N = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRows + (threadIdx.x >> 6);
  if (row >= rows) return;
  float yv[VPT][N], g[VPT][N];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t c = (static_cast<int64_t>(k) * 64 + lane) * N;
    if (c < cols) {
      Vec16<T> a = load16(y + row * cols + c);
      Vec16<T> d = load16(dy + row * cols + c);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        yv[k][j] = to_f32(a.v[j]);
        g[k][j] = to_f32(d.v[j]);
        dot += yv[k][j] * g[k][j];
      }
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t c = (static_cast<int64_t>(k) * 64 + lane) * N;
    if (c < cols) {
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < N; ++j) o.v[j] = from_f32<T>(scale * yv[k][j] * (g[k][j] - dot));
      store16(dx + row * cols + c, o);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_stream(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dx, int64_t rows, int64_t cols, float scale) {
  __shared__ float smem[16];
  const int64_t row = blockIdx.x;
  float dot = 0.f;
  for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) dot += to_f32(y[row * cols + c]) * to_f32(dy[row * cols + c]);
  dot = block_sum(dot, smem);
  for (int64_t c = threadIdx.x; c < cols; c += blockDim.x)
    dx[row * cols + c] = from_f32<T>(scale * to_f32(y[row * cols + c]) * (to_f32(dy[row * cols + c]) - dot));
}

template <typename T, int MODE>
int launch_fwd(const void* x, const uint8_t* mask, void* y, int64_t rows, int64_t heads, int64_t sq, int64_t sk,
               int64_t mask_batch, float scale, hipStream_t s) {
  constexpr int N = Vec16<T>::N;
  const bool aligned = (sk % N == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  const int64_t vpt = (sk + 64 * N - 1) / (64 * N);
  const int grid = static_cast<int>((rows + kRows - 1) / kRows);
  const T* xx = static_cast<const T*>(x);
  T* yy = static_cast<T*>(y);
#define SMPK_SM_CASE(V)                                                                                   \
  if (aligned && vpt <= V) {                                                                              \
    softmax_fwd_reg<T, V, MODE><<<grid, 256, 0, s>>>(xx, mask, yy, rows, heads, sq, sk, mask_batch, scale); \
    return static_cast<int>(hipGetLastError());                                                           \
  }
  SMPK_SM_CASE(1)
  SMPK_SM_CASE(2)
  SMPK_SM_CASE(4)
  SMPK_SM_CASE(8)
  SMPK_SM_CASE(16)
#undef SMPK_SM_CASE
  softmax_fwd_stream<T, MODE><<<static_cast<int>(rows), 256, 0, s>>>(xx, mask, yy, rows, heads, sq, sk, mask_batch,
                                                                     scale);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int scaled_masked_softmax_fwd(int dt, const void* x, const uint8_t* mask, void* y, int64_t batch, int64_t heads,
                              int64_t sq, int64_t sk, int64_t mask_batch, float scale, hipStream_t s) {
  const int64_t rows = batch * heads * sq;
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    if (mask != nullptr) return launch_fwd<T, 0>(x, mask, y, rows, heads, sq, sk, mask_batch, scale, s);
    return launch_fwd<T, 2>(x, nullptr, y, rows, heads, sq, sk, 1, scale, s);
  });
  return 0;
}

int scaled_upper_triang_softmax_fwd(int dt, const void* x, void* y, int64_t attn_batches, int64_t sq, int64_t sk,
                                    float scale, hipStream_t s) {
  const int64_t rows = attn_batches * sq;
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, { return launch_fwd<T, 1>(x, nullptr, y, rows, 1, sq, sk, 1, scale, s); });
  return 0;
}

int scaled_softmax_bwd(int dt, const void* dy, const void* y, void* dx, int64_t rows, int64_t cols, float scale,
                       hipStream_t s) {
  if (rows <= 0) return 0;
  SMPK_DISPATCH(dt, T, {
    constexpr int N = Vec16<T>::N;
    const bool aligned = (cols % N == 0) && ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(y) |
                                              reinterpret_cast<uintptr_t>(dx)) & 15) == 0;
    const int64_t vpt = (cols + 64 * N - 1) / (64 * N);
    const int grid = static_cast<int>((rows + kRows - 1) / kRows);
    const T* d = static_cast<const T*>(dy);
    const T* yy = static_cast<const T*>(y);
    T* o = static_cast<T*>(dx);
    if (aligned && vpt <= 1) softmax_bwd_reg<T, 1><<<grid, 256, 0, s>>>(d, yy, o, rows, cols, scale);
    else if (aligned && vpt <= 2) softmax_bwd_reg<T, 2><<<grid, 256, 0, s>>>(d, yy, o, rows, cols, scale);
    else if (aligned && vpt <= 4) softmax_bwd_reg<T, 4><<<grid, 256, 0, s>>>(d, yy, o, rows, cols, scale);
    else if (aligned && vpt <= 8) softmax_bwd_reg<T, 8><<<grid, 256, 0, s>>>(d, yy, o, rows, cols, scale);
    else if (aligned && vpt <= 16) softmax_bwd_reg<T, 16><<<grid, 256, 0, s>>>(d, yy, o, rows, cols, scale);
    else softmax_bwd_stream<T><<<static_cast<int>(rows), 256, 0, s>>>(d, yy, o, rows, cols, scale);
  });
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
