// Weight-gradient GEMM for CDNA4 (gfx950):  C[N][K] (+)= sum_t A[t][N] * B[t][K]
// (A = dY [tokens, out], B = X [tokens, in], both row-major; C = dW [out, in]).
//
// Why a hand-written kernel: the reduction runs over the token dimension, which is the
// SLOW (row) dimension of both operands, and the output is small (GPT-2 XL: 1600 x 1600 ..
// 6400 x 1600 for 65 536 tokens).  hipBLASLt runs this "NT" layout at 0.7-0.9 PFLOP/s on
// MI355X (TunableOp-selected, configs/tunableop) against 1.3-1.4 for the K-contiguous
// forward GEMMs of the same size: its row-major-operand kernels transpose through
// registers, and 256 x 256 output tiles give 49-175 workgroups for 256 CUs.
//
// Design:
//  * operands are staged row-major exactly as they sit in HBM (512-B rows, fully
//    coalesced 16-B loads, no transpose kernels) and the MFMA fragments -- which need 8
//    consecutive reduction elements per lane -- come from ds_read_b64_tr_b16, the gfx950
//    LDS transpose read;
//  * v_mfma_f32_32x32x16_bf16 (f16), 256 threads = 4 waves in 2 x 2, each wave owns a
//    128 x 128 output block = 16 accumulator tiles (256 fp32 AGPRs);
//  * 64-token tiles, register-staged (the next tile's global loads are issued before the
//    current tile's 64 MFMAs per wave), one 64 KB LDS buffer with XOR-swizzled 16-B
//    chunks (conflict-free transposed reads); staging registers are native vectors (HIP's
//    uint4 class left them in scratch) and loads are unpredicated (edge chunks re-read a
//    valid chunk) so no vmcnt(0) lands before the MFMAs;
//  * split-K over tokens: the split count is chosen on the host so that the grid fills the
//    256 CUs in whole waves of workgroups (tile count x splits / 256 close to an integer);
//    each split writes an fp32 partial tile and a vectorised reduction adds the partials
//    into the gradient (beta = 1: the gradient buffer accumulates across microbatches, no
//    temporary dW and no separate "grad += dW" pass);
//  * workgroups are dealt to XCDs in contiguous runs of (split, n-tile) so that the
//    workgroups sharing an A strip share one XCD's L2.
//
// Status (MI355X, GPT-2 XL shapes, tools/wgrad_bench.py, profiles/r2/wgrad_kernel.md): the
// register-staged version ran 630-775 TFLOP/s; the LDS-DMA version (wgrad_glds_kernel:
// global_load_lds from inline asm so hipcc does not drain the prefetch before every ds_read,
// two 64 KB stages, one barrier per tile, bijective XCD mapping) 750-900 TFLOP/s against
// hipBLASLt's 700-1030.  ops/linear.py times both per shape on first use and keeps the faster
// (in the GPT-2 XL step: the kernel wins the 1600 x 1600 weight gradient).  A stream-K
// schedule (one persistent workgroup per CU) was slower: workgroups sharing a tile read
// disjoint token ranges, so concurrent workgroups no longer share A / B strips in L2.
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
// native 16-B vector (HIP's uint4 is a class wrapper that SROA leaves in scratch here)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct WMF;
template <>
struct WMF<bf16> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct WMF<f16> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

constexpr int kT = 256;     // threads
constexpr int TM = 256;     // output tile rows (N)
constexpr int TN = 256;     // output tile cols (K)
constexpr int TK = 64;      // tokens per staged tile
constexpr int RW = 256;     // LDS row width (elements) of both staged tiles
constexpr int CH = RW / 8;  // 16-B chunks per row

// XOR swizzle of the 16-B chunks of a 512-B row (row bits 0-3): conflict-free for the
// row-wise stores and the 4-row transposed reads.
__device__ __forceinline__ int swz(int row, int chunk) {
  const int g = ((row & 3) << 2) | ((row >> 2) & 3);
  return row * RW + ((chunk ^ g) << 3);
}

// Staging of one operand tile (TK rows x 256 columns, 8 x 16 B per thread): thread t owns
// chunk t % 32 of rows t / 32 + 8 i.  Chunks past vc re-read the last valid chunk: those
// columns only feed output rows / columns beyond the matrix, which are never written -- so
// the loads are unconditional and stay in flight across the MFMA work (a predicated load
// whose zero-fill shares the destination register forces a vmcnt(0) before it).
constexpr int NR = TK * CH / kT;  // 8 registers per operand

__device__ __forceinline__ void stage_load(u32x4 (&v)[NR], const uint16_t* src, int64_t ld, int vc) {
  const int r0 = threadIdx.x / CH, c0 = threadIdx.x % CH;
  const int c = c0 < vc ? c0 : vc - 1;
  const uint16_t* p = src + static_cast<int64_t>(r0) * ld + c * 8;
#pragma unroll
  for (int i = 0; i < NR; ++i) v[i] = *reinterpret_cast<const u32x4*>(p + static_cast<int64_t>(8 * i) * ld);
}

// rows r0 + 8 i: row bits 0-3 alternate between r0 and r0 + 8, so two swizzled bases
__device__ __forceinline__ void stage_store(const u32x4 (&v)[NR], uint16_t* lds, int lo0, int lo1) {
#pragma unroll
  for (int i = 0; i < NR; ++i) *reinterpret_cast<u32x4*>(lds + ((i & 1) ? lo1 : lo0) + (i >> 1) * 16 * RW) = v[i];
}

template <typename T>
__device__ __forceinline__ typename WMF<T>::e8 ld_tr(const uint16_t* tile, int off_lo, int off_hi) {
  s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_lo));
  s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_hi));
  s16x8 v = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  return __builtin_bit_cast(typename WMF<T>::e8, v);
}

// Workgroup -> (split, n tile, k tile), XCD-aware: the hardware deals workgroups to the 8
// XCDs round-robin; logical tile L = (id % 8) * per + id / 8 gives XCD x a contiguous run.
__device__ __forceinline__ void wg_map(int tiles_n, int tiles_k, int& s, int& tn, int& tk) {
  // bijective for any grid size: XCD x owns logical tiles [start(x), start(x) + q (+1))
  const int total = gridDim.x;
  const int id = blockIdx.x;
  const int q = total / 8, rem = total % 8, xcd = id % 8;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + id / 8;
  tk = L % tiles_k;
  const int rest = L / tiles_k;
  tn = rest % tiles_n;
  s = rest / tiles_n;
}

template <typename T>
__global__ __launch_bounds__(kT, 1) void wgrad_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                        float* __restrict__ ws, int64_t Tn, int N, int K,
                                                        int64_t lda, int64_t ldb, int64_t t_split) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[TK * RW];
  __shared__ __attribute__((aligned(16))) uint16_t sB[TK * RW];
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, split, tn, tk);
  const int n0 = tn * TM, k0 = tk * TN;
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int hh = lane >> 5;

  // transposed-read offsets: lane supplies (row 4hh+q [+8], cols c..c+3) and receives
  // column (lane & 31) of each 32-wide block, rows {4hh..4hh+3, 4hh+8..4hh+11}
  int aLo[4], aHi[4], bLo[4], bHi[4];
  {
    const int q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ca = wm * 128 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      const int cb = wn * 128 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      aLo[i] = swz(4 * hh + q, ca >> 3) + (ca & 7);
      aHi[i] = swz(4 * hh + 8 + q, ca >> 3) + (ca & 7);
      bLo[i] = swz(4 * hh + q, cb >> 3) + (cb & 7);
      bHi[i] = swz(4 * hh + 8 + q, cb >> 3) + (cb & 7);
    }
  }

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0.f};

  const int vcA = (N - n0) >= TM ? CH : (N - n0) / 8;
  const int vcB = (K - k0) >= TN ? CH : (K - k0) / 8;
  // one register set: tile t+1's loads are issued before tile t's MFMAs and written to LDS
  // after them (two 2-register-set variants spilled: 256 arch VGPRs + 256 accumulators)
  u32x4 ra[NR], rb[NR];
  const int lo0 = swz(threadIdx.x / CH, threadIdx.x % CH), lo1 = swz(threadIdx.x / CH + 8, threadIdx.x % CH);

  int64_t t0 = t_begin;
  if (t0 < t_end) {
    stage_load(ra, A + t0 * lda + n0, lda, vcA);
    stage_load(rb, B + t0 * ldb + k0, ldb, vcB);
    stage_store(ra, sA, lo0, lo1);
    stage_store(rb, sB, lo0, lo1);
  }
  __syncthreads();
  while (t0 < t_end) {
    const int64_t tnext = t0 + TK;
    {
      // branch-free: the last tile re-reads itself (never stored)
      const int64_t tl = tnext < t_end ? tnext : t0;
      stage_load(ra, A + tl * lda + n0, lda, vcA);
      stage_load(rb, B + tl * ldb + k0, ldb, vcB);
    }
#pragma unroll
    for (int s = 0; s < TK / 16; ++s) {
      typename WMF<T>::e8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = ld_tr<T>(sA, aLo[i] + s * 16 * RW, aHi[i] + s * 16 * RW);
        fb[i] = ld_tr<T>(sB, bLo[i] + s * 16 * RW, bHi[i] + s * 16 * RW);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = WMF<T>::mma(fa[i], fb[j], acc[i][j]);
    }
    __syncthreads();
    if (tnext < t_end) {
      stage_store(ra, sA, lo0, lo1);
      stage_store(rb, sB, lo0, lo1);
    }
    __syncthreads();
    t0 = tnext;
  }

  // fp32 partial tile -> workspace [split][N][K]; lane holds column (lane & 31) of each
  // 32 x 32 block, rows (r & 3) + 8 (r >> 2) + 4 hh
  float* out = ws + static_cast<int64_t>(split) * N * K;
  const int col_l = lane & 31;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + wn * 128 + 32 * j + col_l;
    if (k >= K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wm * 128 + 32 * i + 4 * hh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = nb + (r & 3) + 8 * (r >> 2);
        if (n < N) out[static_cast<int64_t>(n) * K + k] = acc[i][j][r];
      }
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA variant
// Same tiling and MFMA work; operand tiles arrive by global_load_lds (16 B per lane, no VGPR
// staging, no ds_write pass) into TWO 64 KB stage buffers: tile t+1 is in flight while tile
// t is multiplied, one barrier per tile.  The LDS image is lane-linear per wave-instruction
// (2 rows of 512 B), so the XOR swizzle moves to the SOURCE address: physical chunk pc of row
// r is filled from logical chunk pc ^ g(r).
//
// The DMA is issued from inline asm: with the builtin, hipcc (ROCm 7.2) cannot tell the
// buffer being filled from the one being read and drains vmcnt(0) before the first ds_read
// of every tile -- the prefetch would never overlap the MFMAs.  The loop waits for its own
// DMA explicitly (vmcnt(0) before the end-of-tile barrier).
__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint16_t*)lds_wave_base)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}

// one operand tile (TK rows x 256 cols) -> LDS; this wave issues rows 16 w + 2 i + (lane >> 5)
__device__ __forceinline__ void stage_glds(uint16_t* lds, const uint16_t* src, int64_t ld, int vc, int wave,
                                           int lane) {
  const int pc = lane & 31, half = lane >> 5;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 16 * wave + 2 * i + half;
    const int g = ((r & 3) << 2) | ((r >> 2) & 3);
    int c = pc ^ g;
    c = c < vc ? c : vc - 1;
    glds16(src + static_cast<int64_t>(r) * ld + c * 8, lds + (16 * wave + 2 * i) * RW);
  }
}

template <typename T>
__global__ __launch_bounds__(kT, 1) void wgrad_glds_kernel(const uint16_t* __restrict__ A,
                                                             const uint16_t* __restrict__ B, float* __restrict__ ws,
                                                             int64_t Tn, int N, int K, int64_t lda, int64_t ldb,
                                                             int64_t t_split) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];  // 2 stages x (A, B) x 32 KB
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, split, tn, tk);
  const int n0 = tn * TM, k0 = tk * TN;
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int hh = lane >> 5;
  int aLo[4], aHi[4], bLo[4], bHi[4];
  {
    const int q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ca = wm * 128 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      const int cb = wn * 128 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      aLo[i] = swz(4 * hh + q, ca >> 3) + (ca & 7);
      aHi[i] = swz(4 * hh + 8 + q, ca >> 3) + (ca & 7);
      bLo[i] = swz(4 * hh + q, cb >> 3) + (cb & 7);
      bHi[i] = swz(4 * hh + 8 + q, cb >> 3) + (cb & 7);
    }
  }
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0.f};
  const int vcA = (N - n0) >= TM ? CH : (N - n0) / 8;
  const int vcB = (K - k0) >= TN ? CH : (K - k0) / 8;
  const int64_t ntiles = (t_end - t_begin) / TK;
  const uint16_t* pa = A + t_begin * lda + n0;
  const uint16_t* pb = B + t_begin * ldb + k0;
  constexpr int STAGE = 2 * TK * RW;  // elements per stage (A then B)
  if (ntiles > 0) {
    stage_glds(smem, pa, lda, vcA, wave, lane);
    stage_glds(smem + TK * RW, pb, ldb, vcB, wave, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // publishes the first tile
  for (int64_t t = 0; t < ntiles; ++t) {
    uint16_t* cur = smem + (t & 1) * STAGE;
    if (t + 1 < ntiles) {
      uint16_t* nxt = smem + ((t + 1) & 1) * STAGE;
      stage_glds(nxt, pa + (t + 1) * TK * lda, lda, vcA, wave, lane);
      stage_glds(nxt + TK * RW, pb + (t + 1) * TK * ldb, ldb, vcB, wave, lane);
    }
    const uint16_t* sA = cur;
    const uint16_t* sB = cur + TK * RW;
#pragma unroll
    for (int s = 0; s < TK / 16; ++s) {
      typename WMF<T>::e8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = ld_tr<T>(sA, aLo[i] + s * 16 * RW, aHi[i] + s * 16 * RW);
        fb[i] = ld_tr<T>(sB, bLo[i] + s * 16 * RW, bHi[i] + s * 16 * RW);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = WMF<T>::mma(fa[i], fb[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t+1 landed
    __syncthreads();  // ... everyone's, and every wave is done reading tile t
  }
  float* out = ws + static_cast<int64_t>(split) * N * K;
  const int col_l = lane & 31;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + wn * 128 + 32 * j + col_l;
    if (k >= K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wm * 128 + 32 * i + 4 * hh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = nb + (r & 3) + 8 * (r >> 2);
        if (n < N) out[static_cast<int64_t>(n) * K + k] = acc[i][j][r];
      }
    }
  }
}

inline bool wgrad_use_glds() {
  const char* e = getenv("SMP_WGRAD_GLDS");
  return e == nullptr || e[0] != '0';
}

// C (+)= sum over splits of ws, 4 elements per thread
template <typename TO>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, TO* __restrict__ c,
                                                            int64_t nk, int splits, int accumulate) {
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
  if (i >= nk) return;
  float4 s = *reinterpret_cast<const float4*>(ws + i);
  for (int p = 1; p < splits; ++p) {
    const float4 t = *reinterpret_cast<const float4*>(ws + p * nk + i);
    s.x += t.x;
    s.y += t.y;
    s.z += t.z;
    s.w += t.w;
  }
  if (accumulate) {
    s.x += to_f32(c[i]);
    s.y += to_f32(c[i + 1]);
    s.z += to_f32(c[i + 2]);
    s.w += to_f32(c[i + 3]);
  }
  c[i] = from_f32<TO>(s.x);
  c[i + 1] = from_f32<TO>(s.y);
  c[i + 2] = from_f32<TO>(s.z);
  c[i + 3] = from_f32<TO>(s.w);
}

}  // namespace

int wgrad_splits(int64_t tokens, int n, int k, int num_cus) {
  const int64_t tiles = static_cast<int64_t>((n + TM - 1) / TM) * ((k + TN - 1) / TN);
  const int64_t max_s = tokens / (TK * 8) > 1 ? tokens / (TK * 8) : 1;  // >= 8 token tiles per split
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= 16 && s <= max_s; ++s) {
    const int64_t wgs = tiles * s;
    const int64_t waves = (wgs + num_cus - 1) / num_cus;
    // fraction of CU-slots doing work, lightly penalising extra partial traffic
    const double eff = static_cast<double>(wgs) / static_cast<double>(waves * num_cus) - 0.004 * s;
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

int wgrad(int dt, const void* a, const void* b, int c_dt, void* c, float* ws, int64_t tokens, int n, int k,
          int64_t lda, int64_t ldb, int splits, int accumulate, hipStream_t s) {
  // whole 64-token tiles only (the caller adds the token remainder)
  if (n % 8 != 0 || k % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || splits < 1 || tokens % TK != 0) return -1;
  const int tiles = ((n + TM - 1) / TM) * ((k + TN - 1) / TN);
  int64_t t_split = (tokens + splits - 1) / splits;
  t_split = (t_split + TK - 1) / TK * TK;
  const int grid = tiles * splits;
  if (wgrad_use_glds()) {
    constexpr size_t lds = 2 * 2 * TK * RW * sizeof(uint16_t);  // 128 KB
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_glds_kernel<bf16>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_glds_kernel<f16>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      attr_set = true;
    }
    if (dt == BF16)
      wgrad_glds_kernel<bf16><<<grid, kT, lds, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                                    tokens, n, k, lda, ldb, t_split);
    else if (dt == F16)
      wgrad_glds_kernel<f16><<<grid, kT, lds, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                                   tokens, n, k, lda, ldb, t_split);
    else
      return -2;
  } else if (dt == BF16)
    wgrad_kernel<bf16><<<grid, kT, 0, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                            tokens, n, k, lda, ldb, t_split);
  else if (dt == F16)
    wgrad_kernel<f16><<<grid, kT, 0, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                           tokens, n, k, lda, ldb, t_split);
  else
    return -2;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t nk = static_cast<int64_t>(n) * k;  // multiple of 64 (n, k multiples of 8)
  const int rgrid = static_cast<int>((nk / 4 + 255) / 256);
  if (c_dt == F32)
    wgrad_reduce_kernel<float><<<rgrid, 256, 0, s>>>(ws, static_cast<float*>(c), nk, splits, accumulate);
  else if (c_dt == BF16)
    wgrad_reduce_kernel<bf16><<<rgrid, 256, 0, s>>>(ws, static_cast<bf16*>(c), nk, splits, accumulate);
  else if (c_dt == F16)
    wgrad_reduce_kernel<f16><<<rgrid, 256, 0, s>>>(ws, static_cast<f16*>(c), nk, splits, accumulate);
  else
    return -2;
  return hipGetLastError();
}

}  // namespace smpk
