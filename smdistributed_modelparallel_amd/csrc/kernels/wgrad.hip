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
// Within a split, L walks `group` n-tiles fastest and then the k-tiles, so the 32 workgroups
// an XCD runs at once cover a compact group x (32 / group) block of output tiles and share
// their A and B strips in that XCD's L2 (group 1: a row of k-tiles sharing one A strip).
__device__ __forceinline__ void wg_map(int tiles_n, int tiles_k, int group, int& s, int& tn, int& tk) {
  // bijective for any grid size: XCD x owns logical tiles [start(x), start(x) + q (+1))
  const int total = gridDim.x;
  const int id = blockIdx.x;
  const int q = total / 8, rem = total % 8, xcd = id % 8;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + id / 8;
  const int per = tiles_n * tiles_k;
  s = L / per;
  const int p = L - s * per;
  const int gfull = group * tiles_k;
  const int gid = p / gfull;
  const int first = gid * group;
  const int gs = tiles_n - first < group ? tiles_n - first : group;
  const int r = p - gid * gfull;
  tn = first + r % gs;
  tk = r / gs;
}

template <typename T>
__global__ __launch_bounds__(kT, 1) void wgrad_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                        float* __restrict__ ws, int64_t Tn, int N, int K,
                                                        int64_t lda, int64_t ldb, int64_t t_split, int group) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[TK * RW];
  __shared__ __attribute__((aligned(16))) uint16_t sB[TK * RW];
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, group, split, tn, tk);
  const int n0 = tn * TM, k0 = tk * TN;
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_wave_base) { lds_dma16(src, lds_wave_base); }

// one operand tile (TKS rows x 256 cols) -> LDS by W waves; wave w issues rows
// (TKS / W) w + 2 i + (lane >> 5), i < TKS / (2 W)
template <int W, int TKS>
__device__ __forceinline__ void stage_glds(uint16_t* lds, const uint16_t* src, int64_t ld, int vc, int wave,
                                           int lane) {
  constexpr int RPW = TKS / W;
  static_assert(RPW >= 2 && RPW % 2 == 0, "each wave stages whole row pairs");
  const int pc = lane & 31, half = lane >> 5;
  if (ld < (1 << 24)) {
    // saddr form: `src` (the tile base) is wave-uniform, the per-lane byte offset is
    // loop-invariant -- no 64-bit address arithmetic per load per tile
#pragma unroll
    for (int i = 0; i < RPW / 2; ++i) {
      const int r = RPW * wave + 2 * i + half;
      const int g = ((r & 3) << 2) | ((r >> 2) & 3);
      int c = pc ^ g;
      c = c < vc ? c : vc - 1;
      lds_dma16_sv(src, static_cast<uint32_t>((r * static_cast<int>(ld) + c * 8) * 2), lds + (RPW * wave + 2 * i) * RW);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < RPW / 2; ++i) {
    const int r = RPW * wave + 2 * i + half;
    const int g = ((r & 3) << 2) | ((r >> 2) & 3);
    int c = pc ^ g;
    c = c < vc ? c : vc - 1;
    glds16(src + static_cast<int64_t>(r) * ld + c * 8, lds + (RPW * wave + 2 * i) * RW);
  }
}

// instruction i (< TKS / W / 2) of stage_glds: the two rows RPW w + 2 i + {0, 1}
template <int W, int TKS>
__device__ __forceinline__ void stage_glds_one(uint16_t* lds, const uint16_t* src, int64_t ld, int vc, int wave,
                                               int lane, int i) {
  constexpr int RPW = TKS / W;
  const int pc = lane & 31, half = lane >> 5;
  const int r = RPW * wave + 2 * i + half;
  const int g = ((r & 3) << 2) | ((r >> 2) & 3);
  int c = pc ^ g;
  c = c < vc ? c : vc - 1;
  if (ld < (1 << 24))
    lds_dma16_sv(src, static_cast<uint32_t>((r * static_cast<int>(ld) + c * 8) * 2), lds + (RPW * wave + 2 * i) * RW);
  else
    glds16(src + static_cast<int64_t>(r) * ld + c * 8, lds + (RPW * wave + 2 * i) * RW);
}

// s_waitcnt vmcnt(N) leaving expcnt / lgkmcnt unconstrained (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// WN waves along the output columns (2 -> 4 waves of 128 x 128, 4 -> 8 waves of 128 x 64:
// two waves per SIMD, each with half the accumulators).  NS-stage ring of TKS-token tiles:
// the DMA of tile t + NS - 1 is issued right after the barrier that opens tile t, so a load
// has NS - 1 tiles of MFMA work to land; one barrier per tile.
// SPREAD: the next tile's DMA instructions are issued one A and one B piece per 16-token
// k-step, between that step's LDS reads and its MFMAs, instead of as one burst after the
// barrier (an LDS-DMA issue holds the wave ~60 cycles; in a burst both waves of a SIMD stall
// their MFMAs at the same time).
template <typename T, int WN, int TKS, int NS, bool SPREAD = false>
__global__ __launch_bounds__(128 * WN, 1) void wgrad_glds_kernel(const uint16_t* __restrict__ A,
                                                             const uint16_t* __restrict__ B, float* __restrict__ ws,
                                                             int64_t Tn, int N, int K, int64_t lda, int64_t ldb,
                                                             int64_t t_split, int group) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];  // NS stages x (A, B) x TKS rows
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, group, split, tn, tk);
  const int n0 = tn * TM, k0 = tk * TN;
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  constexpr int W = 2 * WN, NJ = 8 / WN, WCOLS = 32 * NJ;
  constexpr int L = 2 * (TKS / W / 2);  // DMA instructions per wave per tile (A and B)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int hh = lane >> 5;
  int aLo[4], aHi[4], bLo[NJ], bHi[NJ];
  {
    const int q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ca = wm * 128 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      aLo[i] = swz(4 * hh + q, ca >> 3) + (ca & 7);
      aHi[i] = swz(4 * hh + 8 + q, ca >> 3) + (ca & 7);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cb = wn * WCOLS + 32 * j + 16 * ((lane >> 4) & 1) + 4 * pp;
      bLo[j] = swz(4 * hh + q, cb >> 3) + (cb & 7);
      bHi[j] = swz(4 * hh + 8 + q, cb >> 3) + (cb & 7);
    }
  }
  f32x16 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{0.f};
  const int vcA = (N - n0) >= TM ? CH : (N - n0) / 8;
  const int vcB = (K - k0) >= TN ? CH : (K - k0) / 8;
  const int64_t ntiles = (t_end - t_begin) / TKS;
  const uint16_t* pa = A + t_begin * lda + n0;
  const uint16_t* pb = B + t_begin * ldb + k0;
  constexpr int STAGE = 2 * TKS * RW;  // elements per stage (A then B)
  const bool active = n0 + wm * 128 < N && k0 + wn * WCOLS < K;  // wave-uniform
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) {
    if (p < ntiles) {
      stage_glds<W, TKS>(smem + p * STAGE, pa + p * TKS * lda, lda, vcA, wave, lane);
      stage_glds<W, TKS>(smem + p * STAGE + TKS * RW, pb + p * TKS * ldb, ldb, vcB, wave, lane);
    }
  }
  int cur_slot = 0, load_slot = NS - 1;
  for (int64_t t = 0; t < ntiles; ++t) {
    if (t + NS - 2 < ntiles)
      wait_vm<(NS - 2) * L>();  // this wave's DMA of tile t landed (later tiles may fly)
    else
      wait_vm<0>();
    __syncthreads();  // ... everyone's, and every wave is done reading tile t - 1's slot
    const bool issue = t + NS - 1 < ntiles;
    uint16_t* nxt = smem + load_slot * STAGE;
    const int64_t tt = t + NS - 1;
    if (!SPREAD && issue) {
      stage_glds<W, TKS>(nxt, pa + tt * TKS * lda, lda, vcA, wave, lane);
      stage_glds<W, TKS>(nxt + TKS * RW, pb + tt * TKS * ldb, ldb, vcB, wave, lane);
    }
    load_slot = load_slot + 1 == NS ? 0 : load_slot + 1;
    const uint16_t* sA = smem + cur_slot * STAGE;
    const uint16_t* sB = sA + TKS * RW;
    cur_slot = cur_slot + 1 == NS ? 0 : cur_slot + 1;
#pragma unroll
    for (int s = 0; s < TKS / 16; ++s) {
      typename WMF<T>::e8 fa[4], fb[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = ld_tr<T>(sA, aLo[i] + s * 16 * RW, aHi[i] + s * 16 * RW);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = ld_tr<T>(sB, bLo[j] + s * 16 * RW, bHi[j] + s * 16 * RW);
      if constexpr (SPREAD) {
        constexpr int PER = (TKS / W / 2) / (TKS / 16);  // pieces per operand per k-step
        static_assert(PER >= 1 && PER * (TKS / 16) == TKS / W / 2, "pieces split evenly over the k-steps");
        if (issue) {
#pragma unroll
          for (int q = 0; q < PER; ++q) {
            stage_glds_one<W, TKS>(nxt, pa + tt * TKS * lda, lda, vcA, wave, lane, s * PER + q);
            stage_glds_one<W, TKS>(nxt + TKS * RW, pb + tt * TKS * ldb, ldb, vcB, wave, lane, s * PER + q);
          }
        }
      }
      // a wave whose whole output block lies past the matrix edge (e.g. 3 of the 4 column
      // waves of the last 64 of 1600 columns) skips its MFMAs
      if (active) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = WMF<T>::mma(fa[i], fb[j], acc[i][j]);
      }
    }
  }
  float* out = ws + static_cast<int64_t>(split) * N * K;
  const int col_l = lane & 31;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = k0 + wn * WCOLS + 32 * j + col_l;
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

// n-tiles per workgroup group in wg_map (SMP_WGRAD_GROUP, default 1: measured no better at 2-8)
inline int wgrad_group() {
  static const int v = [] {
    const char* e = getenv("SMP_WGRAD_GROUP");
    const int g = e != nullptr ? atoi(e) : 1;
    return g >= 1 && g <= 32 ? g : 1;
  }();
  return v;
}

// ---------------------------------------------------------------- phased (ping-pong) variant
// 8 waves (2 along N x 4 along K, 128 x 64 outputs each), 64-token K-tiles in two buffers.
// A buffer holds four 16 KB QUARTERS, each the part of the tile one MFMA phase consumes:
//   slot 0: A columns {0..63, 128..191}   (qm = 0 of both N wave rows)
//   slot 1: B columns {64 w + 0..31}      (qn = 0 of the four K wave columns)
//   slot 2: B columns {64 w + 32..63}     (qn = 1)
//   slot 3: A columns {64..127, 192..255} (qm = 1)
// Each tile runs 4 phases, one output quadrant each: (qm, qn) = (0,0) (0,1) (1,1) (1,0).
// A phase = [this phase's transposed LDS reads; DMA of one quarter of the NEXT tile; counted
// vmcnt; barrier; 8 MFMAs at raised priority; barrier].  Quarter j of tile t + 1 is issued in
// phase j of tile t and first read 3-4 phases later; the wait is counted (vmcnt 4, never 0 in
// steady state).  With PP the two N wave rows run one barrier apart (the second row takes an
// extra barrier up front), so on every SIMD one wave multiplies while the other reads LDS and
// issues DMA.  A wave waits for the data of phase p + 1 before its mid-phase barrier of phase
// p: with the one-barrier stagger that still precedes every reader's phase p + 1.
constexpr int QR = 128;       // elements per quarter row (256 B)
constexpr int QE = TK * QR;   // elements per quarter
constexpr int QBUF = 4 * QE;  // elements per K-tile buffer

// 16 chunks per 256-B row, chunk ^= 4 (row & 3): the 4-row x 32-column transposed reads of a
// 32-lane half hit all 64 banks once
__device__ __forceinline__ int qswz(int row, int col) {
  return row * QR + ((((col >> 3) ^ ((row & 3) << 2))) << 3) + (col & 7);
}

// one quarter (64 tokens x 128 region columns): region column x reads source column
// qoff + (x >> plog) * stride + (x & (piece - 1)) of the tile; 16 four-row DMA instructions,
// two per wave.  Columns at or past vcols (matrix edge) re-read column 0 -- they only feed
// outputs that are never stored.
__device__ __forceinline__ void stage_quarter(uint16_t* region, const uint16_t* src, int64_t ld, int qoff, int plog,
                                              int stride, int vcols, int wave, int lane) {
  const int sub = lane >> 4;
  const int lc = (lane & 15) ^ (sub << 2);
  const int x = lc * 8;
  int col = qoff + (x >> plog) * stride + (x & ((1 << plog) - 1));
  col = col < vcols ? col : 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = 2 * wave + i;
    glds16(src + static_cast<int64_t>(4 * m + sub) * ld + col, region + 4 * m * QR);
  }
}

__device__ __forceinline__ void phase_sync() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <typename T>
__device__ __forceinline__ void ld_frags(typename WMF<T>::e8 (&f)[4], const uint16_t* region, int off) {
#pragma unroll
  for (int s = 0; s < 4; ++s) f[s] = ld_tr<T>(region, off + s * 16 * QR, off + s * 16 * QR + 8 * QR);
}

template <typename T>
__device__ __forceinline__ void mma_quadrant(f32x16& c0, f32x16& c1, const typename WMF<T>::e8 (&a0)[4],
                                             const typename WMF<T>::e8 (&a1)[4], const typename WMF<T>::e8 (&b)[4]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    c0 = WMF<T>::mma(a0[s], b[s], c0);
    c1 = WMF<T>::mma(a1[s], b[s], c1);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <typename T, bool PP>
__global__ __launch_bounds__(512, 1) void wgrad_pp_kernel(const uint16_t* __restrict__ A,
                                                          const uint16_t* __restrict__ B, float* __restrict__ ws,
                                                          int64_t Tn, int N, int K, int64_t lda, int64_t ldb,
                                                          int64_t t_split, int group) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];  // 2 K-tile buffers x 4 quarters
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, group, split, tn, tk);
  const int n0 = tn * TM, k0 = tk * TN;
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int aOff0, aOff1, bOff;
  {
    const int row = 4 * (lane >> 5) + ((lane & 15) >> 2);
    const int c = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
    aOff0 = qswz(row, wr * 64 + c);
    aOff1 = qswz(row, wr * 64 + 32 + c);
    bOff = qswz(row, wc * 32 + c);
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x16{0.f};
  const int vA = (N - n0) >= TM ? TM : N - n0;
  const int vB = (K - k0) >= TN ? TN : K - k0;
  const int64_t ntiles = t_end > t_begin ? (t_end - t_begin) / TK : 0;
  const uint16_t* pa = A + t_begin * lda + n0;
  const uint16_t* pb = B + t_begin * ldb + k0;
  if (ntiles > 0) {
    stage_quarter(smem + 0 * QE, pa, lda, 0, 6, 128, vA, wave, lane);
    stage_quarter(smem + 1 * QE, pb, ldb, 0, 5, 64, vB, wave, lane);
    stage_quarter(smem + 2 * QE, pb, ldb, 32, 5, 64, vB, wave, lane);
    stage_quarter(smem + 3 * QE, pa, lda, 64, 6, 128, vA, wave, lane);
    wait_vm<4>();  // slots 0, 1 of tile 0
    phase_sync();
    if (PP && wr == 1) phase_sync();
    typename WMF<T>::e8 fa0[4], fa1[4], fb0[4], fb1[4];
    for (int64_t t = 0; t < ntiles; ++t) {
      const uint16_t* cb = smem + (t & 1) * QBUF;
      uint16_t* nb = smem + ((t + 1) & 1) * QBUF;
      const bool next = t + 1 < ntiles;
      const uint16_t* na = pa + (t + 1) * TK * lda;
      const uint16_t* nbp = pb + (t + 1) * TK * ldb;
      // phase 0: (qm 0, qn 0)
      ld_frags<T>(fa0, cb + 0 * QE, aOff0);
      ld_frags<T>(fa1, cb + 0 * QE, aOff1);
      ld_frags<T>(fb0, cb + 1 * QE, bOff);
      if (next) {
        stage_quarter(nb + 0 * QE, na, lda, 0, 6, 128, vA, wave, lane);
        wait_vm<4>();  // slot 2 of tile t
      } else {
        wait_vm<0>();
      }
      phase_sync();
      mma_quadrant<T>(acc[0][0], acc[1][0], fa0, fa1, fb0);
      phase_sync();
      // phase 1: (qm 0, qn 1)
      ld_frags<T>(fb1, cb + 2 * QE, bOff);
      if (next) {
        stage_quarter(nb + 1 * QE, nbp, ldb, 0, 5, 64, vB, wave, lane);
        wait_vm<4>();  // slot 3 of tile t
      } else {
        wait_vm<0>();
      }
      phase_sync();
      mma_quadrant<T>(acc[0][1], acc[1][1], fa0, fa1, fb1);
      phase_sync();
      // phase 2: (qm 1, qn 1)
      ld_frags<T>(fa0, cb + 3 * QE, aOff0);
      ld_frags<T>(fa1, cb + 3 * QE, aOff1);
      if (next) stage_quarter(nb + 2 * QE, nbp, ldb, 32, 5, 64, vB, wave, lane);
      phase_sync();
      mma_quadrant<T>(acc[2][1], acc[3][1], fa0, fa1, fb1);
      phase_sync();
      // phase 3: (qm 1, qn 0)
      if (next) {
        stage_quarter(nb + 3 * QE, na, lda, 64, 6, 128, vA, wave, lane);
        wait_vm<4>();  // slots 0, 1 of tile t + 1
      }
      phase_sync();
      mma_quadrant<T>(acc[2][0], acc[3][0], fa0, fa1, fb0);
      phase_sync();
    }
    if (PP && wr == 0) phase_sync();
  }
  float* out = ws + static_cast<int64_t>(split) * N * K;
  const int col_l = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = k0 + wc * 64 + 32 * j + col_l;
    if (k >= K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wr * 128 + 32 * i + 4 * hh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = nb + (r & 3) + 8 * (r >> 2);
        if (n < N) out[static_cast<int64_t>(n) * K + k] = acc[i][j][r];
      }
    }
  }
}

template <typename T, bool PP>
int launch_pp(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
              int64_t ldb, int64_t t_split, int grid, hipStream_t s) {
  constexpr size_t lds = 2 * QBUF * sizeof(uint16_t);  // 128 KB
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<T, PP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr_set = true;
  }
  wgrad_pp_kernel<T, PP><<<grid, 512, lds, s>>>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, wgrad_group());
  return 0;
}

// ------------------------------------------------------ 16x16x32 MFMA variant
// Same staging (LDS-DMA ring, swizzled 512-B rows) and 8-wave 128 x 64 output blocks, but
// v_mfma_f32_16x16x32: 16 cycles per instruction instead of 32, which on gfx950 delivers
// ~1.12-1.15x the FLOP/s of 32x32x16 in MFMA loops (MI355X_MICROARCH.md).  A 16 x 32 operand
// fragment is two ds_read_b64_tr_b16: the 16-lane group g takes tokens 8 g .. 8 g + 7 of the
// 32-token k-step, lane 4 q + p supplying row q (+4), columns 4 p .. 4 p + 3 of its 16-column
// block; lane l receives column l % 16.  Accumulator: lane l holds C[4 (l / 16) + r][l % 16].
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <typename T>
struct WMF16;
template <>
struct WMF16<bf16> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct WMF16<f16> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// the idle-wave column-sum mode applies: the last 256-wide K tile leaves a 64-wide wave column free
__host__ __device__ __forceinline__ bool wgrad_cs_idle(int K) { return K % 256 != 0 && K % 256 <= 192; }

template <typename T>
__device__ __forceinline__ typename WMF16<T>::e8 ld_tr16(const uint16_t* tile, int off_lo, int off_hi) {
  s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_lo));
  s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_hi));
  s16x8 v = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  return __builtin_bit_cast(typename WMF16<T>::e8, v);
}

// cs != nullptr: the kernel also sums the staged A (= dY) rows per column -- the bias gradient
// of the layer, sum over tokens of dY -- in the same pass over dY, one of two ways:
//  * idle-wave MFMA (K % 256 in [1, 192]; every GPT-2 XL layer with K = 1600): in the last K
//    tile the wave columns past K have no output; the first of them multiplies its A fragments
//    by an all-ones B fragment instead (acc[n][c] = sum over tokens of A[t][n]), on a SIMD that
//    would otherwise idle -- 8 extra MFMAs per k-step in one workgroup per (split, tn).  Output
//    cs[split][N].
//  * otherwise, through LDS: the tiles_k workgroups that share an A strip split the work
//    (workgroup tk sums the 64-token tiles t with t % tiles_k == tk) into
//    cs[split * tiles_k + tk][N] (fp32, fixed order: rows of a tile per thread, 16 row groups
//    through LDS, partials in order).  Measured in-step (profiles/r3/wgrad_variants.md) this
//    costs the MFMA loop about what a separate column-sum pass would.
//
// One SEGMENT = output tile (tn, tk) over `ntiles` 64-token tiles from token t_begin; the fp32
// partial goes to out[(n - nb0) * ldo + (k - kb0)] and (colsum) the column sums to
// cso[n - nb0].  Split mode: one segment per workgroup, out = the split's [N][K] slice.
// (A stream-K style schedule -- equal runs of (tile, token-tile) items per workgroup, up to two
// segments each, partial tiles summed in order -- was built on these segments and measured
// 10-35 % SLOWER on every GPT-2 XL shape (profiles/r3/wgrad_variants.md): concurrent
// workgroups then stream disjoint token ranges and stop sharing A / B strips in L2.)
template <typename T, int TKS, int NS, bool SPREAD>
__device__ __forceinline__ void glds16_segment(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                               uint16_t* smem, int N, int K, int64_t lda, int64_t ldb, int tn, int tk,
                                               int64_t t_begin, int64_t ntiles, float* __restrict__ out,
                                               int64_t ldo, int nb0, int kb0, float* __restrict__ cso, bool colsum,
                                               int cs_mod, int cs_rem, bool cs_idle) {
  constexpr int W = 8, WCOLS = 64, NI = 8, NJ = 4;  // wave block 128 x 64 = 8 x 4 tiles of 16 x 16
  constexpr int L = 2 * (TKS / W / 2);
  const int n0 = tn * TM, k0 = tk * TN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / 4, wn = wave % 4;
  // transposed-read offsets for k-step 0: row 8 (l / 16) + q (+4), column block base + 4 p
  int aLo[NI], aHi[NI], bLo[NJ], bHi[NJ];
  {
    const int row = 8 * (lane >> 4) + ((lane & 15) >> 2), pp = lane & 3;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int ca = wm * 128 + 16 * i + 4 * pp;
      aLo[i] = swz(row, ca >> 3) + (ca & 7);
      aHi[i] = swz(row + 4, ca >> 3) + (ca & 7);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cb = wn * WCOLS + 16 * j + 4 * pp;
      bLo[j] = swz(row, cb >> 3) + (cb & 7);
      bHi[j] = swz(row + 4, cb >> 3) + (cb & 7);
    }
  }
  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int vcA = (N - n0) >= TM ? CH : (N - n0) / 8;
  const int vcB = (K - k0) >= TN ? CH : (K - k0) / 8;
  const uint16_t* pa = A + t_begin * lda + n0;
  const uint16_t* pb = B + t_begin * ldb + k0;
  constexpr int STAGE = 2 * TKS * RW;
  // idle-wave column sums: the first wave column past K (only exists in the last K tile) runs
  // the normal MFMA loop with its first B fragment replaced by ones (no extra live registers)
  const bool cs_wave = cs_idle && n0 + wm * 128 < N && wn == (K - k0 + WCOLS - 1) / WCOLS;
  const bool active = (n0 + wm * 128 < N && k0 + wn * WCOLS < K) || cs_wave;  // wave-uniform
  typename WMF16<T>::e8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = 1.0f;
  // column-sum accumulators in LDS after the operand ring (no registers held across the
  // loop: the kernel is at its VGPR limit): thread (row group t >> 5, chunk t & 31) owns
  // floats [(t >> 5) * 256 + (t & 31) * 8, +8)
  float* csl = reinterpret_cast<float*>(smem + NS * STAGE) + (threadIdx.x >> 5) * 256 + (threadIdx.x & 31) * 8;
  if (colsum) {
    *reinterpret_cast<f32x4*>(csl) = f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(csl + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) {
    if (p < ntiles) {
      stage_glds<W, TKS>(smem + p * STAGE, pa + p * TKS * lda, lda, vcA, wave, lane);
      stage_glds<W, TKS>(smem + p * STAGE + TKS * RW, pb + p * TKS * ldb, ldb, vcB, wave, lane);
    }
  }
  int cur_slot = 0, load_slot = NS - 1;
  for (int64_t t = 0; t < ntiles; ++t) {
    if (t + NS - 2 < ntiles)
      wait_vm<(NS - 2) * L>();
    else
      wait_vm<0>();
    __syncthreads();
    const bool issue = t + NS - 1 < ntiles;
    uint16_t* nxt = smem + load_slot * STAGE;
    const int64_t tt = t + NS - 1;
    if (!SPREAD && issue) {
      stage_glds<W, TKS>(nxt, pa + tt * TKS * lda, lda, vcA, wave, lane);
      stage_glds<W, TKS>(nxt + TKS * RW, pb + tt * TKS * ldb, ldb, vcB, wave, lane);
    }
    load_slot = load_slot + 1 == NS ? 0 : load_slot + 1;
    const uint16_t* sA = smem + cur_slot * STAGE;
    const uint16_t* sB = sA + TKS * RW;
    cur_slot = cur_slot + 1 == NS ? 0 : cur_slot + 1;
    if (colsum && static_cast<int>(t % cs_mod) == cs_rem) {
      const int ch = threadIdx.x & 31;
      f32x4 c0 = *reinterpret_cast<const f32x4*>(csl), c1 = *reinterpret_cast<const f32x4*>(csl + 4);
#pragma unroll
      for (int i = 0; i < TKS / 16; ++i) {
        const int row = (threadIdx.x >> 5) + 16 * i;
        const u32x4 v = *reinterpret_cast<const u32x4*>(sA + swz(row, ch));
        c0[0] += __uint_as_float(v[0] << 16);
        c0[1] += __uint_as_float(v[0] & 0xffff0000u);
        c0[2] += __uint_as_float(v[1] << 16);
        c0[3] += __uint_as_float(v[1] & 0xffff0000u);
        c1[0] += __uint_as_float(v[2] << 16);
        c1[1] += __uint_as_float(v[2] & 0xffff0000u);
        c1[2] += __uint_as_float(v[3] << 16);
        c1[3] += __uint_as_float(v[3] & 0xffff0000u);
      }
      *reinterpret_cast<f32x4*>(csl) = c0;
      *reinterpret_cast<f32x4*>(csl + 4) = c1;
    }
#pragma unroll
    for (int s = 0; s < TKS / 32; ++s) {
      typename WMF16<T>::e8 fa[NI / 2], fb[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = ld_tr16<T>(sB, bLo[j] + s * 32 * RW, bHi[j] + s * 32 * RW);
      if (cs_wave) fb[0] = ones;
#pragma unroll
      for (int i = 0; i < NI / 2; ++i) fa[i] = ld_tr16<T>(sA, aLo[i] + s * 32 * RW, aHi[i] + s * 32 * RW);
      if constexpr (SPREAD) {
        constexpr int PER = (TKS / W / 2) / (TKS / 32);
        static_assert(PER >= 1 && PER * (TKS / 32) == TKS / W / 2, "pieces split evenly over the k-steps");
        if (issue) {
#pragma unroll
          for (int q = 0; q < PER; ++q) {
            stage_glds_one<W, TKS>(nxt, pa + tt * TKS * lda, lda, vcA, wave, lane, s * PER + q);
            stage_glds_one<W, TKS>(nxt + TKS * RW, pb + tt * TKS * ldb, ldb, vcB, wave, lane, s * PER + q);
          }
        }
      }
      // the A fragments in two halves of 4 (fewer live registers)
      if (active) {
#pragma unroll
        for (int i = 0; i < NI / 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = WMF16<T>::mma(fa[i], fb[j], acc[i][j]);
      }
#pragma unroll
      for (int i = 0; i < NI / 2; ++i)
        fa[i] = ld_tr16<T>(sA, aLo[NI / 2 + i] + s * 32 * RW, aHi[NI / 2 + i] + s * 32 * RW);
      if (active) {
#pragma unroll
        for (int i = 0; i < NI / 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[NI / 2 + i][j] = WMF16<T>::mma(fa[i], fb[j], acc[NI / 2 + i][j]);
      }
    }
  }
  if (colsum) {
    // the 16 row groups' sums of each of the 256 columns
    __syncthreads();
    const float* red = reinterpret_cast<const float*>(smem + NS * STAGE);
    if (threadIdx.x < 256 && n0 + static_cast<int>(threadIdx.x) < N) {
      float a = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) a += red[g * 256 + threadIdx.x];
      cso[n0 + threadIdx.x - nb0] = a;
    }
  }
  const int col_l = lane & 15, rq = 4 * (lane >> 4);
  if (cs_wave && col_l == 0) {  // every column of acc[i][0] holds the row sums
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * 128 + 16 * i + rq + r;
        if (n < N) cso[n - nb0] = acc[i][0][r];
      }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = k0 + wn * WCOLS + 16 * j + col_l;
    if (k >= K) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int nb = n0 + wm * 128 + 16 * i + rq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nb + r;
        if (n < N) out[static_cast<int64_t>(n - nb0) * ldo + (k - kb0)] = acc[i][j][r];
      }
    }
  }
}

template <typename T, int TKS, int NS, bool SPREAD>
__global__ __launch_bounds__(512, 1) void wgrad_glds16_kernel(const uint16_t* __restrict__ A,
                                                             const uint16_t* __restrict__ B, float* __restrict__ ws,
                                                             int64_t Tn, int N, int K, int64_t lda, int64_t ldb,
                                                             int64_t t_split, int group, float* __restrict__ cs) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, group, split, tn, tk);
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const bool idle = wgrad_cs_idle(K);
  glds16_segment<T, TKS, NS, SPREAD>(
      A, B, smem, N, K, lda, ldb, tn, tk, t_begin, (t_end - t_begin) / TKS, ws + static_cast<int64_t>(split) * N * K,
      K, 0, 0, cs == nullptr ? nullptr : cs + (static_cast<int64_t>(split) * (idle ? 1 : tiles_k) + (idle ? 0 : tk)) * N,
      cs != nullptr && !idle, tiles_k, tk, cs != nullptr && idle);
}

template <typename T, int TKS, int NS, bool SPREAD>
int launch_glds16(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
                  int64_t ldb, int64_t t_split, int grid, hipStream_t s, float* cs = nullptr) {
  // operand ring + the column-sum accumulators (16 row groups x 256 fp32)
  constexpr size_t lds = static_cast<size_t>(NS) * 2 * TKS * RW * sizeof(uint16_t) + 16 * 256 * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS per CU");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_glds16_kernel<T, TKS, NS, SPREAD>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr_set = true;
  }
  wgrad_glds16_kernel<T, TKS, NS, SPREAD><<<grid, 512, lds, s>>>(pa, pb, ws, tokens, n, k, lda, ldb, t_split,
                                                                 wgrad_group(), cs);
  return 0;
}

// SMP_WGRAD_PIPE: 0 = 4 waves, 2 x 64-token stages; 1 = 8 waves, 2 x 64; 2 = 8 waves,
// 4 x 32; 3 = 8 waves, 5 x 32 (all 160 KB of LDS); 4 = phased, lockstep; 5 = phased ping-pong;
// 6 / 7 = 1 / 2 with the DMA spread over the k-steps; 8 / 9 = 1 / 6 on 16x16x32 MFMAs.
// Default 8 (tools/gpu_wgrad_ab.sh, same box, interleaved, ms at T = 65536: 4800x1600 s8
// 1.123 vs 1.163, 6400x1600 s4 1.359-1.364 vs 1.419, 1600x6400 s4 1.454-1.471 vs 1.498,
// 1600x1600 s5 0.360-0.363 vs 0.370; spreading the DMA over the k-steps: no gain)
inline int wgrad_pipe() {
  static const int v = [] {
    const char* e = getenv("SMP_WGRAD_PIPE");
    if (e != nullptr && e[0] >= '0' && e[0] <= '9') return e[0] - '0';
    const char* w = getenv("SMP_WGRAD_WAVES");
    return (w != nullptr && w[0] == '4') ? 0 : 8;
  }();
  return v;
}

template <typename T, int WN, int TKS, int NS, bool SPREAD = false>
int launch_glds(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
                int64_t ldb, int64_t t_split, int grid, hipStream_t s) {
  constexpr size_t lds = static_cast<size_t>(NS) * 2 * TKS * RW * sizeof(uint16_t);
  static_assert(lds <= 160 * 1024, "LDS per CU");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_glds_kernel<T, WN, TKS, NS, SPREAD>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr_set = true;
  }
  wgrad_glds_kernel<T, WN, TKS, NS, SPREAD><<<grid, 128 * WN, lds, s>>>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, wgrad_group());
  return 0;
}

template <typename T>
int launch_glds_pipe(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
                     int64_t ldb, int64_t t_split, int grid, hipStream_t s) {
  switch (wgrad_pipe()) {
    case 0:
      return launch_glds<T, 2, 64, 2>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 2:
      return launch_glds<T, 4, 32, 4>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 3:
      return launch_glds<T, 4, 32, 5>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 4:
      return launch_pp<T, false>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 5:
      return launch_pp<T, true>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 6:
      return launch_glds<T, 4, 64, 2, true>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 7:
      return launch_glds<T, 4, 32, 4, true>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 8:
      return launch_glds16<T, 64, 2, false>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    case 9:
      return launch_glds16<T, 64, 2, true>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    default:
      return launch_glds<T, 4, 64, 2>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
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

// bias (+)= sum over the partial rows of cs[part][n], in order
template <typename TO>
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ cs, TO* __restrict__ bias, int n,
                                                            int splits, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float a = accumulate ? to_f32(bias[i]) : 0.f;
  for (int p = 0; p < splits; ++p) a += cs[static_cast<int64_t>(p) * n + i];
  bias[i] = from_f32<TO>(a);
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
          int64_t lda, int64_t ldb, int splits, int accumulate, hipStream_t s, int bias_dt, void* bias, float* cs,
          int bias_accumulate) {
  // whole 64-token tiles only (the caller adds the token remainder)
  if (n % 8 != 0 || k % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || splits < 1 || tokens % TK != 0) return -1;
  if (bias != nullptr && (dt != BF16 || cs == nullptr)) return -3;  // column sums: bf16 operands
  const int tiles = ((n + TM - 1) / TM) * ((k + TN - 1) / TN);
  int64_t t_split = (tokens + splits - 1) / splits;
  t_split = (t_split + TK - 1) / TK * TK;
  const int grid = tiles * splits;
  if (bias != nullptr) {
    // the column-sum pass lives in the 16x16x32 kernel
    const auto* pa = static_cast<const uint16_t*>(a);
    const auto* pb = static_cast<const uint16_t*>(b);
    if (wgrad_pipe() == 9)
      launch_glds16<bf16, 64, 2, true>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, cs);
    else
      launch_glds16<bf16, 64, 2, false>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, cs);
  } else if (wgrad_use_glds()) {
    const auto* pa = static_cast<const uint16_t*>(a);
    const auto* pb = static_cast<const uint16_t*>(b);
    if (dt == BF16)
      launch_glds_pipe<bf16>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    else if (dt == F16)
      launch_glds_pipe<f16>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
    else
      return -2;
  } else if (dt == BF16)
    wgrad_kernel<bf16><<<grid, kT, 0, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                            tokens, n, k, lda, ldb, t_split, 1);
  else if (dt == F16)
    wgrad_kernel<f16><<<grid, kT, 0, s>>>(static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), ws,
                                           tokens, n, k, lda, ldb, t_split, 1);
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
  if (bias != nullptr) {
    const int parts = splits * (wgrad_cs_idle(k) ? 1 : (k + TN - 1) / TN);
    const unsigned g = static_cast<unsigned>((n + 255) / 256);
    if (bias_dt == F32)
      colsum_reduce_kernel<float><<<g, 256, 0, s>>>(cs, static_cast<float*>(bias), n, parts, bias_accumulate);
    else if (bias_dt == BF16)
      colsum_reduce_kernel<bf16><<<g, 256, 0, s>>>(cs, static_cast<bf16*>(bias), n, parts, bias_accumulate);
    else
      return -2;
  }
  return hipGetLastError();
}

}  // namespace smpk
