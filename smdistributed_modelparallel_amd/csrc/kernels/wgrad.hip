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
// Design (one kernel, wgrad_glds16_kernel):
//  * operands are staged row-major exactly as they sit in HBM (512-B rows, fully coalesced)
//    by LDS-DMA (global_load_lds from inline asm, so hipcc does not drain the prefetch before
//    every ds_read) into a two-stage ring of 64-token tiles, one barrier per tile; the XOR
//    swizzle of the 16-B chunks moves to the source address (conflict-free transposed reads);
//  * the MFMA fragments -- 8 consecutive reduction elements per lane -- come from
//    ds_read_b64_tr_b16, the gfx950 LDS transpose read;
//  * v_mfma_f32_16x16x32_bf16 (f16), 512 threads = 8 waves (2 per SIMD) in 2 x 4, each wave
//    owns a 128 x 64 block of the 256 x 256 output tile (32 accumulator tiles);
//  * split-K over tokens: the split count comes from the host (a fixed per-shape table in
//    ops/linear.py, or the occupancy model wgrad_splits); each split writes an fp32 partial
//    tile and a vectorised reduction adds the partials into the gradient (beta = 1: the
//    gradient buffer accumulates across microbatches, no temporary dW);
//  * workgroups are dealt to XCDs in contiguous runs of (split, n-tile) so that the
//    workgroups sharing an A strip share one XCD's L2;
//  * optional bias gradient (sum over tokens of dY) from the same staged dY tiles.
//
// Measured and removed (A/B records in profiles/r2/wgrad_kernel.md, profiles/r3/wgrad_variants.md):
// a register-staged 32x32x16 kernel (630-775 TFLOP/s), the 32x32x16 LDS-DMA kernel with 4 or 8
// waves and 2-5 stages (750-900), a phased ping-pong 8-wave variant, DMA issue spread over the
// k-steps (no gain), and a stream-K schedule (10-35 % slower: workgroups sharing a tile then
// read disjoint token ranges and stop sharing A / B strips in L2).
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
// native 16-B vector (HIP's uint4 is a class wrapper that SROA leaves in scratch here)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 256;     // output tile rows (N)
constexpr int TN = 256;     // output tile cols (K)
constexpr int TK = 64;      // tokens per staged tile
// fallback kernel geometry: 8 waves (2 per SIMD, 128 x 64 wave blocks), 64-token LDS stages,
// 2 stages.  (Round 4 A/B: 4 waves with 128 x 128 blocks was 10-14 % slower, 32-token / 3-stage
// and a raised MFMA-wave priority lost too -- profiles/r4/attention_r4c.md,
// profiles/r4/parallel_residual_fusion.md.)
constexpr int kW = 8;
constexpr int kWCOLS = 256 / (kW / 2);  // output columns per wave (2 wave rows of 128)
constexpr int kTK = 64;  // tokens per LDS stage of the kernel
constexpr int kNS = 2;   // LDS stages (2 x 64-token operand tiles + 16 KB column sums)
constexpr int RW = 256;     // LDS row width (elements) of both staged tiles
constexpr int CH = RW / 8;  // 16-B chunks per row

// XOR swizzle of the 16-B chunks of a 512-B row (row bits 0-3): conflict-free for the
// row-wise stores and the 4-row transposed reads.
__device__ __forceinline__ int swz(int row, int chunk) {
  const int g = ((row & 3) << 2) | ((row >> 2) & 3);
  return row * RW + ((chunk ^ g) << 3);
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

// s_waitcnt vmcnt(N) leaving expcnt / lgkmcnt unconstrained (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// n-tiles per workgroup group in wg_map: 1 = a row of k-tiles shares one A strip per XCD
// (groups of 2-8 n-tiles measured no better, profiles/r2/wgrad_kernel.md)
constexpr int kWgradGroup = 1;

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
__host__ __device__ __forceinline__ bool wgrad_cs_idle(int K) { return K % 256 != 0 && K % 256 <= 256 - kWCOLS; }

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
template <typename T, int TKS, int NS>
__device__ __forceinline__ void glds16_segment(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                               uint16_t* smem, int N, int K, int64_t lda, int64_t ldb, int tn, int tk,
                                               int64_t t_begin, int64_t ntiles, float* __restrict__ out,
                                               int64_t ldo, int nb0, int kb0, float* __restrict__ cso, bool colsum,
                                               int cs_mod, int cs_rem, bool cs_idle) {
  // wave block 128 x WCOLS = 8 x NJ tiles of 16 x 16; waves in 2 rows x (W / 2) columns
  constexpr int W = kW, WCOLS = kWCOLS, NI = 8, NJ = WCOLS / 16, RG = W * 2;
  constexpr int L = 2 * (TKS / W / 2);
  const int n0 = tn * TM, k0 = tk * TN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / (W / 2), wn = wave % (W / 2);
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
  // loop: the kernel is at its VGPR limit): thread (row group t >> 5 of RG, chunk t & 31) owns
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
    if (issue) {
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
      for (int i = 0; i < TKS / RG; ++i) {
        const int row = (threadIdx.x >> 5) + RG * i;
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
    // the RG row groups' sums of each of the 256 columns
    __syncthreads();
    const float* red = reinterpret_cast<const float*>(smem + NS * STAGE);
    if (threadIdx.x < 256 && n0 + static_cast<int>(threadIdx.x) < N) {
      float a = 0.f;
#pragma unroll
      for (int g = 0; g < RG; ++g) a += red[g * 256 + threadIdx.x];
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

template <typename T, int TKS, int NS>
__global__ __launch_bounds__(64 * kW, 1) void wgrad_glds16_kernel(const uint16_t* __restrict__ A,
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
  glds16_segment<T, TKS, NS>(
      A, B, smem, N, K, lda, ldb, tn, tk, t_begin, (t_end - t_begin) / TKS, ws + static_cast<int64_t>(split) * N * K,
      K, 0, 0, cs == nullptr ? nullptr : cs + (static_cast<int64_t>(split) * (idle ? 1 : tiles_k) + (idle ? 0 : tk)) * N,
      cs != nullptr && !idle, tiles_k, tk, cs != nullptr && idle);
}

template <typename T, int TKS, int NS>
int launch_glds16(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
                  int64_t ldb, int64_t t_split, int grid, hipStream_t s, float* cs = nullptr) {
  // operand ring + the column-sum accumulators (16 row groups x 256 fp32)
  constexpr size_t lds = static_cast<size_t>(NS) * 2 * TKS * RW * sizeof(uint16_t) + 16 * 256 * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS per CU");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_glds16_kernel<T, TKS, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr_set = true;
  }
  wgrad_glds16_kernel<T, TKS, NS><<<grid, 64 * kW, lds, s>>>(pa, pb, ws, tokens, n, k, lda, ldb, t_split,
                                                                 kWgradGroup, cs);
  return 0;
}

// ------------------------------------------------------------ ping-pong kernel (round 5)
// Same problem, same 256 x 256 output tile and split-K partials, restructured as the
// phased two-row schedule of the fast CDNA4 GEMM template (cdna_hip_programming.md §5,
// "The 256² 8-phase template"; T3/T4/T5): every 64-token K-tile is FOUR phases, one per
// 64 x 32 quadrant of a wave's output (16 MFMAs each), and every phase is
//     load segment: LDS transpose reads of the fragments this phase needs, 2 LDS-DMA
//                   pieces of the NEXT tile, a COUNTED vmcnt, barrier
//     MFMA segment: 16 v_mfma_f32_16x16x32 at raised priority, barrier.
// Wave row 1 starts one barrier late, so on every SIMD the row-0 wave's MFMA segment runs
// beside the row-1 wave's load segment and vice versa (ping-pong): the matrix pipe never
// waits for an LDS read burst, and the DMA of tile t+1 stays in flight for 2-3 phases
// (vmcnt never drains to 0 in the loop).
//
// LDS: 8 half-tile slots of 16 KB (two tiles in flight).  A K-tile is four half-tiles --
// A columns [0,128) / [128,256) and B columns [0,128) / [128,256) -- and wave (wm, wn) owns
// output rows {qa*128 + wm*64 + [0,64)} x columns {qb*128 + wn*32 + [0,32)}, qa, qb in {0,1},
// so quadrant (qa, qb) reads exactly A half qa and B half qb.  Phase order (0,0) (0,1) (1,1)
// (1,0): a phase needs at most one half-tile it has not read before, and the next tile's
// halves are staged in that order, one per phase.
//
// Half-tile image: [token quad 16][16-column block 8][4 tokens][16 columns], 128 B per
// block, block index XOR (quad & 1).  One LDS-DMA wave instruction (1 KiB, lane-linear) is
// one token quad; the XOR is applied on the SOURCE columns (rule 21).  ds_read_b64_tr_b16:
// 16-lane group g reads token quad 8s + 4r + g (r = 0, 1 -> fragment elements 4r .. 4r + 3)
// of the k-step s; the two groups of a 32-lane half read quads of opposite parity, i.e.
// opposite 128-B halves of a bank row: conflict-free.  The A and B fragments use the same
// (group, element) -> token permutation, so the MFMA k-sums are exact.
namespace pp {
constexpr int kBK = 64;                        // tokens per K-tile
constexpr int kHalfElems = 64 * 128;           // one half-tile image (16 KB)
constexpr size_t kLds = 8 * kHalfElems * 2;    // 128 KB

typedef WMF16<bf16>::e8 e8b;

template <typename T>
struct Regs {
  f32x4 acc[2][2][4][2];                       // [qa][qb][i][j]
  f32x4 accs[2];                               // CS 2: row sums of A, 16 rows (i = wn) per qa
  typename WMF16<T>::e8 fa[4][2];              // A fragments of the current qa: [i][k-step]
  typename WMF16<T>::e8 fb[2][2][2];           // B fragments: [qb][j][k-step]
};

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// fragment (8 elements) from two transposed reads r = 0, 1 at element offsets off, off + 2048
template <typename T>
__device__ __forceinline__ typename WMF16<T>::e8 frag(const uint16_t* base) {
  return ld_tr16<T>(base, 0, 2048);
}

struct Geo {
  int lbA[2], lbB[2];    // per-lane element offsets of the transposed reads, by block parity
  uint32_t vA[2][2];     // staging byte offsets [half qa][quad u] relative to the tile's first token row
  uint32_t vB[2][2];
};

// MFMAs of quadrant (QA, QB): 2 k-steps x 4 i x 2 j
template <typename T, int QA, int QB>
__device__ __forceinline__ void mfma_quadrant(Regs<T>& R, bool act, bool cs_quad,
                                              const typename WMF16<T>::e8& ones) {
  if (act) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          R.acc[QA][QB][i][j] = WMF16<T>::mma(R.fa[i][s], R.fb[QB][j][s], R.acc[QA][QB][i][j]);
    __builtin_amdgcn_s_setprio(0);
  } else if (cs_quad) {
    // bias-gradient quadrant: B = ones -> every column of acc[QA][QB][i][0] = sum over tokens of A
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) R.acc[QA][QB][i][0] = WMF16<T>::mma(R.fa[i][s], ones, R.acc[QA][QB][i][0]);
    __builtin_amdgcn_s_setprio(0);
  }
}

// CS 2 (any K, e.g. K % 256 == 0 where no quadrant idles): in the last K tile's workgroups each
// wave also multiplies ONE of its four A fragments of the phase's fresh A half (i = wave column)
// by the ones fragment -- 2 extra MFMAs in phases 0 and 2, spread over the four wave columns.
template <typename T, int QA>
__device__ __forceinline__ void mfma_rowsum(Regs<T>& R, int wn, const typename WMF16<T>::e8& ones) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    // wn is wave-uniform (SGPR): a scalar branch selects the fragment, no dynamic register index
    if (wn == 0)
      R.accs[QA] = WMF16<T>::mma(R.fa[0][s], ones, R.accs[QA]);
    else if (wn == 1)
      R.accs[QA] = WMF16<T>::mma(R.fa[1][s], ones, R.accs[QA]);
    else if (wn == 2)
      R.accs[QA] = WMF16<T>::mma(R.fa[2][s], ones, R.accs[QA]);
    else
      R.accs[QA] = WMF16<T>::mma(R.fa[3][s], ones, R.accs[QA]);
  }
  __builtin_amdgcn_s_setprio(0);
}

// One phase P (0..3) of a tile whose slots are set PAR (0, 1).  ISSUE: stage half-tile P of
// the next tile into set PAR ^ 1.  VM: the counted wait ending the load segment.
// CS: 0 no bias gradient, 1 idle-quadrant row sums (K % 256 in [1, 128]), 2 extra row-sum MFMAs.
template <typename T, int CS, int P, int PAR, int VM_ISSUE, int VM_LAST>
__device__ __forceinline__ void phase(Regs<T>& R, const Geo& G, const uint16_t* smem, const uint16_t* nxtA,
                                      const uint16_t* nxtB, bool issue, int wave, const bool (&act)[2][2],
                                      bool cs_q1, const typename WMF16<T>::e8& ones) {
  constexpr int QA = (P == 0 || P == 1) ? 0 : 1;
  constexpr int QB = (P == 0 || P == 3) ? 0 : 1;
  const uint16_t* set = smem + PAR * 4 * kHalfElems;
  // ---- load segment
  if (P == 0 || P == 2) {  // A half QA: 4 m-tiles x 2 k-steps
    const uint16_t* sa = set + (P == 0 ? 0 : 3) * kHalfElems;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) R.fa[i][s] = frag<T>(sa + G.lbA[i & 1] + s * 4096 + i * 64);
  }
  if (P == 0 || P == 1) {  // B half QB: 2 n-tiles x 2 k-steps (qb 0 is kept for phase 3)
    const uint16_t* sb = set + (P == 0 ? 1 : 2) * kHalfElems;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) R.fb[QB][j][s] = frag<T>(sb + G.lbB[j & 1] + s * 4096 + j * 64);
  }
  if (issue) {
    uint16_t* dst = const_cast<uint16_t*>(smem) + ((PAR ^ 1) * 4 + P) * kHalfElems + (2 * wave) * 512;
    const uint16_t* src = (P == 0 || P == 3) ? nxtA : nxtB;
    const uint32_t v0 = P == 0 ? G.vA[0][0] : P == 3 ? G.vA[1][0] : P == 1 ? G.vB[0][0] : G.vB[1][0];
    const uint32_t v1 = P == 0 ? G.vA[0][1] : P == 3 ? G.vA[1][1] : P == 1 ? G.vB[0][1] : G.vB[1][1];
    lds_dma16_sv(src, v0, dst);
    lds_dma16_sv(src, v1, dst + 512);
  }
  if (issue)
    wait_vm<VM_ISSUE>();
  else
    wait_vm<VM_LAST>();
  bar();
  // ---- MFMA segment
  mfma_quadrant<T, QA, QB>(R, act[QA][QB], CS == 1 && QB == 1 && cs_q1 && act[QA][0], ones);
  if constexpr (CS == 2 && (P == 0 || P == 2)) {
    if (cs_q1 && act[QA][0]) mfma_rowsum<T, QA>(R, wave & 3, ones);
  }
  bar();
}

// a whole tile; issue: there is a next tile to stage (else this is the last tile)
template <typename T, int CS, int PAR>
__device__ __forceinline__ void tile(Regs<T>& R, const Geo& G, const uint16_t* smem, const uint16_t* nxtA,
                                     const uint16_t* nxtB, bool issue, int wave, const bool (&act)[2][2],
                                     bool cs_q1, const typename WMF16<T>::e8& ones) {
  // counted waits (2 LDS-DMA pieces per wave per phase): what the NEXT phase reads must have
  // landed, the youngest issues may stay in flight
  phase<T, CS, 0, PAR, 4, 2>(R, G, smem, nxtA, nxtB, issue, wave, act, cs_q1, ones);
  phase<T, CS, 1, PAR, 4, 0>(R, G, smem, nxtA, nxtB, issue, wave, act, cs_q1, ones);
  phase<T, CS, 2, PAR, 6, 0>(R, G, smem, nxtA, nxtB, issue, wave, act, cs_q1, ones);
  phase<T, CS, 3, PAR, 4, 0>(R, G, smem, nxtA, nxtB, issue, wave, act, cs_q1, ones);
}
}  // namespace pp

template <typename T, int CS>
__global__ __launch_bounds__(512, 2) void wgrad_pp_kernel(const uint16_t* __restrict__ A,
                                                          const uint16_t* __restrict__ B, float* __restrict__ ws,
                                                          int64_t Tn, int N, int K, int64_t lda, int64_t ldb,
                                                          int64_t t_split, float* __restrict__ cs) {
  using namespace pp;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tiles_n = (N + TM - 1) / TM, tiles_k = (K + TN - 1) / TN;
  int split, tn, tk;
  wg_map(tiles_n, tiles_k, 1, split, tn, tk);
  const int64_t t_begin = split * t_split;
  const int64_t t_end = t_begin + t_split < Tn ? t_begin + t_split : Tn;
  const int64_t ntiles = t_end > t_begin ? (t_end - t_begin) / kBK : 0;
  const int n0 = tn * TM, k0 = tk * TN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  Geo G;
  {
    // transposed reads: lane 4q + p of group g -> token row q of quad (.. + g), columns 4p..4p+3
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, gb = g & 1;
    const int common = g * 1024 + q * 32 + p * 8;  // bytes
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int adj = gb ? (par ? -128 : 128) : 0;  // block index XOR (quad & 1)
      G.lbA[par] = (wm * 4 * 128 + adj + common) / 2;
      G.lbB[par] = (wn * 2 * 128 + adj + common) / 2;
    }
    // staging: lane -> (physical block b, token tq, 8-column piece ch) of quad 2 * wave + u
    const int b = lane >> 3, tq = (lane >> 1) & 3, ch = lane & 1;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = (2 * wave + u) * 4 + tq;
      const int col = ((b ^ u) * 16 + ch * 8);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ca = min(n0 + h * 128 + col, N - 8);
        const int cb = min(k0 + h * 128 + col, K - 8);
        G.vA[h][u] = static_cast<uint32_t>((row * static_cast<int64_t>(lda) + ca) * 2);
        G.vB[h][u] = static_cast<uint32_t>((row * static_cast<int64_t>(ldb) + cb) * 2);
      }
    }
  }
  bool act[2][2];
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) act[qa][qb] = (n0 + qa * 128 + wm * 64 < N) && (k0 + qb * 128 + wn * 32 < K);
  // bias-gradient quadrant: the last K tile with no valid column past 128 -> wave column 0
  // turns its (qa, 1) quadrants into row sums of A
  // (CS 2: every wave of the last K tile's workgroups sums its 16 rows i = wn of each A half)
  const bool cs_q1 = CS == 1 ? (wn == 0 && tk == tiles_k - 1 && K - k0 <= 128) : (CS == 2 && tk == tiles_k - 1);

  Regs<T> R;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) R.acc[a][b2][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  R.accs[0] = R.accs[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  typename WMF16<T>::e8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = 1.0f;

  if (ntiles > 0) {
    const uint16_t* a0 = A + t_begin * lda;
    const uint16_t* b0 = B + t_begin * ldb;
    const int64_t stepA = kBK * lda, stepB = kBK * ldb;
    // prologue: tile 0's four halves into set 0; halves 0 and 1 (read first) must land
    {
      uint16_t* s0 = smem + (2 * wave) * 512;
      lds_dma16_sv(a0, G.vA[0][0], s0);
      lds_dma16_sv(a0, G.vA[0][1], s0 + 512);
      lds_dma16_sv(b0, G.vB[0][0], s0 + kHalfElems);
      lds_dma16_sv(b0, G.vB[0][1], s0 + kHalfElems + 512);
      lds_dma16_sv(b0, G.vB[1][0], s0 + 2 * kHalfElems);
      lds_dma16_sv(b0, G.vB[1][1], s0 + 2 * kHalfElems + 512);
      lds_dma16_sv(a0, G.vA[1][0], s0 + 3 * kHalfElems);
      lds_dma16_sv(a0, G.vA[1][1], s0 + 3 * kHalfElems + 512);
      wait_vm<4>();
    }
    bar();
    if (wm == 1) bar();  // row 1 runs one barrier behind row 0
    for (int64_t t = 0; t < ntiles; t += 2) {
      tile<T, CS, 0>(R, G, smem, a0 + (t + 1) * stepA, b0 + (t + 1) * stepB, t + 1 < ntiles, wave, act, cs_q1,
                     ones);
      if (t + 1 < ntiles)
        tile<T, CS, 1>(R, G, smem, a0 + (t + 2) * stepA, b0 + (t + 2) * stepB, t + 2 < ntiles, wave, act, cs_q1,
                       ones);
    }
    if (wm == 0) bar();  // balance row 1's extra barrier
  }

  // fp32 partial tile of this split; lane l holds C[4 (l / 16) + r][l % 16] of each 16 x 16 tile
  float* out = ws + static_cast<int64_t>(split) * N * K;
  const int col_l = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = k0 + qb * 128 + wn * 32 + j * 16 + col_l;
        if (k >= K) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int nb = n0 + qa * 128 + wm * 64 + i * 16 + rq;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nb + r < N) out[static_cast<int64_t>(nb + r) * K + k] = R.acc[qa][qb][i][j][r];
        }
      }
  if (CS == 2 && cs_q1 && col_l == 0) {
    float* cso = cs + static_cast<int64_t>(split) * N;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      const int nb = n0 + qa * 128 + wm * 64 + wn * 16 + rq;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nb + r < N) cso[nb + r] = R.accs[qa][r];
    }
  }
  if (CS == 1 && cs_q1 && col_l == 0) {
    float* cso = cs + static_cast<int64_t>(split) * N;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nb = n0 + qa * 128 + wm * 64 + i * 16 + rq;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nb + r < N) cso[nb + r] = R.acc[qa][1][i][0][r];
      }
  }
}

template <typename T, int CS>
int launch_pp(const uint16_t* pa, const uint16_t* pb, float* ws, int64_t tokens, int n, int k, int64_t lda,
              int64_t ldb, int64_t t_split, int grid, hipStream_t s, float* cs) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<T, CS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(pp::kLds));
    attr_set = true;
  }
  wgrad_pp_kernel<T, CS><<<grid, 512, pp::kLds, s>>>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, cs);
  return 0;
}

// the ping-pong kernel's bias-gradient quadrant exists for this K
__host__ __device__ __forceinline__ bool wgrad_pp_cs_ok(int K) { return K % 256 != 0 && K % 256 <= 128; }

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
  // eight partial rows in flight at a time, added in order (deterministic)
  for (int p = 0; p < splits; p += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p + j < splits ? cs[static_cast<int64_t>(p + j) * n + i] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) a += v[j];
  }
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
          int bias_accumulate, int impl) {
  // whole 64-token tiles only (the caller adds the token remainder)
  if (n % 8 != 0 || k % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || splits < 1 || tokens % TK != 0) return -1;
  if (bias != nullptr && (dt != BF16 || cs == nullptr)) return -3;  // column sums: bf16 operands
  const int tiles = ((n + TM - 1) / TM) * ((k + TN - 1) / TN);
  int64_t t_split = (tokens + splits - 1) / splits;
  t_split = (t_split + TK - 1) / TK * TK;
  const int grid = tiles * splits;
  const auto* pa = static_cast<const uint16_t*>(a);
  const auto* pb = static_cast<const uint16_t*>(b);
  // SMP_WGRAD_IMPL=glds keeps the round-4 one-barrier-per-tile kernel (A/B); the ping-pong
  // kernel needs 32-bit staging offsets and, for a fused bias gradient, its ones quadrant
  static const bool env_glds = [] {
    const char* e = getenv("SMP_WGRAD_IMPL");
    return e != nullptr && strcmp(e, "glds") == 0;
  }();
  const bool use_glds = impl == 0 || (impl < 0 && env_glds);
  // a bias gradient: idle-quadrant sums where K % 256 leaves a quadrant idle; the row-sum MFMA
  // mode for other K only on request (impl 2, or SMP_WGRAD_PP_CS=rowsum: it slows every
  // workgroup of the kernel, profiles/r6/wgrad_rowsum_bias.md), else the round-4 kernel
  static const bool env_rowsum = [] {
    const char* e = getenv("SMP_WGRAD_PP_CS");
    return e != nullptr && strcmp(e, "rowsum") == 0;
  }();
  const bool rowsum_ok = impl == 2 || env_rowsum;
  const bool pp_ok = !use_glds && lda < (1 << 24) && ldb < (1 << 24) &&
                     (bias == nullptr || wgrad_pp_cs_ok(k) || rowsum_ok);
  if (pp_ok) {
    if (bias != nullptr && wgrad_pp_cs_ok(k))
      launch_pp<bf16, 1>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, cs);
    else if (bias != nullptr)
      launch_pp<bf16, 2>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, cs);
    else if (dt == BF16)
      launch_pp<bf16, 0>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, nullptr);
    else if (dt == F16)
      launch_pp<f16, 0>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, nullptr);
    else
      return -2;
  } else if (bias != nullptr || dt == BF16)
    launch_glds16<bf16, kTK, kNS>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s, cs);
  else if (dt == F16)
    launch_glds16<f16, kTK, kNS>(pa, pb, ws, tokens, n, k, lda, ldb, t_split, grid, s);
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
    const int parts = splits * ((pp_ok || wgrad_cs_idle(k)) ? 1 : (k + TN - 1) / TN);
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
