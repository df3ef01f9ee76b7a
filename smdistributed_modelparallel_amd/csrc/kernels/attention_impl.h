// Flash-style fused attention for CDNA4 (gfx950): forward, and backward as two kernels
// (dK/dV per key block, dQ per query block -- no fp32 atomics, bitwise reproducible).
//
// Replaces the reference's materialised-score path (QK^T GEMM -> fused softmax ->
// dropout -> PV GEMM, `smp/torch/nn/transformer.py:1617-1835`, capped at sk <= 2048):
// no [s, s] tensor is ever written, causal blocks above the diagonal are skipped, and
// there is no sequence-length cap.
//
// Layout of the MFMA work (v_mfma_f32_32x32x16_{bf16,f16}, wave64):
//  * forward / dQ: each wave owns 32 queries.  Scores are computed TRANSPOSED,
//    S^T = K Q^T, so a lane holds 16 keys of ONE query (its lane & 31): the online-softmax
//    row max / row sum are lane-local plus one cross-half (lane ^ 32) exchange.  The
//    probability accumulator is then directly the B operand of O^T = V^T P^T (k order of
//    the accumulator rows handled by the A-operand fetch), whose output again has the
//    query on the lane -- the rescale by exp(m_old - m_new) is lane-local, no shuffles.
//  * V^T / K^T / dO^T / Q^T operands are fetched with ds_read_b64_tr_b16 (hardware
//    transpose) from row-major LDS tiles; row-major operands with ds_read_b128.
//  * dK/dV: each wave owns 32 keys with the key on the lane (S = Q K^T, dP = dO V^T); P and
//    dS accumulators are the B operands of dV^T = dO^T P and dK^T = Q^T dS.
//  * LDS rows are padded by 16 B (register staging), which makes the 16-byte row reads
//    conflict-free.
// 256 threads (4 waves) per block; 128 queries (fwd, dQ) or 128 keys (dK/dV) per block,
// 64-wide tiles along the reduction axis.  Causal q-blocks are launched heaviest first.
//
// Variants (template flags, one instantiation set per head dim in attention_d*.hip):
//  * BIAS: additive per-key bias [b, sk] (padding masks; reference mask semantics
//    `smp/torch/nn/transformer.py:403-409,1680-1708`), folded into the score MFMA's initial
//    accumulator (bias / scale), so it costs no VALU work per score.
//  * DROP: attention dropout generated in-kernel from a counter-based hash of
//    (seed, offset, b*h, query, key) -- the backward regenerates exactly the same mask, no
//    [s, s] mask tensor exists.  A 32-bit hash serves a key PAIR (16-bit uniform each).
//    The row sums use the undropped P (softmax normalisation), the P.V operand the kept
//    entries, and 1/(1-p) is applied once to O.  Backward: dV = (P o Z)^T dO and
//    dS = P o (Z o dP - delta) with Z = keep / (1 - p); delta = rowsum(dO o O) is unchanged.
//  * head dims 64, 96, 128, 256.  D = 96 uses a 128-element LDS row stride (swizzle needs a
//    power-of-two chunk count) but runs 6 / 3 MFMA k-steps / tiles, not 8 / 4.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace smpk {
namespace attn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct MF;
template <>
struct MF<bf16> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ __bf16 cvt(float x) { return static_cast<__bf16>(x); }
};
template <>
struct MF<f16> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ _Float16 cvt(float x) { return static_cast<_Float16>(x); }
};

constexpr float kLog2e = 1.4426950408889634f;

constexpr int kThreads = 256;

// LDS row stride (elements) for head dim D
template <int D>
struct LdsStride {
  static constexpr int v = D == 96 ? 128 : D;
};

// ---------------------------------------------------------------- dropout hash
// lowbias32 (a bijective 32-bit mixer): distinct (query, key-quad) inputs under one key give
// distinct outputs; byte i of mix32(key ^ (q * nquads + k / 4)) is the 8-bit uniform of key
// 4 (k / 4) + i.  One hash serves four keys (FlashAttention-style 8-bit dropout decisions).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Per-byte keep test without unpacking: bit 8i+7 of the result is set iff byte i of h is
// >= drop_thr.  thr <= 128 (xr = 0, c = (128 - thr) x 0x01010101): a byte >= 128 is kept, a
// smaller one carries into its bit 7 iff b + 128 - thr >= 128 (no carry leaves the byte).
// thr > 128 (xr = ~0): the same test on the complemented bytes with 256 - thr, negated.
__device__ __forceinline__ uint32_t keep_flags(uint32_t h, uint32_t xr, uint32_t c) {
  const uint32_t hx = h ^ xr;
  return (((hx & 0x7f7f7f7fu) + c) | hx) ^ xr;
}

// all-ones iff bit `bit` of f is set (v_bfe_i32)
__device__ __forceinline__ uint32_t bit_mask(uint32_t f, uint32_t bit) {
  return static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(f), bit, 1u));
}


__device__ __forceinline__ float and_mask(float x, uint32_t m) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & m);
}

__device__ __forceinline__ uint32_t drop_key(const AttnParams& p, int64_t bh) {
  const uint32_t s0 = static_cast<uint32_t>(p.seed), s1 = static_cast<uint32_t>(p.seed >> 32);
  const uint32_t o0 = static_cast<uint32_t>(p.offset), o1 = static_cast<uint32_t>(p.offset >> 32);
  return mix32(s0 ^ mix32(s1 + 0x9e3779b9u * static_cast<uint32_t>(bh + 1)) ^ mix32(o0 ^ mix32(o1 + 0x85ebca6bu)));
}

// Exact drop rate from 8-bit uniforms: each 32-query x 32-key block of one (b, h) draws its
// threshold from {thr, thr + 1} with P(thr + 1) = frac / 65536 (one hash per block, keyed by
// mix32(key + C) so it is independent of the element hashes), so every element's drop
// probability is (thr + frac / 65536) / 256 = dropout_p to 2^-24; elements sharing a block
// are correlated by < 2e-4.  Block indices are wave-uniform in all three kernels (the fwd / dQ
// wave owns one query block, the dK/dV wave one key block), so this runs on the scalar unit.
struct DropThr {
  uint32_t xr, c;
};
__device__ __forceinline__ uint32_t drop_block_key(uint32_t dkey) { return mix32(dkey + 0x632be5abu); }
__device__ __forceinline__ DropThr drop_block_thr(const AttnParams& p, uint32_t bkey, uint32_t qb32, uint32_t kb32) {
  const uint32_t nkb = static_cast<uint32_t>((p.sk + 31) >> 5);
  const bool hi = (mix32(bkey ^ (qb32 * nkb + kb32)) & 0xffffu) < p.drop_frac;
  return DropThr{hi ? p.drop_xr1 : p.drop_xr, hi ? p.drop_c1 : p.drop_c};
}

// floor(a / b) for b > 0 and any sign of a
__device__ __forceinline__ int fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// Lazy online softmax: the exponent offset (running row max) only moves when a tile's max
// exceeds it by more than kTau (log2 units), so stored probabilities stay <= 2^kTau (fp32
// sums, bf16 / fp16 PV operands: no overflow) and the O / l rescale runs on a few tiles per
// row instead of on almost every tile.
constexpr float kTau = 8.f;

template <typename T>
__device__ __forceinline__ typename MF<T>::e8 ld8(const uint16_t* p) {
  return __builtin_bit_cast(typename MF<T>::e8, *reinterpret_cast<const s16x8*>(p));
}

// ------------------------------------------------------- XCD-aware block mapping
// Workgroups are dealt round-robin to the 8 XCDs (each with its own 4 MB L2).  A 1-D grid
// of tiles x (b*h) blocks is mapped so that all tiles of one (b, h) run on the SAME XCD,
// consecutively: their shared K/V (fwd, dQ) or Q/dO (dK/dV) tiles stay L2-resident
// instead of being fetched by all 8 XCDs.  Heads beyond the last multiple of 8 fall back
// to the linear order.
__device__ __forceinline__ void xcd_map(int ntiles, int64_t nbh, int& tile, int64_t& bh) {
  const int64_t L = blockIdx.x;
  const int64_t full = (nbh / 8) * 8 * ntiles;
  if (L < full) {
    const int64_t xcd = L % 8, j = L / 8;
    bh = xcd + 8 * (j / ntiles);
    tile = static_cast<int>(j % ntiles);
  } else {
    const int64_t r = L - full;
    bh = (nbh / 8) * 8 + r / ntiles;
    tile = static_cast<int>(r % ntiles);
  }
}

// ------------------------------------------------------------------ LDS tiles
// Tiles are stored unpadded, [rows][D] bf16, with the 16-byte chunks of each row XOR-
// swizzled so that BOTH access patterns are bank-conflict free:
//  * row reads (ds_read_b128, lane = row, 16 rows per LDS cycle group), and
//  * transposed reads (ds_read_b64_tr_b16: 4 rows x 32 columns per 32-lane group).
// D = 64 (128-B rows, two rows per 64-bank line): chunk' = chunk ^ (bit1(row)<<2 | bits2-3(row)).
// D = 128 (256-B rows, one row per line):        chunk' = chunk ^ (bits0-1(row)<<2 | bits2-3(row)).
// D >= 128 rows (and D = 96 stored at stride 128): chunk' = chunk ^ (bits0-1(row)<<2 | bits2-3(row)).
template <int D>
__device__ __forceinline__ int swz(int row, int chunk) {
  constexpr int DS = LdsStride<D>::v;
  const int g = DS == 64 ? ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)) : (((row & 3) << 2) | ((row >> 2) & 3));
  return row * DS + ((chunk ^ g) << 3);
}

// Per-lane LDS element offsets, swizzle resolved ONCE per kernel (the swizzle depends on
// row bits 0-3 only, so rows +16/+32/+64 are immediate offsets of these bases).
//  * RowOff: A/B operand row reads -- row (lane & 31) [+32 j], chunk 2t + (lane >> 5);
//  * TrOff: transposed reads -- lane 4q+p of each 16-lane group supplies row q (and q + 8)
//    at columns c0 + 4p..4p+3, c0 = 32 i + 16 * bit4(lane), rows based at 4 * (lane >> 5).
template <int D>
struct RowOff {
  int o[D / 16];
  __device__ __forceinline__ RowOff(int r, int hh) {
#pragma unroll
    for (int t = 0; t < D / 16; ++t) o[t] = swz<D>(r, 2 * t + hh);
  }
};

template <int D, int NI = D / 32>
struct TrOff {
  int lo[NI], hi[NI];
  // col0: first output column (dK/dV split into column halves for D = 256)
  __device__ __forceinline__ explicit TrOff(int lane, int col0 = 0) {
    const int q = (lane & 15) >> 2, pp = lane & 3, hh = lane >> 5;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int col = col0 + 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
      lo[i] = swz<D>(4 * hh + q, col >> 3) + (col & 7);
      hi[i] = swz<D>(4 * hh + 8 + q, col >> 3) + (col & 7);
    }
  }
};

// Transposed fetch: elements j=0..3 <- rows k0..k0+3, j=4..7 <- rows k0+8..k0+11 (k0 folded
// into the offsets), one ds_read_b64_tr_b16 per half.
template <typename T>
__device__ __forceinline__ typename MF<T>::e8 ld_tr(const uint16_t* tile, int off_lo, int off_hi) {
  s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_lo));
  s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(tile + off_hi));
  s16x8 v = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  return __builtin_bit_cast(typename MF<T>::e8, v);
}

// Accumulator rows 8s..8s+7 -> one 8-element operand fragment (k-step s of a 32-row tile).
template <typename T>
__device__ __forceinline__ typename MF<T>::e8 pack8(const f32x16& a, int s) {
  typename MF<T>::e8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = MF<T>::cvt(a[8 * s + j]);
  return r;
}

// The same from the register pairs (2j, 2j + 1) of a pair array: one v_cvt_pk per pair, no
// cross-pair shuffles (element-wise code written on f32x2 pairs keeps hipcc's packed fp32 ops
// and the conversions on the same pairing)
template <typename T>
__device__ __forceinline__ typename MF<T>::e8 pack8p(const f32x2 (&a)[8], int s) {
  typename MF<T>::e8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[2 * j] = MF<T>::cvt(a[4 * s + j].x);
    r[2 * j + 1] = MF<T>::cvt(a[4 * s + j].y);
  }
  return r;
}

__device__ __forceinline__ int acc_row(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Row max of MFMA results: builtin fmaxf, which hipcc lowers to v_max3_f32 AND pads with
// the XDL->VALU wait states (an inline-asm v_max3 reading the accumulators directly is not
// padded by the compiler and read stale values on some waves -- non-deterministic maxima).
__device__ __forceinline__ float max3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }

// value of lane ^ 32 (the other half-wave) without an LDS round trip.  The lane select is
// needed: with both operands the same value, hipcc may give the swap one register, and then
// each output holds only the OTHER half's value (measured: max / sum over r[0], r[1] without
// the select returned 2x the other half's sum -- wrong softmax normalisers).
__device__ __forceinline__ float xor32(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const int lane = threadIdx.x & 63;
  return __builtin_bit_cast(float, lane < 32 ? r[1] : r[0]);
}
// max / sum of x over the lane pair (lane, lane ^ 32)
__device__ __forceinline__ float pair_max32(float x) { return fmaxf(x, xor32(x)); }
__device__ __forceinline__ float pair_sum32(float x) { return x + xor32(x); }

// Register-staged tile copy (issue global loads early, write LDS late: the HBM/L2 latency
// hides under the MFMA work of the current tile).
template <int D, int ROWS>
struct Stage {
  static constexpr int CH = D / 8;
  static constexpr int N = ROWS * CH / kThreads;
  static_assert(N * kThreads == ROWS * CH, "tile must split evenly over the block");
  // rows advance by RS per register; when RS is a multiple of 16 the swizzle pattern (row
  // bits 0-3) repeats and every LDS / global offset is base + compile-time/scalar step, so
  // only one lane offset pair lives in VGPRs (D = 64, 128); D = 256 (RS = 8) alternates two
  // patterns; D = 96 keeps per-register offsets.
  static constexpr int RS = (kThreads % CH == 0) ? kThreads / CH : 0;
  static constexpr int NB = (RS > 0 && RS % 16 == 0) ? 1 : ((RS > 0 && (2 * RS) % 16 == 0) ? 2 : N);
  uint4 v[N];
  int goff0, row0;
  int loffb[NB];
  int goffa[RS > 0 ? 1 : N], rowa[RS > 0 ? 1 : N];
  int64_t gs_;
  __device__ __forceinline__ explicit Stage(int64_t gs) : gs_(gs) {
    if constexpr (RS > 0) {
      const int r = threadIdx.x / CH, k = threadIdx.x % CH;
      row0 = r;
      goff0 = static_cast<int>(r * gs) + k * 8;
#pragma unroll
      for (int i = 0; i < NB; ++i) loffb[i] = swz<D>(r + i * RS, k);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int c = threadIdx.x + i * kThreads, r = c / CH, k = c % CH;
        rowa[i] = r;
        goffa[i] = static_cast<int>(r * gs) + k * 8;
        loffb[i] = swz<D>(r, k);
      }
    }
  }
  __device__ __forceinline__ int goff(int i) const {
    if constexpr (RS > 0)
      return goff0 + static_cast<int>(i * RS * gs_);
    else
      return goffa[i];
  }
  __device__ __forceinline__ int row(int i) const {
    if constexpr (RS > 0)
      return row0 + i * RS;
    else
      return rowa[i];
  }
  __device__ __forceinline__ int loff(int i) const {
    constexpr int DS = LdsStride<D>::v;
    if constexpr (RS > 0)
      return loffb[i % NB] + (i / NB) * NB * RS * DS;
    else
      return loffb[i];
  }
  // tile: pointer to the tile's first row; rows >= valid read as zeros
  __device__ __forceinline__ void load(const uint16_t* tile, int valid) {
    if (valid >= ROWS) {  // wave-uniform: interior tiles load without per-lane predication
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = *reinterpret_cast<const uint4*>(tile + goff(i));
      return;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      v[i] = row(i) < valid ? *reinterpret_cast<const uint4*>(tile + goff(i)) : make_uint4(0, 0, 0, 0);
  }
  __device__ __forceinline__ void store(uint16_t* lds) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + loff(i)) = v[i];
  }
};

template <typename T, int D, int NI = D / 32>
__device__ __forceinline__ void store_rows(uint16_t* dst, const f32x16* acc, float mul, int hh) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * i + 8 * g + 4 * hh;
      s16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = __builtin_bit_cast(short, MF<T>::cvt(acc[i][4 * g + j] * mul));
      *reinterpret_cast<s16x4*>(dst + d0) = w;
    }
  }
}

// Issues the load of a tile's raw bias value (thread t < 64 holds key kv0 + t).  The value is
// consumed (scaled, stored to LDS) only at the next tile's staging, like the K/V registers:
// using it right away would make wave 0 wait out the global-load latency every tile.
__device__ __forceinline__ float load_bias(const AttnParams& p, int64_t b, int key) {
  return key < p.sk ? p.kbias[b * p.kbias_sb + key] : 0.f;
}

// Adds the staged bias of each register's key to a transposed score tile (key rows in
// registers), 4 consecutive keys per float4 (acc_row(4g..4g+3) = 8g + 4hh + 0..3).  Applied
// after the score MFMAs and only on tiles that carry a bias: the MFMA chains keep their
// zero / row-constant initial accumulators (a runtime choice of initial accumulator would
// cost 32 register moves per tile on every tile).
__device__ __forceinline__ void add_from_keys(f32x16& a, const float* sB, int hh) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 v = *reinterpret_cast<const float4*>(&sB[8 * g + 4 * hh]);
    a[4 * g + 0] += v.x;
    a[4 * g + 1] += v.y;
    a[4 * g + 2] += v.z;
    a[4 * g + 3] += v.w;
  }
}

// Publishes whether the tile being stored carries any nonzero bias: wave 0 holds the 64
// staged values (thread t = key kv0 + t), one ballot, one LDS word; read after the barrier.
// An all-zero bias (e.g. an all-ones padding mask) then costs only the 256-byte staging.
__device__ __forceinline__ void publish_bias_flag(float bstage, int* sFlag) {
  if (threadIdx.x < 64) {
    const bool any = __any(bstage != 0.f);
    if (threadIdx.x == 0) *sFlag = any ? 1 : 0;
  }
}

// Dropout keep words of a transposed tile (query on the lane, 16 keys in registers starting
// at key `kbase`, a multiple of 32): register group g (registers 4g..4g+3) holds keys
// kbase + 8g + 4hh + 0..3 = key quad kbase/4 + 2g + hh, whose keep flags are bits 7, 15, 23,
// 31 of f[g] (keep_flags of the quad's hash).
__device__ __forceinline__ void drop_words(uint32_t (&f)[4], uint32_t key, uint32_t qbase, int kbase, int hh,
                                           uint32_t xr, uint32_t c) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint32_t kq = static_cast<uint32_t>(kbase >> 2) + static_cast<uint32_t>(2 * g + hh);
    f[g] = keep_flags(mix32(key ^ (qbase + kq)), xr, c);
  }
}

// Element i of a keep word as an all-ones / zero 32-bit mask, by v_perm_b32's sign-replicating
// selectors (8: bit 15 of src1, 9: bit 31 of src1, 10: bit 15 of src0, 11: bit 31 of src0) on
// (f, f << 8): flag bits 7 / 23 sit at 15 / 31 of the shifted word.
__device__ __forceinline__ uint32_t elem_mask(uint32_t f, uint32_t sh, int i) {
  constexpr uint32_t kSel[4] = {0x08080808u, 0x0A0A0A0Au, 0x09090909u, 0x0B0B0B0Bu};
  return __builtin_amdgcn_perm(f, sh, kSel[i]);
}

// Zero the dropped entries of a packed MFMA operand (8 bf16/f16 = registers 8 half .. +7 =
// groups 2 half, 2 half + 1): one v_perm mask per element pair, applied with one AND.
template <typename E>
__device__ __forceinline__ E drop_packed(E v, uint32_t f0, uint32_t f1) {
  u32x4 w = __builtin_bit_cast(u32x4, v);
  const uint32_t s0 = f0 << 8, s1 = f1 << 8;
  w[0] &= __builtin_amdgcn_perm(f0, s0, 0x0A0A0808u);  // elements 0, 1 of group 2 half
  w[1] &= __builtin_amdgcn_perm(f0, s0, 0x0B0B0909u);  // elements 2, 3
  w[2] &= __builtin_amdgcn_perm(f1, s1, 0x0A0A0808u);  // group 2 half + 1
  w[3] &= __builtin_amdgcn_perm(f1, s1, 0x0B0B0909u);
  return __builtin_bit_cast(E, w);
}


// ------------------------------------------------------------ stored keep bits
// The forward hashes each element's dropout decision once and stores it as 1 bit: per (b h,
// query row q, 64-key tile t, half-wave hh) one uint32 at ((bh * ntiles + t) * sq + q) * 2 + hh
// holding the decisions of exactly the 32 keys a query-on-lane wave's lane holds (keys
// 64 t + 32 s + acc_row(reg, hh), at bit drop_bit(s, reg)), so the forward writes and dQ
// reads one coalesced dword per lane per tile, and dK/dV stages a block's words through LDS.
// The backward then never regenerates the hash (~100 VALU per 64-key tile per lane).
__device__ __forceinline__ int64_t bits_index(int64_t bh, int ntiles, int tile, int sq, int q, int hh) {
  return ((bh * ntiles + tile) * static_cast<int64_t>(sq) + q) * 2 + hh;
}

// The keep flags of the lane's tile from its stored word (the inverse of pack_keep): the flags
// of register group g of half s sit at bits 8 i + 7 of w << (g + 4 s) -- the bits at other
// positions are ignored by drop_packed's v_perm selectors, so no masking is needed.
__device__ __forceinline__ void unpack_keep(uint32_t w, uint32_t (&f0)[4], uint32_t (&f1)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    f0[g] = w << g;
    f1[g] = w << (4 + g);
  }
}

// The lane's 32 keep bits of a tile from the 8 keep words of its two 32-key halves: word g of
// half s keeps its flags at bits 7, 15, 23, 31 (element i at 8 i + 7); shifted right by g + 4 s
// they interleave without overlap, so register reg = 4 g + i of half s is bit
// drop_bit(s, reg) = 8 i + 7 - g - 4 s (one shift + and-or per word).
__device__ __forceinline__ constexpr uint32_t drop_bit(int s, int reg) {
  return static_cast<uint32_t>(8 * (reg & 3) + 7 - (reg >> 2) - 4 * s);
}
__device__ __forceinline__ uint32_t pack_keep(const uint32_t (&f0)[4], const uint32_t (&f1)[4]) {
  uint32_t w = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) w |= ((f0[g] & 0x80808080u) >> g) | ((f1[g] & 0x80808080u) >> (4 + g));
  return w;
}

// LDS-DMA of one K or V tile (BN rows x D, D = 64 / 128: the LDS image is exactly [BN][D]):
// each wave-instruction fills 1 KB = 1024 / (2 D) consecutive rows, lane-linear, so the
// row's XOR swizzle moves to the SOURCE chunk (physical chunk pc of row r holds logical
// chunk pc ^ g(r), g as in swz).  Rows at or past `sk` re-read row sk - 1 (finite data: the
// masked path gives those keys p = 0).
template <int D, int BN>
__device__ __forceinline__ void dma_tile(uint16_t* lds, const uint16_t* base, int64_t ss, int row0, int sk, int wave,
                                         int lane) {
  constexpr int CPR = D / 8, RPI = 64 / CPR, NI = BN / RPI;  // chunks/row, rows/instr, instrs/tile
  static_assert(NI % (kThreads / 64) == 0, "instructions split evenly over the waves");
  const int rl = lane / CPR, pc = lane % CPR;
  if (row0 + BN <= sk && ss < (1 << 24)) {
    // whole tile in range (wave-uniform): scalar tile base + loop-invariant lane offsets
    const uint16_t* tb = base + static_cast<int64_t>(row0) * ss;
#pragma unroll
    for (int i = 0; i < NI / (kThreads / 64); ++i) {
      const int rb = (wave * (NI / (kThreads / 64)) + i) * RPI;
      const int r = rb + rl;
      const int lc = (swz<D>(r, pc) - r * D) >> 3;
      lds_dma16_sv(tb, static_cast<uint32_t>((r * static_cast<int>(ss) + lc * 8) * 2), lds + rb * D);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < NI / (kThreads / 64); ++i) {
    const int rb = (wave * (NI / (kThreads / 64)) + i) * RPI;
    const int r = rb + rl;
    const int lc = (swz<D>(r, pc) - r * D) >> 3;  // chunk position of logical pc == pc ^ g(r)
    int gr = row0 + r;
    gr = gr < sk ? gr : sk - 1;
    lds_dma16(base + static_cast<int64_t>(gr) * ss + lc * 8, lds + rb * D);
  }
}

// ================================================================== forward
// Block = 4 waves x 32 queries; K/V tiles of 64 keys.  Interior tiles (every key visible
// to every query of the wave) take a mask-free path.
// D = 256: the wave's Q fragments (64 VGPRs) live in LDS instead of registers, so the O
// accumulator, the K/V prefetch and the softmax state fit one wave's register file.
template <int D>
struct QInLds {
  static constexpr bool v = D >= 256;
};

// DMA: K/V tiles arrive by LDS-DMA into two buffers (no staging registers, no ds_write, one
// barrier per tile); D = 64 / 128 without bias.
//
// Tile phases: every wave takes part in every tile's barrier (the block shares its K/V
// tiles) but runs the score work only on its visible tiles, and the per-element masks only on
// its edge tiles: the interior tiles run a separately compiled mask-free body.  (With one loop
// and a per-tile `if (!interior)`, hipcc if-converted the masks into ~100 VALU + ~100 SALU
// selects executed on every tile -- profiles/r4/attention_isa.md.)
// D = 64 DMA without dropout fits 128 VGPRs: 4 waves per SIMD instead of 3, -2 % (611 vs 624 us
// at GPT-2 XL shape); with dropout the same bound spills 35 registers and runs 2-3 % slower
// (profiles/r5/dropout_hash_ab.md)
template <typename T, int D, bool CAUSAL, bool DROP, bool BIAS, bool DMA = false>
__global__ void __launch_bounds__(kThreads, D >= 256 ? 1 : (D == 64 && DMA ? 4 : 2))
    attn_fwd_kernel(AttnParams p) {
  constexpr int BM = 128, BN = 64, DS = LdsStride<D>::v;
  constexpr bool QLDS = QInLds<D>::v;
  static_assert(!DMA || (!QLDS && !BIAS && DS == D && (D == 64 || D == 128)), "DMA variant: D 64 / 128, no bias");
  // K then V of each buffer (one array: a second LDS object beside DMA targets can make
  // hipcc drain vmcnt before ds_reads); DMA + dropout: then the two buffers' keep words (the
  // block's 128 queries x 2 halves = 256 words = 1 KB per tile, one LDS-DMA dword
  // instruction per wave)
  constexpr int KBW = BM * 2;  // keep words per block per tile
  constexpr bool BITS_LDS = DMA && DROP;
  __shared__ __attribute__((aligned(16))) uint16_t sKV[(DMA ? 4 : 2) * BN * DS + (BITS_LDS ? 2 * 2 * KBW : 0)];
  uint16_t* sK = sKV;
  uint16_t* sV = sKV + BN * DS;
  const uint32_t* sBits = reinterpret_cast<const uint32_t*>(sKV + 4 * BN * DS);
  __shared__ __attribute__((aligned(16))) uint16_t sQ[QLDS ? BM * DS : 8];
  __shared__ __attribute__((aligned(16))) float sB[BIAS ? BN : 4];
  __shared__ int sFlag;
  // wave index as a scalar: every wave-derived tile condition (causal / window / edge) then
  // branches on SGPRs instead of being if-converted into per-lane selects on every tile
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = static_cast<int>((p.sq + BM - 1) / BM);
  int tile;
  int64_t bh;
  xcd_map(nqb, p.b * p.h, tile, bh);
  const int64_t b = bh / p.h, h = bh % p.h;
  const int qb = CAUSAL ? (nqb - 1 - tile) : tile;  // heaviest causal blocks first
  const int q0 = qb * BM + wave * 32;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk);
  const int diag = sk - sq;  // key index allowed up to query + diag
  const int win = p.window;
  const int ntiles64 = (sk + 63) >> 6;

  const uint16_t* Q = static_cast<const uint16_t*>(p.q) + b * p.q_sb + h * p.q_sh;
  const uint16_t* K = static_cast<const uint16_t*>(p.k) + b * p.k_sb + h * p.k_sh;
  const uint16_t* V = static_cast<const uint16_t*>(p.v) + b * p.v_sb + h * p.v_sh;

  typename MF<T>::e8 qf[QLDS ? 1 : D / 16];
  const int qrow = q0 + r;
  if constexpr (QLDS) {
    // the block's 128 query rows -> swizzled LDS image (read back per MFMA like K)
    Stage<D, BM> stQ(p.q_ss);
    stQ.load(Q + static_cast<int64_t>(qb * BM) * p.q_ss, sq - qb * BM);
    stQ.store(sQ);
  } else {
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
      if (qrow < sq) {
        qf[t] = ld8<T>(Q + static_cast<int64_t>(qrow) * p.q_ss + 16 * t + 8 * hh);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[t][j] = MF<T>::cvt(0.f);
      }
    }
  }
  const float sl2 = p.scale * kLog2e;
  const float inv_scale = 1.f / p.scale;
  // m_i: exponent offset (lazy running max, log2 units), l_i: this lane's partial row sum
  float m_i = -INFINITY, m_use = 0.f, l_i = 0.f;
  f32x16 o[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) o[i] = f32x16{0};

  int kv_end = sk, kv_begin = 0;
  if (CAUSAL) {
    const int lim = (qb + 1) * BM + diag;
    kv_end = lim < sk ? lim : sk;
  }
  if (win > 0) {
    const int lo = qb * BM + diag - win + 1;
    kv_begin = lo > 0 ? (lo / BN) * BN : 0;
  }
  const int nt = kv_begin < kv_end ? (kv_end - kv_begin + BN - 1) / BN : 0;
  // this wave's visible tiles [tv0, tv1) and mask-free tiles [ti0, ti1) (tile t = keys
  // kv_begin + t BN ...)
  const int wave_last_q = q0 + 31;
  int tv0 = 0, tv1 = nt;
  if (CAUSAL) tv1 = imin(nt, imax(0, fdiv(wave_last_q + diag - kv_begin, BN) + 1));
  if (win > 0) tv0 = imax(0, -fdiv(kv_begin - (q0 + diag - win + 2 - BN), BN));
  tv0 = imin(tv0, tv1);
  int ti0 = tv0, ti1 = wave_last_q < sq ? fdiv(sk - BN - kv_begin, BN) + 1 : 0;
  if (CAUSAL) ti1 = imin(ti1, fdiv(q0 + diag - BN + 1 - kv_begin, BN) + 1);
  if (win > 0) ti0 = imax(ti0, -fdiv(kv_begin - (wave_last_q + diag - win + 1), BN));
  ti0 = imin(ti0, tv1);
  ti1 = imax(ti0, imin(ti1, tv1));

  Stage<D, BN> stK(p.k_ss), stV(p.v_ss);  // (unused by DMA)
  const RowOff<D> ro(r, hh);
  const TrOff<D> tro(lane);
  float bstage = 0.f;
  if constexpr (DMA) {
    // retire the Q loads with a wait hipcc tracks: otherwise it keeps them "pending" across
    // the loop and drains vmcnt(0) -- the in-flight K/V DMA included -- before the first MFMA
    __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
  }
  // Dropout keep bits: generated before the forward by the keep-bits kernel (attention_bits.hip,
  // the words the backward reads too) -- no hash in this kernel (it was ~110 VALU per tile per
  // lane).  DMA: a tile's 1 KB of the block's words arrives by LDS-DMA with the tile's K / V
  // (same vmcnt + barrier) and each lane reads its word from LDS; register staging: each lane
  // loads its word one tile ahead, before that tile's K / V loads (as the dQ kernel does).
  const bool bits_row_ok = DROP && qrow < sq;
  const int64_t sq2 = 2 * static_cast<int64_t>(sq);
  auto bits_ptr = [&](int t) {
    return p.drop_bits + bits_index(bh, ntiles64, (kv_begin + t * BN) >> 6, sq, qrow, hh);
  };
  // the block's tile-t slab (words [q][hh] are contiguous over the block's queries), gathered so
  // that LDS slot wave * 64 + lane holds the word of (query wave * 32 + r, half hh): each lane then
  // reads its own slot, conflict-free; rows past sq re-read the tile's last word (never stored)
  auto dma_bits = [&](int t, int b) {
    const int64_t w = static_cast<int64_t>(qb) * KBW + wave * 64 + 2 * r + hh;
    const int64_t base = (bh * ntiles64 + ((kv_begin + t * BN) >> 6)) * sq2;
    lds_dma4(p.drop_bits + base + (w < sq2 ? w : sq2 - 1), sKV + 4 * BN * DS + b * 2 * KBW + wave * 128);
  };
  const int kb_slot = wave * 64 + lane;  // this lane's word in a tile's slab
  uint32_t kb_cur = 0u, kb_nxt = 0u;
  if constexpr (BITS_LDS) {
    if (nt > 0) dma_bits(0, 0);
  } else {
    if (nt > 0 && bits_row_ok) kb_nxt = *bits_ptr(0);
  }
  if (nt > 0) {
    if constexpr (DMA) {
      dma_tile<D, BN>(sKV, K, p.k_ss, kv_begin, sk, wave, lane);
      dma_tile<D, BN>(sKV + BN * DS, V, p.v_ss, kv_begin, sk, wave, lane);
    } else {
      stK.load(K + static_cast<int64_t>(kv_begin) * p.k_ss, sk - kv_begin);
      stV.load(V + static_cast<int64_t>(kv_begin) * p.v_ss, sk - kv_begin);
      if (BIAS && threadIdx.x < BN) bstage = load_bias(p, b, kv_begin + threadIdx.x);
    }
  }
  int buf = 0;
  bool tile_bias = false;
  // tile t's barrier: its K/V landed in LDS for every wave; the next tile's copy is issued
  auto sync = [&](int t) {
    const int kv0 = kv_begin + t * BN;
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of the tile landed
      __syncthreads();  // ... everyone's; and every wave is done with the other buffer
      sK = sKV + buf * 2 * BN * DS;
      sV = sK + BN * DS;
      if constexpr (BITS_LDS) sBits = reinterpret_cast<const uint32_t*>(sKV + 4 * BN * DS + buf * 2 * KBW);
      if (t + 1 < nt) {
        if constexpr (BITS_LDS) dma_bits(t + 1, buf ^ 1);
        uint16_t* nb = sKV + (buf ^ 1) * 2 * BN * DS;
        dma_tile<D, BN>(nb, K, p.k_ss, kv0 + BN, sk, wave, lane);
        dma_tile<D, BN>(nb + BN * DS, V, p.v_ss, kv0 + BN, sk, wave, lane);
      }
      buf ^= 1;
    } else {
      kb_cur = kb_nxt;
      __syncthreads();
      stK.store(sK);
      stV.store(sV);
      if (BIAS) {
        if (threadIdx.x < BN) sB[threadIdx.x] = bstage * inv_scale;
        publish_bias_flag(bstage, &sFlag);
      }
      __syncthreads();
      tile_bias = BIAS && sFlag != 0;
      if (t + 1 < nt) {
        if (bits_row_ok) kb_nxt = *bits_ptr(t + 1);
        stK.load(K + static_cast<int64_t>(kv0 + BN) * p.k_ss, sk - kv0 - BN);
        stV.load(V + static_cast<int64_t>(kv0 + BN) * p.v_ss, sk - kv0 - BN);
        if (BIAS && threadIdx.x < BN) bstage = load_bias(p, b, kv0 + BN + threadIdx.x);
      }
    }
  };
  // one visible tile: S^T = K Q^T, (edge masks), online softmax, (dropout), O^T += V^T P^T
  auto body = [&](int t, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int kv0 = kv_begin + t * BN;
    f32x16 s0 = f32x16{0}, s1 = f32x16{0};
#pragma unroll
    for (int k = 0; k < D / 16; ++k) {
      const typename MF<T>::e8 qt = QLDS ? ld8<T>(sQ + ro.o[k] + wave * 32 * DS) : qf[k];
      s0 = MF<T>::mma(ld8<T>(sK + ro.o[k]), qt, s0);
      s1 = MF<T>::mma(ld8<T>(sK + ro.o[k] + 32 * DS), qt, s1);
    }
    if (BIAS && tile_bias) {
      add_from_keys(s0, sB, hh);
      add_from_keys(s1, sB + 32, hh);
    }
    if constexpr (MASK) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int k0 = kv0 + acc_row(reg, hh);
        const int k1 = k0 + 32;
        if (k0 >= sk || (CAUSAL && k0 > qrow + diag) || (win > 0 && k0 <= qrow + diag - win)) s0[reg] = -INFINITY;
        if (k1 >= sk || (CAUSAL && k1 > qrow + diag) || (win > 0 && k1 <= qrow + diag - win)) s1[reg] = -INFINITY;
      }
    }
    // raw-score row max (scale > 0 keeps the order), two independent v_max3 chains
    float mx0 = max3(s0[0], s1[0], s0[1]), mx1 = max3(s1[1], s0[2], s1[2]);
#pragma unroll
    for (int reg = 3; reg < 15; reg += 2) {
      mx0 = max3(mx0, s0[reg], s1[reg]);
      mx1 = max3(mx1, s0[reg + 1], s1[reg + 1]);
    }
    const float mx = pair_max32(max3(mx0, mx1, max3(s0[15], s1[15], s0[15])) * sl2);
    if (__any(mx > m_i + kTau)) {  // first visible tile, or a max jump: move the offset
      // (a side-effecting statement: keeps hipcc from if-converting the rescale into 16
      // packed multiplies on every tile)
      asm volatile("" ::: "memory");
      const float m_new = fmaxf(m_i, mx);
      const float mu = m_new == -INFINITY ? 0.f : m_new;  // fully masked so far: keep p = 0
      const float alpha = fast_exp2(m_i - mu);
#pragma unroll
      for (int i = 0; i < D / 32; ++i) o[i] *= alpha;
      l_i *= alpha;
      m_i = m_new;
      m_use = mu;
    }
    // p = exp2(S sl2 - m), scalar (the packed-pair form measured slower here: profiles/r4/attention_r4c.md)
    float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const float e0 = fast_exp2(fmaf(s0[reg], sl2, -m_use));
      const float e1 = fast_exp2(fmaf(s1[reg], sl2, -m_use));
      s0[reg] = e0;
      s1[reg] = e1;
      rs0 += e0;
      rs1 += e1;
    }
    l_i += rs0 + rs1;
    typename MF<T>::e8 pf[4] = {pack8<T>(s0, 0), pack8<T>(s0, 1), pack8<T>(s1, 0), pack8<T>(s1, 1)};
    if (DROP) {  // the normaliser above used every p; only kept entries reach P.V
      // the tile's keep word, read here so its flags are live only for these masks: register
      // group g of half s has its flags at bits 8 i + 7 of w << (g + 4 s) (unpack_keep)
      const uint32_t w = BITS_LDS ? sBits[kb_slot] : kb_cur;
      pf[0] = drop_packed(pf[0], w, w << 1);
      pf[1] = drop_packed(pf[1], w << 2, w << 3);
      pf[2] = drop_packed(pf[2], w << 4, w << 5);
      pf[3] = drop_packed(pf[3], w << 6, w << 7);
    }
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        o[i] = MF<T>::mma(ld_tr<T>(sV, tro.lo[i] + 16 * s * DS, tro.hi[i] + 16 * s * DS), pf[s], o[i]);
      }
    }
  };
  int t = 0;
  for (; t < tv0; ++t) sync(t);
  for (; t < ti0; ++t) {
    sync(t);
    body(t, std::true_type{});
  }
  for (; t < ti1; ++t) {
    sync(t);
    body(t, std::false_type{});
  }
  for (; t < tv1; ++t) {
    sync(t);
    body(t, std::true_type{});
  }
  for (; t < nt; ++t) sync(t);
  const float lt = pair_sum32(l_i);  // the two half-waves' partial row sums
  if (qrow >= sq) return;
  const float inv = lt > 0.f ? (DROP ? p.drop_rs : 1.f) / lt : 0.f;
  uint16_t* O = static_cast<uint16_t*>(p.o) + b * p.o_sb + h * p.o_sh + static_cast<int64_t>(qrow) * p.o_ss;
  store_rows<T, D>(O, o, inv, hh);
  if (hh == 0) p.lse[bh * p.sq + qrow] = (lt > 0.f) ? (m_i + log2f(lt)) / kLog2e : -INFINITY;
}

// ===================================================================== dK / dV
// Block = 4 waves x 32 keys (key on the MFMA lane); Q/dO tiles of 64 queries, two 32-query
// sub-steps.  S and dP accumulators start from the per-query row constants
// (-lse*log2e/(scale*log2e) [+ key bias / scale], -delta), so p = exp2(S' * scale*log2e)
// and dS = p * dP' (with dropout the delta is applied after the keep mask).
// D = 256: the dK/dV output columns are split over two blocks (NSPLIT), each recomputing S
// and dP in full -- 256 accumulator registers for a whole 32-key x 256 dK/dV pair do not fit
// beside the K/V fragments.
template <int D>
struct DkdvSplit {
  static constexpr int v = D >= 256 ? 2 : 1;
};

template <typename T, int D, bool CAUSAL, bool DROP, bool BIAS>
__global__ void __launch_bounds__(kThreads, D == 64 ? 2 : 1) attn_bwd_dkdv_kernel(AttnBwdParams P) {
  constexpr int BKEYS = 128, BQ = 64, DS = LdsStride<D>::v;
  constexpr int NSPLIT = DkdvSplit<D>::v, DO = D / NSPLIT;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[BQ * DS];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[BQ * DS];
  __shared__ __attribute__((aligned(16))) float sL[BQ], sDl[BQ];
  // keep bits of the Q tile x the block's 128 keys: [64-key half][word half-wave][query]
  // rows padded to 72 words: the 4 rows a wave reads start 8 banks apart (with the 4-word
  // half-wave offset: 8 distinct 4-bank groups), where a 64-word stride put all four on the
  // same banks (SQ_LDS_BANK_CONFLICT 7.1e6 per dispatch, profiles/pmc/r4_attention_counters.md)
  constexpr int BROW = BQ + 8;
  __shared__ __attribute__((aligned(16))) uint32_t sBits[DROP ? 4 * BROW : 4];
  const AttnParams& p = P.f;
  // wave index as a scalar: every wave-derived tile condition (causal / window / edge) then
  // branches on SGPRs instead of being if-converted into per-lane selects on every tile
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  int kb;
  int64_t bh;
  xcd_map(static_cast<int>((p.sk + BKEYS - 1) / BKEYS) * NSPLIT, p.b * p.h, kb, bh);
  const int col0 = (kb % NSPLIT) * DO;  // first dK/dV column of this block
  kb /= NSPLIT;
  const int64_t b = bh / p.h, h = bh % p.h;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk), diag = sk - sq;
  const int win = p.window;
  const int k0w = kb * BKEYS + wave * 32;  // wave's first key
  const int krow = k0w + r;                // this lane's key (as B-operand column)

  const uint16_t* Q = static_cast<const uint16_t*>(p.q) + b * p.q_sb + h * p.q_sh;
  const uint16_t* K = static_cast<const uint16_t*>(p.k) + b * p.k_sb + h * p.k_sh;
  const uint16_t* V = static_cast<const uint16_t*>(p.v) + b * p.v_sb + h * p.v_sh;
  const uint16_t* dO = static_cast<const uint16_t*>(P.dout) + b * P.do_sb + h * P.do_sh;
  const float* LSE = p.lse + bh * p.sq;
  const float* DL = P.delta + bh * p.sq;

  typename MF<T>::e8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int t = 0; t < D / 16; ++t) {
    if (krow < sk) {
      kf[t] = ld8<T>(K + static_cast<int64_t>(krow) * p.k_ss + 16 * t + 8 * hh);
      vf[t] = ld8<T>(V + static_cast<int64_t>(krow) * p.v_ss + 16 * t + 8 * hh);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        kf[t][j] = MF<T>::cvt(0.f);
        vf[t][j] = MF<T>::cvt(0.f);
      }
    }
  }
  f32x16 dv[DO / 32], dk[DO / 32];
#pragma unroll
  for (int i = 0; i < DO / 32; ++i) dv[i] = dk[i] = f32x16{0};
  const float sl2 = p.scale * kLog2e;
  const float inv_sl2 = 1.f / sl2;
  // the lane's key bias: loaded now, first consumed after the first tile's staging wait
  // (an immediate use would stall every block on the load latency)
  const float kbias_raw = BIAS ? load_bias(p, b, krow) : 0.f;
  float kbias = 0.f;
  bool blk_bias = false;  // this wave's 32 keys carry a bias
  // dropout: the forward's keep bits.  This lane's key kr = krow & 31 in 32-key half s =
  // wave & 1 of 64-key tile kb * 2 + wave / 2 is register 4 (kr >> 3) + (kr & 3) of the words
  // with half-wave index (kr >> 2) & 1: bit drop_bit(s, that register).  Thread t stages word
  // (tile half t >> 7, query (t >> 1) & 63, half-wave t & 1) of each Q tile (coalesced 512 B
  // runs) into sBits[(t >> 7) * 2 + (t & 1)][query].
  const int ntiles64 = (sk + 63) >> 6;
  const uint32_t kbit = drop_bit(wave & 1, 4 * (r >> 3) + (r & 3));
  const int bits_row = ((wave >> 1) * 2 + ((r >> 2) & 1)) * BROW;  // this lane's sBits row
  const int st_tile = kb * 2 + static_cast<int>(threadIdx.x >> 7), st_q = (threadIdx.x >> 1) & 63;
  const int st_hh = threadIdx.x & 1;
  uint32_t bits_stage = 0u;
  auto load_bits = [&](int qt) {
    const int qq = qt + st_q;
    bits_stage = qq < sq && st_tile < ntiles64 ? p.drop_bits[bits_index(bh, ntiles64, st_tile, sq, qq, st_hh)] : 0u;
  };
  const uint32_t rsd_bits = __builtin_bit_cast(uint32_t, p.drop_rs);
  int q_start = 0, q_end = sq;
  if (CAUSAL) {
    q_start = kb * BKEYS - diag;
    q_start = q_start < 0 ? 0 : (q_start / BQ) * BQ;
  }
  if (win > 0) {
    const int hi = (kb + 1) * BKEYS - 1 - diag + win;  // last query that sees the block's last key
    q_end = hi + 1 < sq ? hi + 1 : sq;
  }
  Stage<D, BQ> stQ(p.q_ss), stO(P.do_ss);
  const RowOff<D> ro(r, hh);
  const TrOff<D, DO / 32> tro(lane, col0);
  float l_stage = 0.f, d_stage = 0.f;
  if (q_start < q_end) {
    stQ.load(Q + static_cast<int64_t>(q_start) * p.q_ss, sq - q_start);
    stO.load(dO + static_cast<int64_t>(q_start) * P.do_ss, sq - q_start);
    if (threadIdx.x < BQ) {
      const int qq = q_start + threadIdx.x;
      l_stage = qq < sq ? LSE[qq] : 0.f;
      d_stage = qq < sq ? DL[qq] : 0.f;
    }
    if (DROP) load_bits(q_start);
  }
  const int klast = k0w + 31;
  // 64-query tiles: this wave's visible tiles [tv0, tv1) and mask-free tiles [ti0, ti1) (tile
  // t = queries q_start + 64 t ...; edge tiles run the masked sub-step body)
  const int nt = q_start < q_end ? (q_end - q_start + BQ - 1) / BQ : 0;
  int tv0 = 0, tv1 = nt;
  if (CAUSAL) tv0 = imax(0, -fdiv(q_start - (k0w - diag - (BQ - 1)), BQ));
  if (win > 0) tv1 = imin(nt, imax(0, fdiv(klast - diag + win - 1 - q_start, BQ) + 1));
  tv0 = imin(tv0, tv1);
  int ti0 = tv0, ti1 = klast < sk ? fdiv(sq - BQ - q_start, BQ) + 1 : 0;
  if (CAUSAL) ti0 = imax(ti0, -fdiv(q_start - (klast - diag), BQ));
  if (win > 0) ti1 = imin(ti1, fdiv(k0w - BQ - diag + win - q_start, BQ) + 1);
  ti0 = imin(ti0, tv1);
  ti1 = imax(ti0, imin(ti1, tv1));
  auto sync = [&](int t) {
    const int qt = q_start + t * BQ;
    __syncthreads();
    stQ.store(sQ);
    stO.store(sdO);
    if (threadIdx.x < BQ) {
      // lse == -inf (fully masked row) contributes nothing: any finite constant works
      sL[threadIdx.x] = l_stage == -INFINITY ? 0.f : -l_stage * kLog2e * inv_sl2;
      sDl[threadIdx.x] = -d_stage;
    }
    if (DROP) sBits[((threadIdx.x >> 7) * 2 + (threadIdx.x & 1)) * BROW + ((threadIdx.x >> 1) & 63)] = bits_stage;
    __syncthreads();
    if (BIAS) {
      kbias = kbias_raw * (1.f / p.scale);
      blk_bias = __any(kbias != 0.f);
    }
    if (t + 1 < nt) {
      stQ.load(Q + static_cast<int64_t>(qt + BQ) * p.q_ss, sq - qt - BQ);
      stO.load(dO + static_cast<int64_t>(qt + BQ) * P.do_ss, sq - qt - BQ);
      if (threadIdx.x < BQ) {
        const int qq = qt + BQ + threadIdx.x;
        l_stage = qq < sq ? LSE[qq] : 0.f;
        d_stage = qq < sq ? DL[qq] : 0.f;
      }
      if (DROP) load_bits(qt + BQ);
    }
  };
  // one 32-query sub-step (queries qs .. qs + 31 = LDS rows 32 sub ..)
  auto step = [&](int qs, int sub, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    // S' = Q K^T - lse/scale [+ bias/scale], dP' = dO V^T - delta (query rows in regs, key on lane)
    f32x16 s, dp, ndl;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 lv = *reinterpret_cast<const float4*>(&sL[32 * sub + 8 * g + 4 * hh]);
      const float4 dv4 = *reinterpret_cast<const float4*>(&sDl[32 * sub + 8 * g + 4 * hh]);
      s[4 * g + 0] = lv.x; s[4 * g + 1] = lv.y; s[4 * g + 2] = lv.z; s[4 * g + 3] = lv.w;
      if (DROP) {
        ndl[4 * g + 0] = dv4.x; ndl[4 * g + 1] = dv4.y; ndl[4 * g + 2] = dv4.z; ndl[4 * g + 3] = dv4.w;
        dp[4 * g + 0] = dp[4 * g + 1] = dp[4 * g + 2] = dp[4 * g + 3] = 0.f;
      } else {
        dp[4 * g + 0] = dv4.x; dp[4 * g + 1] = dv4.y; dp[4 * g + 2] = dv4.z; dp[4 * g + 3] = dv4.w;
      }
    }
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
      s = MF<T>::mma(ld8<T>(sQ + ro.o[t] + 32 * sub * DS), kf[t], s);
      dp = MF<T>::mma(ld8<T>(sdO + ro.o[t] + 32 * sub * DS), vf[t], dp);
    }
    // dO^T / Q^T fragments of the dV / dK MFMAs now (independent of the exp / dS work below),
    // so those MFMAs issue back to back instead of each waiting on its own LDS reads
    constexpr bool TPRE = D <= 128 && !BIAS && !DROP && CAUSAL;  // (others: spills)
    // with dropout (D = 64) the dO^T fragments only: dK/dV -4.5 %; both spill 60 B and lose
    // 10 % (profiles/r4/attention_r4c.md)
    constexpr bool TPRE_DO = TPRE || (D == 64 && !BIAS && DROP && CAUSAL);
    typename MF<T>::e8 tdo[TPRE_DO ? DO / 32 : 1][2], tq[TPRE ? DO / 32 : 1][2];
    if constexpr (TPRE_DO) {
      const int a0 = 32 * sub * DS, a1 = (32 * sub + 16) * DS;
#pragma unroll
      for (int i = 0; i < DO / 32; ++i) {
        tdo[i][0] = ld_tr<T>(sdO, tro.lo[i] + a0, tro.hi[i] + a0);
        tdo[i][1] = ld_tr<T>(sdO, tro.lo[i] + a1, tro.hi[i] + a1);
        if constexpr (TPRE) {
          tq[i][0] = ld_tr<T>(sQ, tro.lo[i] + a0, tro.hi[i] + a0);
          tq[i][1] = ld_tr<T>(sQ, tro.lo[i] + a1, tro.hi[i] + a1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (blk_bias) {
#pragma unroll
      for (int j = 0; j < 16; ++j) s[j] += kbias;
    }
    // the forward's keep words of the 16 query registers (query 32 sub + 8 g + 4 hh + i):
    // four 16-byte LDS reads (4 distinct addresses per wave: broadcasts)
    uint4 kw[4];
    if (DROP) {
#pragma unroll
      for (int g = 0; g < 4; ++g) kw[g] = *reinterpret_cast<const uint4*>(&sBits[bits_row + 32 * sub + 8 * g + 4 * hh]);
    }
    // element-wise on register pairs (2j, 2j + 1): packed fp32 multiplies / FMAs
    f32x2 po[8], dso[8];
    const f32x2 sl2v = {sl2, sl2};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int reg = 2 * j;
      const f32x2 sa = f32x2{s[reg], s[reg + 1]} * sl2v;
      f32x2 pv = {fast_exp2(sa.x), fast_exp2(sa.y)};
      if constexpr (MASK) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int qq = qs + acc_row(reg + e, hh);
          if (qq >= sq || krow >= sk || (CAUSAL && krow > qq + diag) || (win > 0 && krow <= qq + diag - win))
            pv[e] = 0.f;
        }
      }
      const f32x2 dpv = {dp[reg], dp[reg + 1]};
      if (DROP) {
        // keep / (1 - p) or 0 from the forward's bits (words reg, reg + 1 of group reg / 4)
        const uint4 w4 = kw[reg >> 2];
        const uint32_t wa = (reg & 2) ? w4.z : w4.x, wb = (reg & 2) ? w4.w : w4.y;
        const f32x2 z = {__builtin_bit_cast(float, bit_mask(wa, kbit) & rsd_bits),
                         __builtin_bit_cast(float, bit_mask(wb, kbit) & rsd_bits)};
        po[j] = pv * z;                                                              // (P o Z) for dV
        dso[j] = pv * __builtin_elementwise_fma(dpv, z, f32x2{ndl[reg], ndl[reg + 1]});  // P o (Z o dP - delta)
      } else {
        po[j] = pv;
        dso[j] = dpv * pv;
      }
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (B operands = accumulators, A via transposed reads)
    typename MF<T>::e8 pf0 = pack8p<T>(po, 0), pf1 = pack8p<T>(po, 1);
    typename MF<T>::e8 sf0 = pack8p<T>(dso, 0), sf1 = pack8p<T>(dso, 1);
#pragma unroll
    for (int i = 0; i < DO / 32; ++i) {
      const int a0 = 32 * sub * DS, a1 = (32 * sub + 16) * DS;
      if constexpr (TPRE) {
        dv[i] = MF<T>::mma(tdo[i][0], pf0, dv[i]);
        dv[i] = MF<T>::mma(tdo[i][1], pf1, dv[i]);
        dk[i] = MF<T>::mma(tq[i][0], sf0, dk[i]);
        dk[i] = MF<T>::mma(tq[i][1], sf1, dk[i]);
      } else if constexpr (TPRE_DO) {
        dv[i] = MF<T>::mma(tdo[i][0], pf0, dv[i]);
        dv[i] = MF<T>::mma(tdo[i][1], pf1, dv[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a0, tro.hi[i] + a0), sf0, dk[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a1, tro.hi[i] + a1), sf1, dk[i]);
      } else {
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, tro.lo[i] + a0, tro.hi[i] + a0), pf0, dv[i]);
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, tro.lo[i] + a1, tro.hi[i] + a1), pf1, dv[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a0, tro.hi[i] + a0), sf0, dk[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a1, tro.hi[i] + a1), sf1, dk[i]);
      }
    }
  };
  // edge tile: each visible sub-step with the per-element masks
  auto edge = [&](int t) {
    const int qt = q_start + t * BQ;
#pragma unroll 1
    for (int sub = 0; sub < 2; ++sub) {
      const int qs = qt + 32 * sub;
      if (CAUSAL && qs + 31 + diag < k0w) continue;          // no query sees these keys
      if (win > 0 && qs + diag - win + 1 > klast) continue;  // all keys left the window
      step(qs, sub, std::true_type{});
    }
  };
  int t = 0;
  for (; t < tv0; ++t) sync(t);
  for (; t < ti0; ++t) {
    sync(t);
    edge(t);
  }
  for (; t < ti1; ++t) {
    sync(t);
    // D = 64 (except dropout + key bias): both sub-steps in one unrolled body (the second one's
    // S / dP MFMAs overlap the first one's exp / dS / dropout work; with a key bias the
    // unrolled body spills)
#pragma unroll(D == 64 && (!DROP || !BIAS) ? 2 : 1)
    for (int sub = 0; sub < 2; ++sub) step(q_start + t * BQ + 32 * sub, sub, std::false_type{});
  }
  for (; t < tv1; ++t) {
    sync(t);
    edge(t);
  }
  for (; t < nt; ++t) sync(t);
  if (krow >= sk) return;
  uint16_t* dK = static_cast<uint16_t*>(P.dk) + b * P.dk_sb + h * P.dk_sh + static_cast<int64_t>(krow) * P.dk_ss;
  uint16_t* dV = static_cast<uint16_t*>(P.dv) + b * P.dv_sb + h * P.dv_sh + static_cast<int64_t>(krow) * P.dv_ss;
  store_rows<T, D, DO / 32>(dK + col0, dk, p.scale, hh);
  store_rows<T, D, DO / 32>(dV + col0, dv, 1.f, hh);
}

// ========================================================================= dQ
// Block = 4 waves x 32 queries (query on the lane: S^T = K Q^T, dP^T = V dO^T); K/V tiles
// of 64 keys; dQ^T += K^T dS^T with K^T from transposed LDS reads.  Tile phases as in the
// forward (edge masks only on edge tiles).  Accumulators start at zero (an inline-constant
// operand of the first MFMA) and the row constants enter the exponent's fma / the dS
// subtraction instead of 64 register moves per tile.
// Fused delta: the block computes delta = rowsum(dO o O) of its own query rows from the dO
// fragments it holds anyway plus one read of the O rows, and publishes it for the dK/dV kernel
// launched after it -- no separate delta pass over O and dO.
template <typename T, int D, bool CAUSAL, bool DROP, bool BIAS>
__global__ void __launch_bounds__(kThreads, D == 64 ? 2 : 1) attn_bwd_dq_kernel(AttnBwdParams P) {
  constexpr int BM = 128, BN = 64, DS = LdsStride<D>::v;
  constexpr int NSPLIT = DkdvSplit<D>::v, DO = D / NSPLIT;  // dQ columns per block
  __shared__ __attribute__((aligned(16))) uint16_t sK[BN * DS];
  __shared__ __attribute__((aligned(16))) uint16_t sV[BN * DS];
  __shared__ __attribute__((aligned(16))) float sB[BIAS ? BN : 4];
  __shared__ int sFlag;
  const AttnParams& p = P.f;
  // wave index as a scalar: every wave-derived tile condition (causal / window / edge) then
  // branches on SGPRs instead of being if-converted into per-lane selects on every tile
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = static_cast<int>((p.sq + BM - 1) / BM);
  int tile;
  int64_t bh;
  xcd_map(nqb * NSPLIT, p.b * p.h, tile, bh);
  const int col0 = (tile % NSPLIT) * DO;
  tile /= NSPLIT;
  const int64_t b = bh / p.h, h = bh % p.h;
  const int qb = CAUSAL ? (nqb - 1 - tile) : tile;
  const int q0 = qb * BM + wave * 32;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk), diag = sk - sq;
  const int win = p.window;
  const int qrow = q0 + r;
  const uint16_t* Q = static_cast<const uint16_t*>(p.q) + b * p.q_sb + h * p.q_sh;
  const uint16_t* K = static_cast<const uint16_t*>(p.k) + b * p.k_sb + h * p.k_sh;
  const uint16_t* V = static_cast<const uint16_t*>(p.v) + b * p.v_sb + h * p.v_sh;
  const uint16_t* dO = static_cast<const uint16_t*>(P.dout) + b * P.do_sb + h * P.do_sh;

  typename MF<T>::e8 qf[D / 16], df[D / 16];
#pragma unroll
  for (int t = 0; t < D / 16; ++t) {
    if (qrow < sq) {
      qf[t] = ld8<T>(Q + static_cast<int64_t>(qrow) * p.q_ss + 16 * t + 8 * hh);
      df[t] = ld8<T>(dO + static_cast<int64_t>(qrow) * P.do_ss + 16 * t + 8 * hh);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        qf[t][j] = MF<T>::cvt(0.f);
        df[t][j] = MF<T>::cvt(0.f);
      }
    }
  }
  float lse = qrow < sq ? p.lse[bh * p.sq + qrow] : 0.f;
  if (lse == -INFINITY) lse = 0.f;  // fully masked row: every p is masked to 0 below
  const float sl2 = p.scale * kLog2e;
  const float inv_scale = 1.f / p.scale;
  const float lse2 = lse * kLog2e;  // p = exp2(S sl2 - lse2)
  float dl;
  {
    // lane (r, hh) holds elements [16 t + 8 hh, +8) of dO row qrow: the matching O elements,
    // a lane-local partial dot product, and the other half-row from lane ^ 32
    const uint16_t* Orow = static_cast<const uint16_t*>(p.o) + b * p.o_sb + h * p.o_sh;
    float part = 0.f;
    if (qrow < sq) {
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        const typename MF<T>::e8 o8 = ld8<T>(Orow + static_cast<int64_t>(qrow) * p.o_ss + 16 * t + 8 * hh);
#pragma unroll
        for (int j = 0; j < 8; ++j) part = fmaf(static_cast<float>(df[t][j]), static_cast<float>(o8[j]), part);
      }
    }
    dl = pair_sum32(part);
    if (col0 == 0 && hh == 0 && qrow < sq) P.delta[bh * p.sq + qrow] = dl;
  }
  const int ntiles64 = (sk + 63) >> 6;
  const uint32_t rsd_bits = __builtin_bit_cast(uint32_t, p.drop_rs);
  const f32x2 sl2v = {sl2, sl2}, nlse2 = {-lse2, -lse2}, ndl2 = {-dl, -dl};
  f32x16 dq[DO / 32];
#pragma unroll
  for (int i = 0; i < DO / 32; ++i) dq[i] = f32x16{0};
  int kv_end = sk, kv_begin = 0;
  if (CAUSAL) {
    const int lim = (qb + 1) * BM + diag;
    kv_end = lim < sk ? lim : sk;
  }
  if (win > 0) {
    const int lo = qb * BM + diag - win + 1;
    kv_begin = lo > 0 ? (lo / BN) * BN : 0;
  }
  const int nt = kv_begin < kv_end ? (kv_end - kv_begin + BN - 1) / BN : 0;
  // visible tiles [tv0, tv1), mask-free tiles [ti0, ti1) of this wave (as in the forward)
  const int wave_last_q = q0 + 31;
  int tv0 = 0, tv1 = nt;
  if (CAUSAL) tv1 = imin(nt, imax(0, fdiv(wave_last_q + diag - kv_begin, BN) + 1));
  if (win > 0) tv0 = imax(0, -fdiv(kv_begin - (q0 + diag - win + 2 - BN), BN));
  tv0 = imin(tv0, tv1);
  int ti0 = tv0, ti1 = wave_last_q < sq ? fdiv(sk - BN - kv_begin, BN) + 1 : 0;
  if (CAUSAL) ti1 = imin(ti1, fdiv(q0 + diag - BN + 1 - kv_begin, BN) + 1);
  if (win > 0) ti0 = imax(ti0, -fdiv(kv_begin - (wave_last_q + diag - win + 1), BN));
  ti0 = imin(ti0, tv1);
  ti1 = imax(ti0, imin(ti1, tv1));

  Stage<D, BN> stK(p.k_ss), stV(p.v_ss);
  const RowOff<D> ro(r, hh);
  const TrOff<D, DO / 32> tro(lane, col0);
  float bstage = 0.f;
  if (nt > 0) {
    stK.load(K + static_cast<int64_t>(kv_begin) * p.k_ss, sk - kv_begin);
    stV.load(V + static_cast<int64_t>(kv_begin) * p.v_ss, sk - kv_begin);
    if (BIAS && threadIdx.x < BN) bstage = load_bias(p, b, kv_begin + threadIdx.x);
  }
  bool tile_bias = false;
  // keep bits of the next visible tile, loaded one tile ahead and BEFORE that tile's K / V
  // staging loads: the in-order vmcnt then retires them without draining the K / V prefetch
  // (read in the body they sat behind it: dQ with dropout waited on the next tile's K / V)
  const bool bits_row_ok = DROP && qrow < sq;
  auto bits_at = [&](int t) -> uint32_t {
    return P.f.drop_bits[bits_index(bh, ntiles64, (kv_begin + t * BN) >> 6, sq, qrow, hh)];
  };
  uint32_t kb_cur = 0u, kb_nxt = 0u;
  if (bits_row_ok && tv0 < tv1 && tv0 == 0) kb_nxt = bits_at(0);
  auto sync = [&](int t) {
    const int kv0 = kv_begin + t * BN;
    kb_cur = kb_nxt;
    __syncthreads();
    stK.store(sK);
    stV.store(sV);
    if (BIAS) {
      if (threadIdx.x < BN) sB[threadIdx.x] = bstage * inv_scale;
      publish_bias_flag(bstage, &sFlag);
    }
    __syncthreads();
    tile_bias = BIAS && sFlag != 0;
    if (t + 1 < nt) {
      if (bits_row_ok && t + 1 >= tv0 && t + 1 < tv1) kb_nxt = bits_at(t + 1);
      stK.load(K + static_cast<int64_t>(kv0 + BN) * p.k_ss, sk - kv0 - BN);
      stV.load(V + static_cast<int64_t>(kv0 + BN) * p.v_ss, sk - kv0 - BN);
      if (BIAS && threadIdx.x < BN) bstage = load_bias(p, b, kv0 + BN + threadIdx.x);
    }
  };
  auto body = [&](int t, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int kv0 = kv_begin + t * BN;
    const uint32_t kbits = kb_cur;
    // D <= 128: both 32-key halves' dS^T, then the dQ MFMAs (the two halves' MFMA chains
    // overlap each other's softmax VALU work).  D = 256: half by half, so only one half's
    // S / dP accumulators are live next to the 16 Q / dO fragments.
    constexpr bool SEQ = D >= 256;
    // K^T fragments of the dQ MFMAs (independent of the softmax work): read up front
    constexpr bool KPRE = !SEQ && !BIAS && !DROP;  // (with dropout: no gain, r4 notes)
    typename MF<T>::e8 ktf[KPRE ? DO / 32 : 1][4];
    if constexpr (KPRE) {
#pragma unroll
      for (int i = 0; i < DO / 32; ++i)
#pragma unroll
        for (int st = 0; st < 4; ++st) ktf[i][st] = ld_tr<T>(sK, tro.lo[i] + 16 * st * DS, tro.hi[i] + 16 * st * DS);
    }
    f32x16 s[2], dp[2];
    f32x2 dsp[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      s[u] = f32x16{0};
      dp[u] = f32x16{0};
#pragma unroll
      for (int k = 0; k < D / 16; ++k) {
        s[u] = MF<T>::mma(ld8<T>(sK + ro.o[k] + 32 * u * DS), qf[k], s[u]);
        dp[u] = MF<T>::mma(ld8<T>(sV + ro.o[k] + 32 * u * DS), df[k], dp[u]);
      }
      if (BIAS && tile_bias) add_from_keys(s[u], sB + 32 * u, hh);
      // dS^T = P o (Z o dP - delta), Z = keep / (1 - p) from the forward's bits (one dword per
      // lane per tile) -- with dropout element-wise on register pairs (packed fp32 FMAs /
      // multiplies: dQ -7 %); without it the scalar form measured 2 % faster
      // (profiles/r4/attention_r4c.md)
      if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int reg = 2 * j;
        const f32x2 a = __builtin_elementwise_fma(f32x2{s[u][reg], s[u][reg + 1]}, sl2v, nlse2);
        f32x2 pv = {fast_exp2(a.x), fast_exp2(a.y)};
        if constexpr (MASK) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int kk = kv0 + 32 * u + acc_row(reg + e, hh);
            if (qrow >= sq || kk >= sk || (CAUSAL && kk > qrow + diag) || (win > 0 && kk <= qrow + diag - win))
              pv[e] = 0.f;
          }
        }
        const f32x2 d = {dp[u][reg], dp[u][reg + 1]};
        if (DROP) {
          const f32x2 z = {__builtin_bit_cast(float, bit_mask(kbits, drop_bit(u, reg)) & rsd_bits),
                           __builtin_bit_cast(float, bit_mask(kbits, drop_bit(u, reg + 1)) & rsd_bits)};
          dsp[u][j] = pv * __builtin_elementwise_fma(d, z, ndl2);
        } else {
          dsp[u][j] = pv * (d + ndl2);
        }
      }
      } else {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        float pv = fast_exp2(fmaf(s[u][reg], sl2, -lse2));
        if constexpr (MASK) {
          const int kk = kv0 + 32 * u + acc_row(reg, hh);
          if (qrow >= sq || kk >= sk || (CAUSAL && kk > qrow + diag) || (win > 0 && kk <= qrow + diag - win)) pv = 0.f;
        }
        float d = dp[u][reg];
        if (DROP) d = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, d) & bit_mask(kbits, drop_bit(u, reg)));
        const float ds = DROP ? pv * fmaf(d, p.drop_rs, -dl) : pv * (d - dl);
        dsp[u][reg >> 1][reg & 1] = ds;
      }
}
      if (SEQ) {
        const typename MF<T>::e8 sf0 = pack8p<T>(dsp[u], 0), sf1 = pack8p<T>(dsp[u], 1);
#pragma unroll
        for (int i = 0; i < DO / 32; ++i) {
          const int a0 = 32 * u * DS, a1 = (32 * u + 16) * DS;
          dq[i] = MF<T>::mma(ld_tr<T>(sK, tro.lo[i] + a0, tro.hi[i] + a0), sf0, dq[i]);
          dq[i] = MF<T>::mma(ld_tr<T>(sK, tro.lo[i] + a1, tro.hi[i] + a1), sf1, dq[i]);
        }
      }
    }
    if (!SEQ) {
      typename MF<T>::e8 sf[4] = {pack8p<T>(dsp[0], 0), pack8p<T>(dsp[0], 1), pack8p<T>(dsp[1], 0),
                                  pack8p<T>(dsp[1], 1)};
#pragma unroll
      for (int i = 0; i < DO / 32; ++i) {
#pragma unroll
        for (int st = 0; st < 4; ++st)
          dq[i] = MF<T>::mma(KPRE ? ktf[i][st] : ld_tr<T>(sK, tro.lo[i] + 16 * st * DS, tro.hi[i] + 16 * st * DS),
                             sf[st], dq[i]);
      }
    }
  };
  int t = 0;
  for (; t < tv0; ++t) sync(t);
  for (; t < ti0; ++t) {
    sync(t);
    body(t, std::true_type{});
  }
  for (; t < ti1; ++t) {
    sync(t);
    body(t, std::false_type{});
  }
  for (; t < tv1; ++t) {
    sync(t);
    body(t, std::true_type{});
  }
  for (; t < nt; ++t) sync(t);
  if (qrow >= sq) return;
  uint16_t* dQ = static_cast<uint16_t*>(P.dq) + b * P.dq_sb + h * P.dq_sh + static_cast<int64_t>(qrow) * P.dq_ss;
  store_rows<T, D, DO / 32>(dQ + col0, dq, p.scale, hh);
}

// ------------------------------------------------------------------ launchers

template <typename T, int D, bool C, bool DR, bool BI>
int launch_fwd_v(const AttnParams& p, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(((p.sq + 127) / 128) * p.b * p.h);
  if constexpr ((D == 64 || D == 128) && !BI) {  // K/V tiles by LDS-DMA
    attn_fwd_kernel<T, D, C, DR, BI, true><<<grid, kThreads, 0, s>>>(p);
    return static_cast<int>(hipGetLastError());
  }
  attn_fwd_kernel<T, D, C, DR, BI><<<grid, kThreads, 0, s>>>(p);
  return static_cast<int>(hipGetLastError());
}

// dQ launch as its own function template: a head dim can instantiate it in a separate
// translation unit built with other flags (D = 64: attention_d64_dq.hip, no SLP vectorisation
// -- packed fp32 VALU beside the MFMAs costs the dQ kernel 4.5 %, profiles/r3/s3_rehearsal.md)
template <typename T, int D, bool C, bool DR, bool BI>
void launch_dq(const AttnBwdParams& p, unsigned g, hipStream_t s) {
  attn_bwd_dq_kernel<T, D, C, DR, BI><<<g, kThreads, 0, s>>>(p);
}

// X(T, C, DR, BI) for every dtype x variant of one head dim
#define SMPK_ATTN_VARIANTS(X)                                                                 \
  X(bf16, false, false, false) X(bf16, false, false, true) X(bf16, false, true, false)         \
  X(bf16, false, true, true) X(bf16, true, false, false) X(bf16, true, false, true)            \
  X(bf16, true, true, false) X(bf16, true, true, true) X(f16, false, false, false)             \
  X(f16, false, false, true) X(f16, false, true, false) X(f16, false, true, true)              \
  X(f16, true, false, false) X(f16, true, false, true) X(f16, true, true, false)               \
  X(f16, true, true, true)

template <typename T, int D, bool C, bool DR, bool BI>
int launch_bwd_v(const AttnBwdParams& p, hipStream_t s) {
  const unsigned gk = static_cast<unsigned>(((p.f.sk + 127) / 128) * p.f.b * p.f.h * DkdvSplit<D>::v);
  const unsigned gq = static_cast<unsigned>(((p.f.sq + 127) / 128) * p.f.b * p.f.h * DkdvSplit<D>::v);
  // dQ first: it computes delta = rowsum(dO o O) for its rows and writes it for the dK/dV
  // kernel (same stream)
  launch_dq<T, D, C, DR, BI>(p, gq, s);
  attn_bwd_dkdv_kernel<T, D, C, DR, BI><<<gk, kThreads, 0, s>>>(p);
  return static_cast<int>(hipGetLastError());
}

// runtime flags -> template variant
template <typename T, int D>
int launch_fwd(const AttnParams& p, hipStream_t s) {
  const bool dr = p.drop_on != 0, bi = p.kbias != nullptr;
  const int v = (p.causal ? 4 : 0) | (dr ? 2 : 0) | (bi ? 1 : 0);
  switch (v) {
    case 0: return launch_fwd_v<T, D, false, false, false>(p, s);
    case 1: return launch_fwd_v<T, D, false, false, true>(p, s);
    case 2: return launch_fwd_v<T, D, false, true, false>(p, s);
    case 3: return launch_fwd_v<T, D, false, true, true>(p, s);
    case 4: return launch_fwd_v<T, D, true, false, false>(p, s);
    case 5: return launch_fwd_v<T, D, true, false, true>(p, s);
    case 6: return launch_fwd_v<T, D, true, true, false>(p, s);
    default: return launch_fwd_v<T, D, true, true, true>(p, s);
  }
}

template <typename T, int D>
int launch_bwd(const AttnBwdParams& p, hipStream_t s) {
  const bool dr = p.f.drop_on != 0, bi = p.f.kbias != nullptr;
  const int v = (p.f.causal ? 4 : 0) | (dr ? 2 : 0) | (bi ? 1 : 0);
  switch (v) {
    case 0: return launch_bwd_v<T, D, false, false, false>(p, s);
    case 1: return launch_bwd_v<T, D, false, false, true>(p, s);
    case 2: return launch_bwd_v<T, D, false, true, false>(p, s);
    case 3: return launch_bwd_v<T, D, false, true, true>(p, s);
    case 4: return launch_bwd_v<T, D, true, false, false>(p, s);
    case 5: return launch_bwd_v<T, D, true, false, true>(p, s);
    case 6: return launch_bwd_v<T, D, true, true, false>(p, s);
    default: return launch_bwd_v<T, D, true, true, true>(p, s);
  }
}

}  // namespace attn

// Instantiates the per-head-dim entry points (one translation unit per head dim, so the
// 2 dtypes x 8 variants x 3 kernels build in parallel).
#define SMPK_ATTN_HEAD_DIM(D)                                                   \
  int attention_fwd_d##D(int dt, const AttnParams& p, hipStream_t s) {          \
    if (dt == BF16) return attn::launch_fwd<bf16, D>(p, s);                     \
    if (dt == F16) return attn::launch_fwd<f16, D>(p, s);                       \
    return -3;                                                                  \
  }                                                                             \
  int attention_bwd_d##D(int dt, const AttnBwdParams& p, hipStream_t s) {       \
    if (dt == BF16) return attn::launch_bwd<bf16, D>(p, s);                     \
    if (dt == F16) return attn::launch_bwd<f16, D>(p, s);                       \
    return -3;                                                                  \
  }

}  // namespace smpk
