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
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

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
template <int D>
__device__ __forceinline__ int swz(int row, int chunk) {
  const int g = D == 64 ? ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)) : (((row & 3) << 2) | ((row >> 2) & 3));
  return row * D + ((chunk ^ g) << 3);
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

template <int D>
struct TrOff {
  int lo[D / 32], hi[D / 32];
  __device__ __forceinline__ explicit TrOff(int lane) {
    const int q = (lane & 15) >> 2, pp = lane & 3, hh = lane >> 5;
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
      const int col = 32 * i + 16 * ((lane >> 4) & 1) + 4 * pp;
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

__device__ __forceinline__ int acc_row(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// fmaxf on MFMA results makes clang insert a canonicalising v_max per operand; scores are
// never signalling NaNs, so issue v_max3 directly (2 elements per instruction).
__device__ __forceinline__ float max3(float a, float b, float c) {
  float d;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// value of lane ^ 32 (the other half-wave) without an LDS round trip
__device__ __forceinline__ float xor32(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  const int lane = threadIdx.x & 63;
  return __builtin_bit_cast(float, lane < 32 ? r[1] : r[0]);
}

// Register-staged tile copy (issue global loads early, write LDS late: the HBM/L2 latency
// hides under the MFMA work of the current tile).
template <int D, int ROWS>
struct Stage {
  static constexpr int CH = D / 8;
  static constexpr int N = ROWS * CH / kThreads;
  static_assert(N * kThreads == ROWS * CH, "tile must split evenly over the block");
  uint4 v[N];
  int goff[N], loff[N], row[N];
  __device__ __forceinline__ explicit Stage(int64_t gs) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * kThreads, r = c / CH, k = c % CH;
      row[i] = r;
      goff[i] = static_cast<int>(r * gs) + k * 8;
      loff[i] = swz<D>(r, k);
    }
  }
  // tile: pointer to the tile's first row; rows >= valid read as zeros
  __device__ __forceinline__ void load(const uint16_t* tile, int valid) {
    if (valid >= ROWS) {  // wave-uniform: interior tiles load without per-lane predication
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = *reinterpret_cast<const uint4*>(tile + goff[i]);
      return;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      v[i] = row[i] < valid ? *reinterpret_cast<const uint4*>(tile + goff[i]) : make_uint4(0, 0, 0, 0);
  }
  __device__ __forceinline__ void store(uint16_t* lds) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<uint4*>(lds + loff[i]) = v[i];
  }
};

template <typename T, int D>
__device__ __forceinline__ void store_rows(uint16_t* dst, const f32x16* acc, float mul, int hh) {
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
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

// ================================================================== forward
// Block = 4 waves x 32 queries; K/V tiles of 64 keys.  Interior tiles (every key visible
// to every query of the wave) take a mask-free path.
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_kernel(AttnParams p) {
  constexpr int BM = 128, BN = 64;
  __shared__ __attribute__((aligned(16))) uint16_t sK[BN * D];
  __shared__ __attribute__((aligned(16))) uint16_t sV[BN * D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

  const uint16_t* Q = static_cast<const uint16_t*>(p.q) + b * p.q_sb + h * p.q_sh;
  const uint16_t* K = static_cast<const uint16_t*>(p.k) + b * p.k_sb + h * p.k_sh;
  const uint16_t* V = static_cast<const uint16_t*>(p.v) + b * p.v_sb + h * p.v_sh;

  typename MF<T>::e8 qf[D / 16];
  const int qrow = q0 + r;
#pragma unroll
  for (int t = 0; t < D / 16; ++t) {
    if (qrow < sq) {
      qf[t] = ld8<T>(Q + static_cast<int64_t>(qrow) * p.q_ss + 16 * t + 8 * hh);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[t][j] = MF<T>::cvt(0.f);
    }
  }
  const float sl2 = p.scale * kLog2e;
  float m_i = -INFINITY, l_i = 0.f;
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
  Stage<D, BN> stK(p.k_ss), stV(p.v_ss);
  const RowOff<D> ro(r, hh);
  const TrOff<D> tro(lane);
  if (kv_begin < kv_end) {
    stK.load(K + static_cast<int64_t>(kv_begin) * p.k_ss, sk - kv_begin);
    stV.load(V + static_cast<int64_t>(kv_begin) * p.v_ss, sk - kv_begin);
  }
  const int wave_last_q = q0 + 31;
  for (int kv0 = kv_begin; kv0 < kv_end; kv0 += BN) {
    __syncthreads();
    stK.store(sK);
    stV.store(sV);
    __syncthreads();
    if (kv0 + BN < kv_end) {
      stK.load(K + static_cast<int64_t>(kv0 + BN) * p.k_ss, sk - kv0 - BN);
      stV.load(V + static_cast<int64_t>(kv0 + BN) * p.v_ss, sk - kv0 - BN);
    }
    if (CAUSAL && kv0 > wave_last_q + diag) continue;
    if (win > 0 && kv0 + BN - 1 < q0 + diag - win + 1) continue;
    const bool interior = kv0 + BN <= sk && wave_last_q < sq && (!CAUSAL || kv0 + BN - 1 <= q0 + diag) &&
                          (win <= 0 || kv0 > wave_last_q + diag - win);
    f32x16 s0 = f32x16{0}, s1 = f32x16{0};
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
      s0 = MF<T>::mma(ld8<T>(sK + ro.o[t]), qf[t], s0);
      s1 = MF<T>::mma(ld8<T>(sK + ro.o[t] + 32 * D), qf[t], s1);
    }
    if (!interior) {
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
    float mx = max3(mx0, mx1, max3(s0[15], s1[15], s0[15])) * sl2;
    mx = fmaxf(mx, xor32(mx));
    const float m_new = fmaxf(m_i, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;  // fully masked so far: keep p = 0
    const float alpha = fast_exp2(m_i - m_use);
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
    float rs = rs0 + rs1;
    rs += xor32(rs);
    l_i = l_i * alpha + rs;
    if (__any(m_new != m_i)) {  // rescale only when a row max moved
#pragma unroll
      for (int i = 0; i < D / 32; ++i) o[i] *= alpha;
    }
    m_i = m_new;
    typename MF<T>::e8 pf[4] = {pack8<T>(s0, 0), pack8<T>(s0, 1), pack8<T>(s1, 0), pack8<T>(s1, 1)};
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
#pragma unroll
      for (int s = 0; s < 4; ++s) o[i] = MF<T>::mma(ld_tr<T>(sV, tro.lo[i] + 16 * s * D, tro.hi[i] + 16 * s * D), pf[s], o[i]);
    }
  }
  if (qrow >= sq) return;
  const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
  uint16_t* O = static_cast<uint16_t*>(p.o) + b * p.o_sb + h * p.o_sh + static_cast<int64_t>(qrow) * p.o_ss;
  store_rows<T, D>(O, o, inv, hh);
  if (hh == 0) p.lse[bh * p.sq + qrow] = (l_i > 0.f) ? (m_i + log2f(l_i)) / kLog2e : -INFINITY;
}

// ============================================================= delta = rowsum(dO * O)
template <typename T>
__global__ void __launch_bounds__(kThreads) attn_delta_kernel(AttnBwdParams p) {
  // 16 lanes per (b, h, query) row, 8 elements per lane per step (16-byte loads)
  const int sub = threadIdx.x & 15;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 16 + (threadIdx.x >> 4);
  const int64_t total = p.f.b * p.f.h * p.f.sq;
  const bool valid = row < total;
  float acc = 0.f;
  if (valid) {
    const int64_t q = row % p.f.sq, bh = row / p.f.sq, b = bh / p.f.h, h = bh % p.f.h;
    const T* O = static_cast<const T*>(p.f.o) + b * p.f.o_sb + h * p.f.o_sh + q * p.f.o_ss;
    const T* dO = static_cast<const T*>(p.dout) + b * p.do_sb + h * p.do_sh + q * p.do_ss;
    for (int d = sub * 8; d < p.f.d; d += 128) {
      Vec16<T> a = load16<T>(O + d), g = load16<T>(dO + d);
#pragma unroll
      for (int j = 0; j < Vec16<T>::N; ++j) acc += to_f32(a.v[j]) * to_f32(g.v[j]);
    }
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (valid && sub == 0) p.delta[row] = acc;
}

// ===================================================================== dK / dV
// Block = 4 waves x 32 keys (key on the MFMA lane); Q/dO tiles of 64 queries, two 32-query
// sub-steps.  S and dP accumulators start from the per-query row constants
// (-lse*log2e/(scale*log2e), -delta), so p = exp2(S' * scale*log2e) and dS = p * dP'.
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, D == 64 ? 2 : 1) attn_bwd_dkdv_kernel(AttnBwdParams P) {
  constexpr int BKEYS = 128, BQ = 64;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[BQ * D];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[BQ * D];
  __shared__ __attribute__((aligned(16))) float sL[BQ], sDl[BQ];
  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int kb;
  int64_t bh;
  xcd_map(static_cast<int>((p.sk + BKEYS - 1) / BKEYS), p.b * p.h, kb, bh);
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
  f32x16 dv[D / 32], dk[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dv[i] = dk[i] = f32x16{0};
  const float sl2 = p.scale * kLog2e;
  const float inv_sl2 = 1.f / sl2;
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
  const TrOff<D> tro(lane);
  float l_stage = 0.f, d_stage = 0.f;
  if (q_start < q_end) {
    stQ.load(Q + static_cast<int64_t>(q_start) * p.q_ss, sq - q_start);
    stO.load(dO + static_cast<int64_t>(q_start) * P.do_ss, sq - q_start);
    if (threadIdx.x < BQ) {
      const int qq = q_start + threadIdx.x;
      l_stage = qq < sq ? LSE[qq] : 0.f;
      d_stage = qq < sq ? DL[qq] : 0.f;
    }
  }
  const int klast = k0w + 31;
  for (int qt = q_start; qt < q_end; qt += BQ) {
    __syncthreads();
    stQ.store(sQ);
    stO.store(sdO);
    if (threadIdx.x < BQ) {
      // lse == -inf (fully masked row) contributes nothing: any finite constant works
      sL[threadIdx.x] = l_stage == -INFINITY ? 0.f : -l_stage * kLog2e * inv_sl2;
      sDl[threadIdx.x] = -d_stage;
    }
    __syncthreads();
    if (qt + BQ < q_end) {
      stQ.load(Q + static_cast<int64_t>(qt + BQ) * p.q_ss, sq - qt - BQ);
      stO.load(dO + static_cast<int64_t>(qt + BQ) * P.do_ss, sq - qt - BQ);
      if (threadIdx.x < BQ) {
        const int qq = qt + BQ + threadIdx.x;
        l_stage = qq < sq ? LSE[qq] : 0.f;
        d_stage = qq < sq ? DL[qq] : 0.f;
      }
    }
#pragma unroll 1
    for (int sub = 0; sub < 2; ++sub) {
      const int qs = qt + 32 * sub;  // first query of this sub-step
      if (CAUSAL && qs + 31 + diag < k0w) continue;          // no query sees these keys
      if (win > 0 && qs + diag - win + 1 > klast) continue;  // all keys left the window
      const bool interior = qs + 31 < sq && klast < sk && (!CAUSAL || klast <= qs + diag) &&
                            (win <= 0 || k0w > qs + 31 + diag - win);
      // S' = Q K^T - lse/scale, dP' = dO V^T - delta (query rows in regs, key on lane)
      f32x16 s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 lv = *reinterpret_cast<const float4*>(&sL[32 * sub + 8 * g + 4 * hh]);
        const float4 dv4 = *reinterpret_cast<const float4*>(&sDl[32 * sub + 8 * g + 4 * hh]);
        s[4 * g + 0] = lv.x; s[4 * g + 1] = lv.y; s[4 * g + 2] = lv.z; s[4 * g + 3] = lv.w;
        dp[4 * g + 0] = dv4.x; dp[4 * g + 1] = dv4.y; dp[4 * g + 2] = dv4.z; dp[4 * g + 3] = dv4.w;
      }
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        s = MF<T>::mma(ld8<T>(sQ + ro.o[t] + 32 * sub * D), kf[t], s);
        dp = MF<T>::mma(ld8<T>(sdO + ro.o[t] + 32 * sub * D), vf[t], dp);
      }
      if (interior) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const float pv = fast_exp2(s[reg] * sl2);
          s[reg] = pv;
          dp[reg] *= pv;
        }
      } else {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int qq = qs + acc_row(reg, hh);
          float pv = fast_exp2(s[reg] * sl2);
          if (qq >= sq || krow >= sk || (CAUSAL && krow > qq + diag) || (win > 0 && krow <= qq + diag - win))
            pv = 0.f;
          s[reg] = pv;
          dp[reg] *= pv;
        }
      }
      // dV^T += dO^T P ; dK^T += Q^T dS   (B operands = accumulators, A via transposed reads)
      typename MF<T>::e8 pf0 = pack8<T>(s, 0), pf1 = pack8<T>(s, 1);
      typename MF<T>::e8 sf0 = pack8<T>(dp, 0), sf1 = pack8<T>(dp, 1);
#pragma unroll
      for (int i = 0; i < D / 32; ++i) {
        const int a0 = 32 * sub * D, a1 = (32 * sub + 16) * D;
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, tro.lo[i] + a0, tro.hi[i] + a0), pf0, dv[i]);
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, tro.lo[i] + a1, tro.hi[i] + a1), pf1, dv[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a0, tro.hi[i] + a0), sf0, dk[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a1, tro.hi[i] + a1), sf1, dk[i]);
      }
    }
  }
  if (krow >= sk) return;
  uint16_t* dK = static_cast<uint16_t*>(P.dk) + b * P.dk_sb + h * P.dk_sh + static_cast<int64_t>(krow) * P.dk_ss;
  uint16_t* dV = static_cast<uint16_t*>(P.dv) + b * P.dv_sb + h * P.dv_sh + static_cast<int64_t>(krow) * P.dv_ss;
  store_rows<T, D>(dK, dk, p.scale, hh);
  store_rows<T, D>(dV, dv, 1.f, hh);
}

// ========================================================================= dQ
// Block = 4 waves x 32 queries (query on the lane: S^T = K Q^T, dP^T = V dO^T); K/V tiles
// of 64 keys; dQ^T += K^T dS^T with K^T from transposed LDS reads.
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, D == 64 ? 2 : 1) attn_bwd_dq_kernel(AttnBwdParams P) {
  constexpr int BM = 128, BN = 64;
  __shared__ __attribute__((aligned(16))) uint16_t sK[BN * D];
  __shared__ __attribute__((aligned(16))) uint16_t sV[BN * D];
  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = static_cast<int>((p.sq + BM - 1) / BM);
  int tile;
  int64_t bh;
  xcd_map(nqb, p.b * p.h, tile, bh);
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
  const float s_init = -lse * kLog2e / sl2;
  const float dl = qrow < sq ? P.delta[bh * p.sq + qrow] : 0.f;
  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dq[i] = f32x16{0};
  int kv_end = sk, kv_begin = 0;
  if (CAUSAL) {
    const int lim = (qb + 1) * BM + diag;
    kv_end = lim < sk ? lim : sk;
  }
  if (win > 0) {
    const int lo = qb * BM + diag - win + 1;
    kv_begin = lo > 0 ? (lo / BN) * BN : 0;
  }
  Stage<D, BN> stK(p.k_ss), stV(p.v_ss);
  const RowOff<D> ro(r, hh);
  const TrOff<D> tro(lane);
  if (kv_begin < kv_end) {
    stK.load(K + static_cast<int64_t>(kv_begin) * p.k_ss, sk - kv_begin);
    stV.load(V + static_cast<int64_t>(kv_begin) * p.v_ss, sk - kv_begin);
  }
  const int wave_last_q = q0 + 31;
  for (int kv0 = kv_begin; kv0 < kv_end; kv0 += BN) {
    __syncthreads();
    stK.store(sK);
    stV.store(sV);
    __syncthreads();
    if (kv0 + BN < kv_end) {
      stK.load(K + static_cast<int64_t>(kv0 + BN) * p.k_ss, sk - kv0 - BN);
      stV.load(V + static_cast<int64_t>(kv0 + BN) * p.v_ss, sk - kv0 - BN);
    }
    if (CAUSAL && kv0 > wave_last_q + diag) continue;
    if (win > 0 && kv0 + BN - 1 < q0 + diag - win + 1) continue;
    const bool interior = kv0 + BN <= sk && wave_last_q < sq && (!CAUSAL || kv0 + BN - 1 <= q0 + diag) &&
                          (win <= 0 || kv0 > wave_last_q + diag - win);
    f32x16 s[2], dp[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s[u][j] = s_init;
        dp[u][j] = -dl;
      }
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        s[u] = MF<T>::mma(ld8<T>(sK + ro.o[t] + 32 * u * D), qf[t], s[u]);
        dp[u] = MF<T>::mma(ld8<T>(sV + ro.o[t] + 32 * u * D), df[t], dp[u]);
      }
      if (interior) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) dp[u][reg] *= fast_exp2(s[u][reg] * sl2);
      } else {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int kk = kv0 + 32 * u + acc_row(reg, hh);
          float pv = fast_exp2(s[u][reg] * sl2);
          if (qrow >= sq || kk >= sk || (CAUSAL && kk > qrow + diag) || (win > 0 && kk <= qrow + diag - win))
            pv = 0.f;
          dp[u][reg] *= pv;  // dS^T
        }
      }
    }
    typename MF<T>::e8 sf[4] = {pack8<T>(dp[0], 0), pack8<T>(dp[0], 1), pack8<T>(dp[1], 0), pack8<T>(dp[1], 1)};
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
#pragma unroll
      for (int st = 0; st < 4; ++st)
        dq[i] = MF<T>::mma(ld_tr<T>(sK, tro.lo[i] + 16 * st * D, tro.hi[i] + 16 * st * D), sf[st], dq[i]);
    }
  }
  if (qrow >= sq) return;
  uint16_t* dQ = static_cast<uint16_t*>(P.dq) + b * P.dq_sb + h * P.dq_sh + static_cast<int64_t>(qrow) * P.dq_ss;
  store_rows<T, D>(dQ, dq, p.scale, hh);
}

template <typename T, int D>
int launch_fwd(const AttnParams& p, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(((p.sq + 127) / 128) * p.b * p.h);
  if (p.causal)
    attn_fwd_kernel<T, D, true><<<grid, kThreads, 0, s>>>(p);
  else
    attn_fwd_kernel<T, D, false><<<grid, kThreads, 0, s>>>(p);
  return static_cast<int>(hipGetLastError());
}

template <typename T, int D>
int launch_bwd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = p.f.b * p.f.h * p.f.sq;
  attn_delta_kernel<T><<<static_cast<unsigned>((rows + 15) / 16), kThreads, 0, s>>>(p);
  const unsigned gk = static_cast<unsigned>(((p.f.sk + 127) / 128) * p.f.b * p.f.h);
  const unsigned gq = static_cast<unsigned>(((p.f.sq + 127) / 128) * p.f.b * p.f.h);
  if (p.f.causal) {
    attn_bwd_dkdv_kernel<T, D, true><<<gk, kThreads, 0, s>>>(p);
    attn_bwd_dq_kernel<T, D, true><<<gq, kThreads, 0, s>>>(p);
  } else {
    attn_bwd_dkdv_kernel<T, D, false><<<gk, kThreads, 0, s>>>(p);
    attn_bwd_dq_kernel<T, D, false><<<gq, kThreads, 0, s>>>(p);
  }
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int attention_fwd(int dt, const AttnParams& p, hipStream_t s) {
  if (p.b * p.h == 0 || p.sq == 0) return 0;
  if (dt == BF16) {
    if (p.d == 64) return launch_fwd<bf16, 64>(p, s);
    if (p.d == 128) return launch_fwd<bf16, 128>(p, s);
  } else if (dt == F16) {
    if (p.d == 64) return launch_fwd<f16, 64>(p, s);
    if (p.d == 128) return launch_fwd<f16, 128>(p, s);
  }
  return -3;
}

int attention_bwd(int dt, const AttnBwdParams& p, hipStream_t s) {
  if (p.f.b * p.f.h == 0 || p.f.sq == 0) return 0;
  if (dt == BF16) {
    if (p.f.d == 64) return launch_bwd<bf16, 64>(p, s);
    if (p.f.d == 128) return launch_bwd<bf16, 128>(p, s);
  } else if (dt == F16) {
    if (p.f.d == 64) return launch_bwd<f16, 64>(p, s);
    if (p.f.d == 128) return launch_bwd<f16, 128>(p, s);
  }
  return -3;
}

}  // namespace smpk
