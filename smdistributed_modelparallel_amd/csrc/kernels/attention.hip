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

// Transposed fetch of an A/B operand element set from a row-major LDS tile:
// elements j=0..3 <- rows k0..k0+3, j=4..7 <- rows k0+8..k0+11, all at column `col`
// (col = c0 + (lane & 15) implied by the 16-lane group addressing).
template <typename T>
__device__ __forceinline__ typename MF<T>::e8 ld_tr(const uint16_t* tile, int ldrow, int k0, int c0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const uint16_t* a0 = tile + (k0 + q) * ldrow + c0 + 4 * p;
  const uint16_t* a1 = a0 + 8 * ldrow;
  s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
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

// Cooperative copy of a [rows x D] tile (row stride `gs` elements) into padded LDS.
template <int D>
__device__ __forceinline__ void load_tile(uint16_t* lds, const uint16_t* g, int64_t gs, int row0, int nrows_valid,
                                          int rows) {
  constexpr int CH = D / 8;  // 16-byte chunks per row
  constexpr int LD = D + 8;
  for (int c = threadIdx.x; c < rows * CH; c += kThreads) {
    const int r = c / CH, k = c % CH;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nrows_valid) v = *reinterpret_cast<const uint4*>(g + static_cast<int64_t>(row0 + r) * gs + k * 8);
    *reinterpret_cast<uint4*>(lds + r * LD + k * 8) = v;
  }
}

// ================================================================== forward
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_kernel(AttnParams p) {
  constexpr int BM = 128, BN = 64, LD = D + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sK[BN * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sV[BN * LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int64_t bh = blockIdx.y;
  const int64_t b = bh / p.h, h = bh % p.h;
  const int nqb = static_cast<int>((p.sq + BM - 1) / BM);
  const int qb = CAUSAL ? (nqb - 1 - static_cast<int>(blockIdx.x)) : static_cast<int>(blockIdx.x);
  const int q0 = qb * BM + wave * 32;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk);
  const int diag = sk - sq;  // key index allowed up to query + diag

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

  int kv_end = sk;
  if (CAUSAL) {
    const int lim = (qb + 1) * BM + diag;
    kv_end = lim < sk ? lim : sk;
  }
  const int wave_last_q = q0 + 31;
  for (int kv0 = 0; kv0 < kv_end; kv0 += BN) {
    __syncthreads();
    load_tile<D>(sK, K, p.k_ss, kv0, sk - kv0, BN);
    load_tile<D>(sV, V, p.v_ss, kv0, sk - kv0, BN);
    __syncthreads();
    if (CAUSAL && kv0 > wave_last_q + diag) continue;
    if (p.window > 0 && kv0 + BN - 1 < q0 + diag - p.window + 1) continue;
    f32x16 s0 = f32x16{0}, s1 = f32x16{0};
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
      s0 = MF<T>::mma(ld8<T>(sK + r * LD + 16 * t + 8 * hh), qf[t], s0);
      s1 = MF<T>::mma(ld8<T>(sK + (32 + r) * LD + 16 * t + 8 * hh), qf[t], s1);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int k0 = kv0 + acc_row(reg, hh);
      const int k1 = k0 + 32;
      float v0 = s0[reg] * sl2, v1 = s1[reg] * sl2;
      if (k0 >= sk || (CAUSAL && k0 > qrow + diag) || (p.window > 0 && k0 <= qrow + diag - p.window)) v0 = -INFINITY;
      if (k1 >= sk || (CAUSAL && k1 > qrow + diag) || (p.window > 0 && k1 <= qrow + diag - p.window)) v1 = -INFINITY;
      s0[reg] = v0;
      s1[reg] = v1;
      mx = fmaxf(mx, fmaxf(v0, v1));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_i, mx);
    const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m_i - m_new);
    float rs = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const float e0 = (m_new == -INFINITY) ? 0.f : exp2f(s0[reg] - m_new);
      const float e1 = (m_new == -INFINITY) ? 0.f : exp2f(s1[reg] - m_new);
      s0[reg] = e0;
      s1[reg] = e1;
      rs += e0 + e1;
    }
    rs += __shfl_xor(rs, 32, 64);
    l_i = l_i * alpha + rs;
    m_i = m_new;
#pragma unroll
    for (int i = 0; i < D / 32; ++i) o[i] *= alpha;
    typename MF<T>::e8 pf[4] = {pack8<T>(s0, 0), pack8<T>(s0, 1), pack8<T>(s1, 0), pack8<T>(s1, 1)};
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
      const int c0 = 32 * i + 16 * ((lane >> 4) & 1);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kb = 16 * s + 4 * hh;
        o[i] = MF<T>::mma(ld_tr<T>(sV, LD, kb, c0, lane), pf[s], o[i]);
      }
    }
  }
  if (qrow >= sq) return;
  const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
  uint16_t* O = static_cast<uint16_t*>(p.o) + b * p.o_sb + h * p.o_sh + static_cast<int64_t>(qrow) * p.o_ss;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * i + 8 * g + 4 * hh;
      s16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = __builtin_bit_cast(short, MF<T>::cvt(o[i][4 * g + j] * inv));
      *reinterpret_cast<s16x4*>(O + d0) = w;
    }
  }
  if (hh == 0) p.lse[bh * p.sq + qrow] = (l_i > 0.f) ? (m_i + log2f(l_i)) / kLog2e : -INFINITY;
}

// ============================================================= delta = rowsum(dO * O)
template <typename T>
__global__ void __launch_bounds__(kThreads) attn_delta_kernel(AttnBwdParams p) {
  // one wave per (b, h, query) row
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int64_t total = p.f.b * p.f.h * p.f.sq;
  if (row >= total) return;
  const int64_t q = row % p.f.sq, bh = row / p.f.sq, b = bh / p.f.h, h = bh % p.f.h;
  const T* O = static_cast<const T*>(p.f.o) + b * p.f.o_sb + h * p.f.o_sh + q * p.f.o_ss;
  const T* dO = static_cast<const T*>(p.dout) + b * p.do_sb + h * p.do_sh + q * p.do_ss;
  float acc = 0.f;
  for (int d = lane; d < p.f.d; d += 64) acc += to_f32(O[d]) * to_f32(dO[d]);
  acc = wave_sum(acc);
  if (lane == 0) p.delta[row] = acc;
}

// ===================================================================== dK / dV
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, 2) attn_bwd_dkdv_kernel(AttnBwdParams P) {
  constexpr int BKEYS = 128, BQ = 64, LD = D + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[BQ * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[BQ * LD];
  __shared__ float sL[BQ], sDl[BQ];
  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int64_t bh = blockIdx.y, b = bh / p.h, h = bh % p.h;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk), diag = sk - sq;
  const int nkb = (sk + BKEYS - 1) / BKEYS;
  const int kb = CAUSAL ? static_cast<int>(blockIdx.x) : static_cast<int>(blockIdx.x);
  (void)nkb;
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
  int q_start = 0;
  if (CAUSAL) {
    q_start = kb * BKEYS - diag;
    q_start = q_start < 0 ? 0 : (q_start / BQ) * BQ;
  }
  for (int qt = q_start; qt < sq; qt += BQ) {
    __syncthreads();
    load_tile<D>(sQ, Q, p.q_ss, qt, sq - qt, BQ);
    load_tile<D>(sdO, dO, P.do_ss, qt, sq - qt, BQ);
    if (threadIdx.x < BQ) {
      const int qq = qt + threadIdx.x;
      sL[threadIdx.x] = qq < sq ? LSE[qq] * kLog2e : 0.f;
      sDl[threadIdx.x] = qq < sq ? DL[qq] : 0.f;
    }
    __syncthreads();
    if (CAUSAL && qt + BQ - 1 + diag < k0w) continue;  // whole tile sees none of this wave's keys
#pragma unroll 1
    for (int sub = 0; sub < 2; ++sub) {
      // S = Q K^T, dP = dO V^T for 32 queries x 32 keys (query rows in regs, key on lane)
      f32x16 s = f32x16{0}, dp = f32x16{0};
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        s = MF<T>::mma(ld8<T>(sQ + (32 * sub + r) * LD + 16 * t + 8 * hh), kf[t], s);
        dp = MF<T>::mma(ld8<T>(sdO + (32 * sub + r) * LD + 16 * t + 8 * hh), vf[t], dp);
      }
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int ql = 32 * sub + acc_row(reg, hh);
        const int qq = qt + ql;
        float pv = exp2f(s[reg] * sl2 - sL[ql]);
        if (qq >= sq || krow >= sk || (CAUSAL && krow > qq + diag) ||
            (p.window > 0 && krow <= qq + diag - p.window))
          pv = 0.f;
        s[reg] = pv;
        dp[reg] = pv * (dp[reg] - sDl[ql]);
      }
      // dV^T += dO^T P ; dK^T += Q^T dS   (B operands = accumulators, A via transposed reads)
      typename MF<T>::e8 pf0 = pack8<T>(s, 0), pf1 = pack8<T>(s, 1);
      typename MF<T>::e8 sf0 = pack8<T>(dp, 0), sf1 = pack8<T>(dp, 1);
#pragma unroll
      for (int i = 0; i < D / 32; ++i) {
        const int c0 = 32 * i + 16 * ((lane >> 4) & 1);
        const int kq = 32 * sub + 4 * hh;
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, LD, kq, c0, lane), pf0, dv[i]);
        dv[i] = MF<T>::mma(ld_tr<T>(sdO, LD, kq + 16, c0, lane), pf1, dv[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, LD, kq, c0, lane), sf0, dk[i]);
        dk[i] = MF<T>::mma(ld_tr<T>(sQ, LD, kq + 16, c0, lane), sf1, dk[i]);
      }
    }
  }
  if (krow >= sk) return;
  uint16_t* dK = static_cast<uint16_t*>(P.dk) + b * P.dk_sb + h * P.dk_sh + static_cast<int64_t>(krow) * P.dk_ss;
  uint16_t* dV = static_cast<uint16_t*>(P.dv) + b * P.dv_sb + h * P.dv_sh + static_cast<int64_t>(krow) * P.dv_ss;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * i + 8 * g + 4 * hh;
      s16x4 wk, wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wk[j] = __builtin_bit_cast(short, MF<T>::cvt(dk[i][4 * g + j] * p.scale));
        wv[j] = __builtin_bit_cast(short, MF<T>::cvt(dv[i][4 * g + j]));
      }
      *reinterpret_cast<s16x4*>(dK + d0) = wk;
      *reinterpret_cast<s16x4*>(dV + d0) = wv;
    }
  }
}

// ========================================================================= dQ
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, 2) attn_bwd_dq_kernel(AttnBwdParams P) {
  constexpr int BM = 128, BN = 64, LD = D + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sK[BN * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sV[BN * LD];
  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int64_t bh = blockIdx.y, b = bh / p.h, h = bh % p.h;
  const int nqb = static_cast<int>((p.sq + BM - 1) / BM);
  const int qb = CAUSAL ? (nqb - 1 - static_cast<int>(blockIdx.x)) : static_cast<int>(blockIdx.x);
  const int q0 = qb * BM + wave * 32;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk), diag = sk - sq;
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
  const float lse2 = qrow < sq ? p.lse[bh * p.sq + qrow] * kLog2e : 0.f;
  const float dl = qrow < sq ? P.delta[bh * p.sq + qrow] : 0.f;
  const float sl2 = p.scale * kLog2e;
  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dq[i] = f32x16{0};
  int kv_end = sk;
  if (CAUSAL) {
    const int lim = (qb + 1) * BM + diag;
    kv_end = lim < sk ? lim : sk;
  }
  for (int kv0 = 0; kv0 < kv_end; kv0 += BN) {
    __syncthreads();
    load_tile<D>(sK, K, p.k_ss, kv0, sk - kv0, BN);
    load_tile<D>(sV, V, p.v_ss, kv0, sk - kv0, BN);
    __syncthreads();
    if (CAUSAL && kv0 > q0 + 31 + diag) continue;
    // S^T = K Q^T, dP^T = V dO^T  (key rows in regs, query on lane)
    f32x16 s[2], dp[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      s[u] = f32x16{0};
      dp[u] = f32x16{0};
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        s[u] = MF<T>::mma(ld8<T>(sK + (32 * u + r) * LD + 16 * t + 8 * hh), qf[t], s[u]);
        dp[u] = MF<T>::mma(ld8<T>(sV + (32 * u + r) * LD + 16 * t + 8 * hh), df[t], dp[u]);
      }
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int kk = kv0 + 32 * u + acc_row(reg, hh);
        float pv = exp2f(s[u][reg] * sl2 - lse2);
        if (qrow >= sq || kk >= sk || (CAUSAL && kk > qrow + diag) || (p.window > 0 && kk <= qrow + diag - p.window))
          pv = 0.f;
        dp[u][reg] = pv * (dp[u][reg] - dl);  // dS^T
      }
    }
    // dQ^T += K^T dS^T  (B = dS^T accumulator, A = K^T via transposed reads of sK)
    typename MF<T>::e8 sf[4] = {pack8<T>(dp[0], 0), pack8<T>(dp[0], 1), pack8<T>(dp[1], 0), pack8<T>(dp[1], 1)};
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
      const int c0 = 32 * i + 16 * ((lane >> 4) & 1);
#pragma unroll
      for (int st = 0; st < 4; ++st) dq[i] = MF<T>::mma(ld_tr<T>(sK, LD, 16 * st + 4 * hh, c0, lane), sf[st], dq[i]);
    }
  }
  if (qrow >= sq) return;
  uint16_t* dQ = static_cast<uint16_t*>(P.dq) + b * P.dq_sb + h * P.dq_sh + static_cast<int64_t>(qrow) * P.dq_ss;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * i + 8 * g + 4 * hh;
      s16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = __builtin_bit_cast(short, MF<T>::cvt(dq[i][4 * g + j] * p.scale));
      *reinterpret_cast<s16x4*>(dQ + d0) = w;
    }
  }
}

template <typename T, int D>
int launch_fwd(const AttnParams& p, hipStream_t s) {
  dim3 grid(static_cast<unsigned>((p.sq + 127) / 128), static_cast<unsigned>(p.b * p.h));
  if (p.causal)
    attn_fwd_kernel<T, D, true><<<grid, kThreads, 0, s>>>(p);
  else
    attn_fwd_kernel<T, D, false><<<grid, kThreads, 0, s>>>(p);
  return static_cast<int>(hipGetLastError());
}

template <typename T, int D>
int launch_bwd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = p.f.b * p.f.h * p.f.sq;
  attn_delta_kernel<T><<<static_cast<unsigned>((rows + 3) / 4), kThreads, 0, s>>>(p);
  dim3 gk(static_cast<unsigned>((p.f.sk + 127) / 128), static_cast<unsigned>(p.f.b * p.f.h));
  dim3 gq(static_cast<unsigned>((p.f.sq + 127) / 128), static_cast<unsigned>(p.f.b * p.f.h));
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
