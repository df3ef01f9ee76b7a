// Fused flash-attention backward, head dim 64, causal self-attention (sq == sk): ONE kernel
// computes dK, dV AND dQ -- five MFMA products per tile (S = Q K^T, dP = dO V^T, dV^T += dO^T P,
// dK^T += Q^T dS, dQ += dS K) instead of the split design's seven (its dQ kernel recomputes S
// and dP).  Reference: the unfused backward of `smp/torch/nn/transformer.py:1617-1708`.
//
// Structure (MI355X-first):
//  * one workgroup = kWaves waves (default 8: 2 per SIMD, one workgroup per CU) = 32 kWaves keys
//    of one (b, h); each wave owns 32 keys with the key on the MFMA lane (the dK/dV kernel's
//    per-wave code: S / dP accumulators are the B operands of dV^T / dK^T), dK / dV stay in
//    registers for the whole sweep;
//  * the workgroup sweeps the 64-query tiles its keys are visible to, two barriers per tile;
//    every wave writes its dS^T (32 keys x 64 queries, bf16) into ONE LDS image, and after the
//    middle barrier computes its 16 x 16 tiles of the tile's dQ over all the block's keys
//    (v_mfma_f32_16x16x32, dS^T and K both by ds_read_b64_tr_b16 from [key-quad][16-column
//    block][4][16] images, block index XOR quad parity and 8-byte slots XOR quad & 3: the dS^T
//    stores and the transposed reads are bank-conflict free);
//  * dQ is summed across the key blocks of a (b, h) DETERMINISTICALLY by an ordered hand-off
//    (cdna_hip_programming.md §6 Guideline 16, row 1 of the sc1 table): for query tile i the key
//    blocks add in DESCENDING order -- the diagonal block stores first, kb = 0 adds last and
//    writes dQ in bf16.  With ascending query tiles that is exactly the order in which the
//    blocks reach tile i.  Partials are fp32 in a private [tile][wave][part][lane][4] layout,
//    stored and loaded with sc1 (write-through / L1-bypassing) 16-byte buffer accesses; a tile's
//    flag is published at the next tile's middle barrier (every wave retired the stores with a
//    counted vmcnt first) by one lane; the consumer looks at the flag half a tile before it
//    needs the partial and, when it is already up, loads the partial a whole tile ahead; else
//    it polls (relaxed agent-scope loads, bounded spin with s_sleep).  Workgroups are dispatched
//    so that a block's predecessor (kb + 1, same (b, h)) always has the lower id on the same
//    XCD queue.  A timed-out wait sets the error word and proceeds (no GPU hang; tests assert
//    it stayed 0).
//  * delta = rowsum(dO o O) comes from a small pre-kernel (the split design's dQ kernel computed
//    it on the fly).
// Fixed summation order everywhere: bitwise reproducible.
//
// Status (profiles/r5/attention_fused_bwd.md): correct and deterministic, but at the GPT-2 XL
// shape still 4 % (no dropout) / 15 % (dropout) slower than the split kernels -- the dQ partial
// loads cost ~270 us per layer inside the tile schedule -- so it is opt-in (SMP_ATTN_FUSED_BWD=1).
#include "attention_impl.h"

namespace smpk {
namespace attn {
namespace fused {

// waves per workgroup: 8 = one workgroup per CU.  (4 waves / two workgroups per CU doubles the
// hand-off traffic and spilled with dropout: profiles/r5/attention_fused_bwd.md)
constexpr int kWaves = 8;
constexpr int kNT = 64 * kWaves;          // threads per workgroup
constexpr int kKeys = 32 * kWaves;        // keys per workgroup (32 per wave, key on the lane)
constexpr int kQI = 8 / kWaves;           // 16-query dQ row blocks per wave (x 2 d blocks)
constexpr int kParts = 2 * kQI;           // 16 x 16 dQ tiles per wave
constexpr int kBQ = 64;           // queries per tile
constexpr int kD = 64;
constexpr int kBROW = kBQ + 8;    // keep-bit staging row (words), as the dK/dV kernel

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

template <typename T>
struct MF16;
template <>
struct MF16<bf16> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct MF16<f16> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// [key quad][16-column block ^ (quad & 1)][4 keys][16 columns] image of a [256][64] tile, the
// 4-column (8-byte) slots of each 16-column row XOR-swizzled by (quad & 3): element offset of
// (key, col).  The dS^T stores (ds_write_b64: 16 lanes = 4 quads x 4 keys at one column) then
// cover all 32 banks of their group, and the transposed fragment reads (two 32-lane groups =
// 2 quads x 4 keys x 4 slots) all 64.
__device__ __forceinline__ int qimg(int key, int col) {
  const int kq = key >> 2;
  return ((kq * 4 + ((col >> 4) ^ (kq & 1))) << 6) + ((key & 3) << 4) + ((((col >> 2) & 3) ^ (kq & 3)) << 2) + (col & 3);
}

// 16 x 32 operand fragment for v_mfma_16x16x32 from a qimg image at k-step ks (keys 32 ks ..):
// 16-lane group g, read r take key quad 8 ks + g + 4 r (keys 32 ks + 4 g + 16 r + 0..3), lane
// 4 qq + p of the group supplies key row qq, columns col0 + 4 p .. + 3; lane i receives column
// col0 + i.  The A and B operands use the same (group, element) -> key map, so the k-sum is exact.
// Split into a per-lane base (k-step 0) and a compile-time k-step: key quad 8 ks + g has the
// parity (and quad & 3) of g, so k-step ks sits exactly 2048 elements (4 KB) past k-step 0 and
// the second read 1024 elements past the first -- both fold into the ds_read offset field, and a
// fully unrolled k loop needs one address register per operand instead of one per read.
__device__ __forceinline__ const uint16_t* qfrag_base(const uint16_t* img, int col0, int lane) {
  // key quad 8 ks + g (+ 4): quad & 3 == g, so the slot swizzle is p ^ g at every k-step
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  return img + ((g * 4 + ((col0 >> 4) ^ (g & 1))) << 6) + (qq << 4) + ((p ^ g) << 2);
}
template <typename T>
__device__ __forceinline__ typename MF16<T>::e8 qfrag_at(const uint16_t* base, int ks) {
  s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 2048 * ks));
  s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + 2048 * ks + 1024));
  s16x8 v = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  return __builtin_bit_cast(typename MF16<T>::e8, v);
}

__device__ __forceinline__ int poll_flag(int* flag, int want, int* err) {
  // relaxed agent-scope (sc1) loads, one lane; bounded (~30 ms at 2 GHz), then the error word --
  // and once any wait of the launch has timed out, no later wait spins (a protocol bug must not
  // turn into a GPU hang: the launch finishes with wrong dQ and the error word set)
  for (uint32_t spins = 0;; ++spins) {
    const int v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == want) return 1;  // exactly the predecessor's mark (later blocks lower it again)
    if ((spins & 255u) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return 0;
    if (spins > (1u << 20)) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// delta[bh][q] = sum_d dO[q][d] O[q][d] (fp32).  Rows are walked in (b, q, h) order -- the
// memory order of the [b, s, h, d] O / dO tensors -- with 8 lanes per 64-element row (one
// 16-byte vector each, fully coalesced) and a 3-step shuffle sum.
template <typename T>
__global__ __launch_bounds__(256) void delta_kernel(AttnBwdParams P) {
  const AttnParams& p = P.f;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t row = t >> 3;  // (b, q, h) linear
  const int c = static_cast<int>(t & 7);
  const bool ok = row < p.b * p.sq * p.h;
  float acc = 0.f;
  int64_t b = 0, q = 0, h = 0;
  if (ok) {
    h = row % p.h;
    q = (row / p.h) % p.sq;
    b = row / (p.h * p.sq);
    const uint16_t* o = static_cast<const uint16_t*>(p.o) + b * p.o_sb + h * p.o_sh + q * p.o_ss + 8 * c;
    const uint16_t* d = static_cast<const uint16_t*>(P.dout) + b * P.do_sb + h * P.do_sh + q * P.do_ss + 8 * c;
    const typename MF<T>::e8 a = ld8<T>(o), e = ld8<T>(d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(static_cast<float>(a[j]), static_cast<float>(e[j]), acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (ok && c == 0) P.delta[(b * p.h + h) * p.sq + q] = acc;
}

template <typename T, bool DROP>
__global__ void __launch_bounds__(kNT, 2) attn_bwd_fused_kernel(AttnBwdParams P) {
  constexpr int D = kD, DS = kD;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[kBQ * DS];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[kBQ * DS];
  __shared__ __attribute__((aligned(16))) uint16_t sKb[kKeys * D];   // qimg image of the block's K
  __shared__ __attribute__((aligned(16))) uint16_t sDS[kKeys * kBQ];  // qimg image of dS^T
  __shared__ __attribute__((aligned(16))) float sL[kBQ], sDl[kBQ];
  __shared__ __attribute__((aligned(16))) uint32_t sBits[DROP ? 2 * (kKeys / 64) * kBROW : 4];
  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk);
  const int nkb = (sk + kKeys - 1) / kKeys;
  const int ntq = (sq + kBQ - 1) / kBQ;
  int t_id;
  int64_t bh;
  xcd_map(nkb, p.b * p.h, t_id, bh);
  const int kb = nkb - 1 - t_id;  // descending: a block's predecessor (kb + 1) has the lower id
  const int64_t b = bh / p.h, h = bh % p.h;
  const int k0w = kb * kKeys + wave * 32;
  const int krow = k0w + r;

  const uint16_t* Q = static_cast<const uint16_t*>(p.q) + b * p.q_sb + h * p.q_sh;
  const uint16_t* K = static_cast<const uint16_t*>(p.k) + b * p.k_sb + h * p.k_sh;
  const uint16_t* V = static_cast<const uint16_t*>(p.v) + b * p.v_sb + h * p.v_sh;
  const uint16_t* dO = static_cast<const uint16_t*>(P.dout) + b * P.do_sb + h * P.do_sh;
  const float* LSE = p.lse + bh * p.sq;
  const float* DL = P.delta + bh * p.sq;

  // this wave's K / V fragments (B operands of S = Q K^T and dP = dO V^T, key on the lane)
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
  // the block's 256 K rows -> qimg image (B operand of dQ = dS K): 4 x 16 B per thread
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = threadIdx.x + i * kNT, key = c >> 3, ch = c & 7;
    const int gk = kb * kKeys + key;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (gk < sk) v = *reinterpret_cast<const uint4*>(K + static_cast<int64_t>(gk) * p.k_ss + ch * 8);
    *reinterpret_cast<uint2*>(sKb + qimg(key, ch * 8)) = make_uint2(v.x, v.y);  // two swizzled slots
    *reinterpret_cast<uint2*>(sKb + qimg(key, ch * 8 + 4)) = make_uint2(v.z, v.w);
  }
  f32x16 dv[D / 32], dk[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dv[i] = dk[i] = f32x16{0};
  const float sl2 = p.scale * kLog2e;
  const float inv_sl2 = 1.f / sl2;
  const uint32_t kbit = drop_bit(wave & 1, 4 * (r >> 3) + (r & 3));
  const int bits_row = ((wave >> 1) * 2 + ((r >> 2) & 1)) * kBROW;
  const int ntiles64 = (sk + 63) >> 6;
  // keep-bit staging: thread t -> (64-key tile kb*4 + t>>7, query (t>>1)&63, half-wave t&1)
  const int st_tile = kb * (kKeys / 64) + static_cast<int>(threadIdx.x >> 7), st_q = (threadIdx.x >> 1) & 63;
  const int st_hh = threadIdx.x & 1;
  const uint32_t rsd_bits = __builtin_bit_cast(uint32_t, p.drop_rs);

  // query tiles [qt_begin, ntq): the first holds the block's first key
  const int qt_begin = (kb * kKeys) / kBQ;
  // register staging of one 64 x 64 Q / dO tile: kStg 16-B chunks per thread (rows st_row + 32 i)
  constexpr int kStg = kBQ * 8 / kNT;
  const int st_row = threadIdx.x >> 3, st_ch = threadIdx.x & 7;
  uint4 qst[kStg], ost[kStg];
  float l_stage = 0.f, d_stage = 0.f;
  uint32_t bits_stage = 0u;
  auto load_tile = [&](int qt) {
    const int q0 = qt * kBQ;
#pragma unroll
    for (int i = 0; i < kStg; ++i) {
      const int qq = q0 + st_row + i * (kNT / 8);
      qst[i] = qq < sq ? *reinterpret_cast<const uint4*>(Q + static_cast<int64_t>(qq) * p.q_ss + st_ch * 8)
                       : make_uint4(0, 0, 0, 0);
      ost[i] = qq < sq ? *reinterpret_cast<const uint4*>(dO + static_cast<int64_t>(qq) * P.do_ss + st_ch * 8)
                       : make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x < kBQ) {
      const int qr = q0 + threadIdx.x;
      l_stage = qr < sq ? LSE[qr] : 0.f;
      d_stage = qr < sq ? DL[qr] : 0.f;
    }
    if (DROP) {
      const int qb = q0 + st_q;
      bits_stage = qb < sq && st_tile < ntiles64 ? p.drop_bits[bits_index(bh, ntiles64, st_tile, sq, qb, st_hh)] : 0u;
    }
  };
  const RowOff<D> ro(r, hh);
  const TrOff<D> tro(lane);

  // dQ hand-off state
  constexpr int kTileF = kBQ * kD;  // fp32 partial of one query tile
  float* acc_base = P.dq_acc + bh * static_cast<int64_t>(ntq) * kTileF;
  int* flags = P.dq_flags + bh * ntq;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      acc_base, 0, static_cast<int>(static_cast<int64_t>(ntq) * kTileF * sizeof(float)), 0x00020000);
  // this wave's dQ tiles: queries 16 (kQI qg + i), d blocks db0 + j (i < kQI, j < 2)
  const int qg = wave >> 1, db0 = 2 * (wave & 1);
  // the wave's kParts x 16 B of a partial: [tile][wave][i][j][lane][4] fp32
  auto part_off = [&](int qt, int t) {
    return (qt * kTileF + ((wave * kParts + t) * 64 + lane) * 4) * static_cast<int>(sizeof(float));
  };
  int pend = -1;  // the tile whose partial this block stored last, flag not yet published
  bool ready_next = false;  // the next tile's predecessor partial was published a tile early

  // the staged registers -> the tile's LDS images (sQ / sdO / row constants / keep bits)
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < kStg; ++i) {
      const int o = swz<D>(st_row + i * (kNT / 8), st_ch);
      *reinterpret_cast<uint4*>(sQ + o) = qst[i];
      *reinterpret_cast<uint4*>(sdO + o) = ost[i];
    }
    if (threadIdx.x < kBQ) {
      sL[threadIdx.x] = l_stage == -INFINITY ? 0.f : -l_stage * kLog2e * inv_sl2;
      sDl[threadIdx.x] = -d_stage;
    }
    if (DROP) sBits[((threadIdx.x >> 7) * 2 + (threadIdx.x & 1)) * kBROW + ((threadIdx.x >> 1) & 63)] = bits_stage;
  };
  if (qt_begin < ntq) {
    load_tile(qt_begin);
    store_tile();
  }
  // Two barriers per tile.  The top one makes the tile's staging (written during the previous
  // tile's dQ phase) visible and ends every wave's reads of the previous dS^T image; the middle
  // one completes this tile's dS^T image and ends every wave's reads of sQ / sdO, so the next
  // tile's registers are staged right after it -- before this tile's partial stores: the staged
  // loads then never sit behind those stores in the in-order vmcnt (staging at the loop top made
  // the compiler wait for vmcnt(0), i.e. for the stores, on every tile).
  for (int qt = qt_begin; qt < ntq; ++qt) {
    const int q0 = qt * kBQ;
    __syncthreads();
    // the predecessor (block kb + 1) adds into this tile before this block; the diagonal block
    // stores first.  When the flag read half a tile ago already shows the predecessor's partial,
    // its loads go out now and have the whole tile to land; otherwise the flag is looked at again now and
    // awaited between the two sub-steps.
    const int kb_first = imin(nkb - 1, (q0 + kBQ - 1) / kKeys);
    const bool has_pred = kb < kb_first;
    f32x4 pred[kParts];
#pragma unroll
    for (int t = 0; t < kParts; ++t) pred[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool early = has_pred && ready_next;
    if (early) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: loads stay below the flag
#pragma unroll
      for (int t = 0; t < kParts; ++t)
        pred[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, part_off(qt, t), 0, 16));
    }
    const bool prefetch = qt + 1 < ntq;
    if (prefetch) load_tile(qt + 1);
    const bool next_pred = prefetch && kb < imin(nkb - 1, (q0 + 2 * kBQ - 1) / kKeys);
    int fnext;
    // Flag words are loaded by every lane and read unconditionally (readfirstlane): a load whose
    // destination register stays "maybe pending" on some path makes the compiler wait for
    // vmcnt(0) where that register is next written -- behind the partial stores or right after
    // the predecessor loads.
    const int flag0 = __hip_atomic_load(flags + qt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- two 32-query sub-steps: S, dP, dV, dK (key on the lane) and this wave's dS^T columns
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool seen = u == 1 && __builtin_amdgcn_readfirstlane(flag0) == kb + 2;
      if (u == 1 && has_pred && !early) {
        if (lane == 0 && !seen) (void)poll_flag(flags + qt, kb + 2, P.dq_err);
        __builtin_amdgcn_wave_barrier();
        // no instruction: keeps the partial's loads below the poll (the loads are sc1, L1-bypassing)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t = 0; t < kParts; ++t)
          pred[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, part_off(qt, t), 0, 16));
      }
      if (u == 1) {
        // the next tile's flag, for its early start; looked at before this tile's partial stores
        // (no wait on them: vmcnt is in order)
        fnext = __hip_atomic_load(flags + imin(qt + 1, ntq - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int qs = q0 + 32 * u;
      const bool vis = qs + 31 >= k0w;        // some query sees some of the wave's keys
      const bool interior = qs >= k0w + 31 && qs + 31 < sq && k0w + 31 < sk;
      typename MF<T>::e8 sf0, sf1;
      if (vis) {
        f32x16 s, dp, ndl;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 lv = *reinterpret_cast<const float4*>(&sL[32 * u + 8 * g + 4 * hh]);
          const float4 dv4 = *reinterpret_cast<const float4*>(&sDl[32 * u + 8 * g + 4 * hh]);
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
          s = MF<T>::mma(ld8<T>(sQ + ro.o[t] + 32 * u * DS), kf[t], s);
          dp = MF<T>::mma(ld8<T>(sdO + ro.o[t] + 32 * u * DS), vf[t], dp);
        }
        // dO^T fragments of the dV MFMAs ahead of the element-wise work
        typename MF<T>::e8 tdo[D / 32][2];
        {
          const int a0 = 32 * u * DS, a1 = (32 * u + 16) * DS;
#pragma unroll
          for (int i = 0; i < D / 32; ++i) {
            tdo[i][0] = ld_tr<T>(sdO, tro.lo[i] + a0, tro.hi[i] + a0);
            tdo[i][1] = ld_tr<T>(sdO, tro.lo[i] + a1, tro.hi[i] + a1);
          }
        }
        uint4 kw[4];
        if (DROP) {
#pragma unroll
          for (int g = 0; g < 4; ++g) kw[g] = *reinterpret_cast<const uint4*>(&sBits[bits_row + 32 * u + 8 * g + 4 * hh]);
        }
        f32x2 po[8], dso[8];
        const f32x2 sl2v = {sl2, sl2};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int reg = 2 * j;
          const f32x2 sa = f32x2{s[reg], s[reg + 1]} * sl2v;
          f32x2 pv = {fast_exp2(sa.x), fast_exp2(sa.y)};
          if (!interior) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int qq = qs + acc_row(reg + e, hh);
              if (qq >= sq || krow >= sk || krow > qq) pv[e] = 0.f;
            }
          }
          const f32x2 dpv = {dp[reg], dp[reg + 1]};
          if (DROP) {
            const uint4 w4 = kw[reg >> 2];
            const uint32_t wa = (reg & 2) ? w4.z : w4.x, wb = (reg & 2) ? w4.w : w4.y;
            const f32x2 z = {__builtin_bit_cast(float, bit_mask(wa, kbit) & rsd_bits),
                             __builtin_bit_cast(float, bit_mask(wb, kbit) & rsd_bits)};
            po[j] = pv * z;
            dso[j] = pv * __builtin_elementwise_fma(dpv, z, f32x2{ndl[reg], ndl[reg + 1]});
          } else {
            po[j] = pv;
            dso[j] = dpv * pv;
          }
        }
        const typename MF<T>::e8 pf0 = pack8p<T>(po, 0), pf1 = pack8p<T>(po, 1);
        sf0 = pack8p<T>(dso, 0);
        sf1 = pack8p<T>(dso, 1);
#pragma unroll
        for (int i = 0; i < D / 32; ++i) {
          const int a0 = 32 * u * DS, a1 = (32 * u + 16) * DS;
          dv[i] = MF<T>::mma(tdo[i][0], pf0, dv[i]);
          dv[i] = MF<T>::mma(tdo[i][1], pf1, dv[i]);
          dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a0, tro.hi[i] + a0), sf0, dk[i]);
          dk[i] = MF<T>::mma(ld_tr<T>(sQ, tro.lo[i] + a1, tro.hi[i] + a1), sf1, dk[i]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sf0[j] = MF<T>::cvt(0.f);
          sf1[j] = MF<T>::cvt(0.f);
        }
      }
      // dS^T columns (queries 32 u + 8 g + 4 hh + 0..3 of key krow) -> the image, 8 B each:
      // sf0 elements 0-3 = register group 0, 4-7 = group 1; sf1 = groups 2, 3
      const int key = wave * 32 + r;
      const u32x4 a = __builtin_bit_cast(u32x4, sf0), c = __builtin_bit_cast(u32x4, sf1);
      const int qb = 32 * u + 4 * hh;
      *reinterpret_cast<uint2*>(sDS + qimg(key, qb)) = make_uint2(a[0], a[1]);
      *reinterpret_cast<uint2*>(sDS + qimg(key, qb + 8)) = make_uint2(a[2], a[3]);
      *reinterpret_cast<uint2*>(sDS + qimg(key, qb + 16)) = make_uint2(c[0], c[1]);
      *reinterpret_cast<uint2*>(sDS + qimg(key, qb + 24)) = make_uint2(c[2], c[3]);
    }
    // the previous tile's partial stores: retired by every wave before the barrier (the vector
    // memory operations issued after them -- this tile's prefetch and predecessor loads, at least
    // `newer` per wave -- may stay in flight: vmcnt retires in order), then published after it
    if (pend >= 0) {
      const int newer = (prefetch ? 2 * kStg : 0) + (has_pred ? kParts : 0) + 0;
      if (newer >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (newer >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (newer >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (newer >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // the tile's dS^T image is complete; sQ / sdO are free
    if (pend >= 0 && threadIdx.x == 0) __hip_atomic_store(flags + pend, kb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pend = -1;
    if (prefetch) store_tile();
    // ---- dQ tiles of this wave over the block's keys: 4 k-steps of 32, fully unrolled with the
    // fragments read one k-step ahead (a rolled loop exposed the transposed-read latency at every
    // k-step).  Keys no query of the tile sees carry dS = 0.
    f32x4 acc[kQI][2];
#pragma unroll
    for (int t = 0; t < kParts; ++t) acc[t >> 1][t & 1] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      const uint16_t* pa[kQI];
#pragma unroll
      for (int i = 0; i < kQI; ++i) pa[i] = qfrag_base(sDS, 16 * (kQI * qg + i), lane);
      const uint16_t* pb0 = qfrag_base(sKb, 16 * db0, lane);
      const uint16_t* pb1 = qfrag_base(sKb, 16 * db0 + 16, lane);
      typename MF16<T>::e8 af[2][kQI], bf[2][2];
#pragma unroll
      for (int i = 0; i < kQI; ++i) af[0][i] = qfrag_at<T>(pa[i], 0);
      bf[0][0] = qfrag_at<T>(pb0, 0);
      bf[0][1] = qfrag_at<T>(pb1, 0);
#pragma unroll
      for (int ks = 0; ks < kKeys / 32; ++ks) {
        const int c = ks & 1, n = c ^ 1;
        if (ks + 1 < kKeys / 32) {
#pragma unroll
          for (int i = 0; i < kQI; ++i) af[n][i] = qfrag_at<T>(pa[i], ks + 1);
          bf[n][0] = qfrag_at<T>(pb0, ks + 1);
          bf[n][1] = qfrag_at<T>(pb1, ks + 1);
        }
#pragma unroll
        for (int t = 0; t < kParts; ++t) acc[t >> 1][t & 1] = MF16<T>::mma(af[c][t >> 1], bf[c][t & 1], acc[t >> 1][t & 1]);
        __builtin_amdgcn_sched_barrier(0);  // keep the reads one k-step ahead, no further
      }
    }
#pragma unroll
    for (int t = 0; t < kParts; ++t) acc[t >> 1][t & 1] += pred[t];
    // (read unconditionally: a conditional read left the flag register "maybe pending" at the
    // loop top, where the compiler then waited for vmcnt(0) -- i.e. for the partial stores)
    ready_next = (__builtin_amdgcn_readfirstlane(fnext) == kb + 2) && next_pred;
    if (kb == 0) {
      // last in the order: dQ = scale * sum, bf16; lane (l & 15, l >> 4) of tile (i, j) holds
      // rows 16 (kQI qg + i) + 4 (l >> 4) + e, column 16 (db0 + j) + (l & 15)
      uint16_t* dQ = static_cast<uint16_t*>(P.dq) + b * P.dq_sb + h * P.dq_sh;
#pragma unroll
      for (int i = 0; i < kQI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int qq = q0 + 16 * (kQI * qg + i) + 4 * (lane >> 4) + e;
          if (qq < sq) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
              dQ[static_cast<int64_t>(qq) * P.dq_ss + 16 * (db0 + j) + (lane & 15)] =
                  __builtin_bit_cast(uint16_t, MF<T>::cvt(acc[i][j][e] * p.scale));
          }
        }
    } else {
#pragma unroll
      for (int t = 0; t < kParts; ++t)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[t >> 1][t & 1]), rsrc, part_off(qt, t), 0, 16);
      pend = qt;
    }
  }
  // publish what is still pending
  if (pend >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + pend, kb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (krow >= sk) return;
  uint16_t* dK = static_cast<uint16_t*>(P.dk) + b * P.dk_sb + h * P.dk_sh + static_cast<int64_t>(krow) * P.dk_ss;
  uint16_t* dV = static_cast<uint16_t*>(P.dv) + b * P.dv_sb + h * P.dv_sh + static_cast<int64_t>(krow) * P.dv_ss;
  store_rows<T, D, D / 32>(dK, dk, p.scale, hh);
  store_rows<T, D, D / 32>(dV, dv, 1.f, hh);
}

template <typename T, bool DROP>
int launch(const AttnBwdParams& p, hipStream_t s) {
  const int64_t nbh = p.f.b * p.f.h;
  const unsigned gd = static_cast<unsigned>((nbh * p.f.sq * 8 + 255) / 256);
  delta_kernel<T><<<gd, 256, 0, s>>>(p);
  const unsigned g = static_cast<unsigned>(((p.f.sk + kKeys - 1) / kKeys) * nbh);
  attn_bwd_fused_kernel<T, DROP><<<g, kNT, 0, s>>>(p);
  return static_cast<int>(hipGetLastError());
}

}  // namespace fused
}  // namespace attn

// Fused backward for D = 64, causal, sq == sk, no key bias / window.  The caller (bindings)
// zeroes p.dq_flags / p.dq_err on the stream before the call and provides p.dq_acc.
int attention_bwd_fused_d64(int dt, const AttnBwdParams& p, hipStream_t s) {
  if (p.f.d != 64 || !p.f.causal || p.f.sq != p.f.sk || p.f.kbias != nullptr || p.f.window > 0 ||
      p.dq_acc == nullptr || p.dq_flags == nullptr || p.dq_err == nullptr)
    return -5;
  const bool dr = p.f.drop_on != 0;
  if (dt == BF16) return dr ? attn::fused::launch<bf16, true>(p, s) : attn::fused::launch<bf16, false>(p, s);
  if (dt == F16) return dr ? attn::fused::launch<f16, true>(p, s) : attn::fused::launch<f16, false>(p, s);
  return -3;
}

}  // namespace smpk
