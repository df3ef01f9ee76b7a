// Standalone attention kernel bench + numerics check (no torch): times the fused forward
// and backward at a GPT-2 XL shape and checks both against a host fp32 reference at a
// small shape.  Built by tools/gpu_attn_variants.sh with -D switches to A/B kernel
// variants of csrc/kernels/attention.hip inside one GPU call.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<kernels> attention.hip attn_bench.cpp
//   ./attn_bench [B S H D iters]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kernels.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return static_cast<uint16_t>(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

struct Problem {
  int b, s, h, d;
  bool causal;
  // packed qkv [b, s, 3, h, d]; o, dout [b, s, h, d]; dqkv like qkv
  uint16_t *qkv, *o, *dout, *dqkv;
  float *lse, *delta;
  smpk::AttnBwdParams P;

  Problem(int b_, int s_, int h_, int d_, bool c) : b(b_), s(s_), h(h_), d(d_), causal(c) {
    const size_t nq = static_cast<size_t>(b) * s * 3 * h * d, no = static_cast<size_t>(b) * s * h * d;
    CK(hipMalloc(&qkv, nq * 2));
    CK(hipMalloc(&dqkv, nq * 2));
    CK(hipMalloc(&o, no * 2));
    CK(hipMalloc(&dout, no * 2));
    CK(hipMalloc(&lse, static_cast<size_t>(b) * h * s * 4));
    CK(hipMalloc(&delta, static_cast<size_t>(b) * h * s * 4));
    std::mt19937 rng(1234);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<uint16_t> hq(nq), ho(no);
    for (auto& x : hq) x = f2bf(nd(rng));
    for (auto& x : ho) x = f2bf(nd(rng));
    CK(hipMemcpy(qkv, hq.data(), nq * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dout, ho.data(), no * 2, hipMemcpyHostToDevice));
    memset(&P, 0, sizeof(P));
    auto& p = P.f;
    const int64_t ss = 3LL * h * d, sb = ss * s;
    p.q = qkv;
    p.k = qkv + static_cast<size_t>(h) * d;
    p.v = qkv + 2 * static_cast<size_t>(h) * d;
    p.b = b, p.h = h, p.sq = s, p.sk = s, p.d = d;
    p.q_sb = p.k_sb = p.v_sb = sb;
    p.q_ss = p.k_ss = p.v_ss = ss;
    p.q_sh = p.k_sh = p.v_sh = d;
    p.o = o;
    p.o_sb = static_cast<int64_t>(s) * h * d, p.o_ss = static_cast<int64_t>(h) * d, p.o_sh = d;
    p.lse = lse;
    p.scale = 1.f / sqrtf(static_cast<float>(d));
    p.causal = c ? 1 : 0;
    p.window = 0;
    P.dout = dout;
    P.do_sb = p.o_sb, P.do_ss = p.o_ss, P.do_sh = p.o_sh;
    P.dq = dqkv;
    P.dk = dqkv + static_cast<size_t>(h) * d;
    P.dv = dqkv + 2 * static_cast<size_t>(h) * d;
    P.dq_sb = P.dk_sb = P.dv_sb = sb;
    P.dq_ss = P.dk_ss = P.dv_ss = ss;
    P.dq_sh = P.dk_sh = P.dv_sh = d;
    P.delta = delta;
    P.dq_acc = nullptr;
  }
  ~Problem() {
    for (void* x : {static_cast<void*>(qkv), static_cast<void*>(dqkv), static_cast<void*>(o), static_cast<void*>(dout),
                    static_cast<void*>(lse), static_cast<void*>(delta)})
      (void)hipFree(x);
  }
  void fwd() {
    if (smpk::attention_fwd(smpk::BF16, P.f, 0)) {
      fprintf(stderr, "attention_fwd launch failed\n");
      exit(3);
    }
  }
  void bwd() {
    if (smpk::attention_bwd(smpk::BF16, P, 0)) {
      fprintf(stderr, "attention_bwd launch failed\n");
      exit(3);
    }
  }
};

// host fp32 reference of O, dQ, dK, dV (bf16 inputs) for one small problem
static int check(bool causal) {
  const int b = 1, s = 320, h = 2, d = 64;  // s not a multiple of the tiles: edge paths run
  Problem pr(b, s, h, d, causal);
  pr.fwd();
  pr.bwd();
  CK(hipDeviceSynchronize());
  const size_t nq = static_cast<size_t>(b) * s * 3 * h * d, no = static_cast<size_t>(b) * s * h * d;
  std::vector<uint16_t> qkv(nq), o(no), dout(no), dqkv(nq);
  CK(hipMemcpy(qkv.data(), pr.qkv, nq * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o.data(), pr.o, no * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(dout.data(), pr.dout, no * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(dqkv.data(), pr.dqkv, nq * 2, hipMemcpyDeviceToHost));
  auto at = [&](const std::vector<uint16_t>& t, int which, int i, int hh, int c) {
    return bf2f(t[((static_cast<size_t>(i) * 3 + which) * h + hh) * d + c]);
  };
  const float scale = 1.f / sqrtf(static_cast<float>(d));
  double err[4] = {0, 0, 0, 0}, ref[4] = {0, 0, 0, 0};
  for (int hh = 0; hh < h; ++hh) {
    std::vector<float> P(static_cast<size_t>(s) * s), dS(static_cast<size_t>(s) * s), O(static_cast<size_t>(s) * d);
    for (int i = 0; i < s; ++i) {
      float mx = -INFINITY;
      for (int j = 0; j < s; ++j) {
        float a = -INFINITY;
        if (!causal || j <= i) {
          a = 0;
          for (int c = 0; c < d; ++c) a += at(qkv, 0, i, hh, c) * at(qkv, 1, j, hh, c);
          a *= scale;
        }
        P[static_cast<size_t>(i) * s + j] = a;
        mx = fmaxf(mx, a);
      }
      double sum = 0;
      for (int j = 0; j < s; ++j) sum += P[static_cast<size_t>(i) * s + j] = expf(P[static_cast<size_t>(i) * s + j] - mx);
      for (int j = 0; j < s; ++j) P[static_cast<size_t>(i) * s + j] /= static_cast<float>(sum);
      for (int c = 0; c < d; ++c) {
        float a = 0;
        for (int j = 0; j < s; ++j) a += P[static_cast<size_t>(i) * s + j] * at(qkv, 2, j, hh, c);
        O[static_cast<size_t>(i) * d + c] = a;
        const float got = bf2f(o[(static_cast<size_t>(i) * h + hh) * d + c]);
        err[0] = fmax(err[0], fabs(got - a));
        ref[0] = fmax(ref[0], fabs(a));
      }
    }
    auto dO = [&](int i, int c) { return bf2f(dout[(static_cast<size_t>(i) * h + hh) * d + c]); };
    for (int i = 0; i < s; ++i) {
      float dl = 0;
      for (int c = 0; c < d; ++c) dl += dO(i, c) * bf2f(o[(static_cast<size_t>(i) * h + hh) * d + c]);
      for (int j = 0; j < s; ++j) {
        float dp = 0;
        for (int c = 0; c < d; ++c) dp += dO(i, c) * at(qkv, 2, j, hh, c);
        dS[static_cast<size_t>(i) * s + j] = P[static_cast<size_t>(i) * s + j] * (dp - dl);
      }
    }
    for (int i = 0; i < s; ++i)
      for (int c = 0; c < d; ++c) {
        float q = 0, k = 0, v = 0;
        for (int j = 0; j < s; ++j) {
          q += dS[static_cast<size_t>(i) * s + j] * at(qkv, 1, j, hh, c);
          k += dS[static_cast<size_t>(j) * s + i] * at(qkv, 0, j, hh, c);
          v += P[static_cast<size_t>(j) * s + i] * dO(j, c);
        }
        const float r3[3] = {q * scale, k * scale, v};
        for (int w = 0; w < 3; ++w) {
          const float got = at(dqkv, w, i, hh, c);
          err[w + 1] = fmax(err[w + 1], fabs(got - r3[w]));
          ref[w + 1] = fmax(ref[w + 1], fabs(r3[w]));
        }
      }
  }
  const char* nm[4] = {"o", "dq", "dk", "dv"};
  int bad = 0;
  for (int w = 0; w < 4; ++w) {
    const double rel = err[w] / (ref[w] > 0 ? ref[w] : 1);
    printf("check causal=%d %s max_abs_err %.3e (rel to max %.3e)\n", causal ? 1 : 0, nm[w], err[w], rel);
    if (!(rel < 2e-2)) bad = 1;
  }
  return bad;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8, S = argc > 2 ? atoi(argv[2]) : 2048, H = argc > 3 ? atoi(argv[3]) : 25,
            D = argc > 4 ? atoi(argv[4]) : 64, iters = argc > 5 ? atoi(argv[5]) : 20;
  int bad = check(true) | check(false);
  Problem pr(B, S, H, D, true);
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  for (int i = 0; i < 3; ++i) pr.fwd(), pr.bwd();
  CK(hipDeviceSynchronize());
  float tf = 0, tb = 0;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(e0, 0));
    pr.fwd();
    CK(hipEventRecord(e1, 0));
    pr.bwd();
    CK(hipEventRecord(e2, 0));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    tf += a, tb += b;
  }
  tf /= iters, tb /= iters;
  // causal FLOPs: fwd 2 GEMMs, bwd 5 GEMMs over half of the s x s scores
  const double half = 0.5 * B * H * static_cast<double>(S) * S * D * 2;
  printf("B=%d S=%d H=%d D=%d causal: fwd %.1f us (%.0f TFLOP/s)  bwd %.1f us (%.0f TFLOP/s)%s\n", B, S, H, D,
         tf * 1e3, 2 * half / (tf * 1e-3) / 1e12, tb * 1e3, 5 * half / (tb * 1e-3) / 1e12, bad ? "  NUMERICS FAIL" : "");
  return bad;
}
