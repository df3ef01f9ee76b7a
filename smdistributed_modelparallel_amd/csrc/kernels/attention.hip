// Flash attention entry points: dispatch on head dim to the per-D instantiation units
// (attention_d{64,96,128,256}.hip; kernels in attention_impl.h).
#include "kernels.h"

namespace smpk {

int attention_fwd_d64(int, const AttnParams&, hipStream_t);
int attention_fwd_d96(int, const AttnParams&, hipStream_t);
int attention_fwd_d128(int, const AttnParams&, hipStream_t);
int attention_fwd_d256(int, const AttnParams&, hipStream_t);
int attention_bwd_d64(int, const AttnBwdParams&, hipStream_t);
int attention_bwd_d96(int, const AttnBwdParams&, hipStream_t);
int attention_bwd_d128(int, const AttnBwdParams&, hipStream_t);
int attention_bwd_d256(int, const AttnBwdParams&, hipStream_t);

bool attention_head_dim_supported(int64_t d) { return d == 64 || d == 96 || d == 128 || d == 256; }

int attention_fwd(int dt, const AttnParams& p, hipStream_t s) {
  if (p.b * p.h == 0 || p.sq == 0) return 0;
  switch (p.d) {
    case 64: return attention_fwd_d64(dt, p, s);
    case 96: return attention_fwd_d96(dt, p, s);
    case 128: return attention_fwd_d128(dt, p, s);
    case 256: return attention_fwd_d256(dt, p, s);
    default: return -3;
  }
}

int attention_bwd(int dt, const AttnBwdParams& p, hipStream_t s) {
  if (p.f.b * p.f.h == 0 || p.f.sq == 0) return 0;
  if (p.f.drop_on && p.f.drop_bits == nullptr) return -4;  // dropout backward reads the forward's keep bits
  switch (p.f.d) {
    case 64: return attention_bwd_d64(dt, p, s);
    case 96: return attention_bwd_d96(dt, p, s);
    case 128: return attention_bwd_d128(dt, p, s);
    case 256: return attention_bwd_d256(dt, p, s);
    default: return -3;
  }
}

}  // namespace smpk
