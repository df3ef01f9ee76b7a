// Flash attention, head dim 64: the dQ kernel's instantiation unit, built with
// -fno-slp-vectorize (_build.py): without packed fp32 VALU beside its MFMAs the dQ kernel runs
// 1203 vs 1260 us at GPT-2 XL b32 (same-box kernel traces, profiles/r3/s3_rehearsal.md), while
// the dK/dV kernel is faster with it (1546 vs 1590 us) and stays in attention_d64.hip.
#include "attention_impl.h"

namespace smpk {
namespace attn {
#define SMPK_DQ64_INST(T, C, DR, BI)                                                   \
  template void launch_dq<T, 64, C, DR, BI>(const AttnBwdParams&, unsigned, hipStream_t);
SMPK_ATTN_VARIANTS(SMPK_DQ64_INST)
}  // namespace attn
}  // namespace smpk
