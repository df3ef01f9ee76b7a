// Flash attention, head dim 64: instantiation unit of attention_impl.h.  The dQ kernel is
// instantiated in attention_d64_dq.hip (built without SLP vectorisation).
#include "attention_impl.h"

namespace smpk {
namespace attn {
#define SMPK_DQ64_EXTERN(T, C, DR, BI)                                                 \
  extern template void launch_dq<T, 64, C, DR, BI>(const AttnBwdParams&, unsigned, hipStream_t);
SMPK_ATTN_VARIANTS(SMPK_DQ64_EXTERN)
}  // namespace attn
SMPK_ATTN_HEAD_DIM(64)
}  // namespace smpk
