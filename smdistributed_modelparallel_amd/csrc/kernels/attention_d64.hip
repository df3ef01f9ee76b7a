// Flash attention, head dim 64: instantiation unit of attention_impl.h.
#include "attention_impl.h"

namespace smpk {
SMPK_ATTN_HEAD_DIM(64)
}  // namespace smpk
