// Flash attention, head dim 96: instantiation unit of attention_impl.h.
#include "attention_impl.h"

namespace smpk {
SMPK_ATTN_HEAD_DIM(96)
}  // namespace smpk
