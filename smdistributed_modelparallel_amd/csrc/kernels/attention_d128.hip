// Flash attention, head dim 128: instantiation unit of attention_impl.h.
#include "attention_impl.h"

namespace smpk {
SMPK_ATTN_HEAD_DIM(128)
}  // namespace smpk
