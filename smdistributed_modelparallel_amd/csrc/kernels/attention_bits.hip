// Attention dropout keep bits regenerated from the hash, for the backward of layers whose
// stored bits would be too large (long sequences: b h sq sk / 8 bytes per layer).  The flash
// forward normally stores them (attention_impl.h, "stored keep bits"); above the per-layer
// budget of ops/attention.py it stores none and this kernel writes, right before the layer's
// backward, exactly the words the forward would have stored -- same hash inputs (drop_key,
// drop_block_thr, drop_words, pack_keep) -- into a buffer that lives for that backward only.
//
// One thread per uint32 word ((bh, 64-key tile, query, half) = bits_index order: coalesced
// stores).  Tiles that no key of the query's row can see under the causal mask are skipped
// (the backward never reads their bits as anything but masked).
#include "attention_impl.h"

namespace smpk {
namespace {

__global__ void __launch_bounds__(256) keep_bits_kernel(AttnParams p, uint32_t* __restrict__ bits, int64_t total) {
  const int64_t w = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (w >= total) return;
  const int sq = static_cast<int>(p.sq), sk = static_cast<int>(p.sk);
  const int ntiles64 = (sk + 63) >> 6;
  const int hh = static_cast<int>(w & 1);
  const int64_t r = w >> 1;
  const int q = static_cast<int>(r % sq);
  const int64_t rt = r / sq;
  const int kt = static_cast<int>(rt % ntiles64);
  const int64_t bh = rt / ntiles64;
  const int kv0 = kt * 64;
  if (p.causal && kv0 > q + (sk - sq)) return;
  const uint32_t dkey = attn::drop_key(p, bh);
  const uint32_t bkey = attn::drop_block_key(dkey);
  const uint32_t qbase = static_cast<uint32_t>(q) * static_cast<uint32_t>((sk + 3) >> 2);
  const attn::DropThr d0 = attn::drop_block_thr(p, bkey, static_cast<uint32_t>(q >> 5), static_cast<uint32_t>(kv0 >> 5));
  const attn::DropThr d1 =
      attn::drop_block_thr(p, bkey, static_cast<uint32_t>(q >> 5), static_cast<uint32_t>(kv0 >> 5) + 1);
  uint32_t f0[4], f1[4];
  attn::drop_words(f0, dkey, qbase, kv0, hh, d0.xr, d0.c);
  attn::drop_words(f1, dkey, qbase, kv0 + 32, hh, d1.xr, d1.c);
  bits[w] = attn::pack_keep(f0, f1);
}

}  // namespace

int attention_keep_bits(const AttnParams& p, uint32_t* bits, hipStream_t s) {
  if (!p.drop_on) return -4;
  const int64_t total = p.b * p.h * ((p.sk + 63) / 64) * p.sq * 2;
  if (total == 0) return 0;
  keep_bits_kernel<<<static_cast<unsigned>((total + 255) / 256), 256, 0, s>>>(p, bits, total);
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
