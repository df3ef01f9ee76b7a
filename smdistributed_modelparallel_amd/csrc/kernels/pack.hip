// Pack / unpack for the tensor-parallel collectives (K21; reference native
// smp_torch_nccl_allgatherv / scatter_and_merge, smp/torch/collectives.py:214-242).
//
// One generic strided 4-D copy dst[i0,i1,i2,i3] = src[i0,i1,i2,i3] (element strides on both
// sides) moves a shard between its tensor layout and the [rank, rows, ...] layout RCCL's
// all-gather / reduce-scatter / all-to-all want, in ONE pass -- instead of pad (cat with
// zeros) + movedim().contiguous() + split/cat.  Padding rows of an uneven split are left
// uninitialised: the receiver discards them.
//
// When the innermost dim is unit-stride on both sides and 16-byte aligned, each thread
// moves 16 bytes; otherwise one element.  Grid-stride loop over the flattened index, the
// 4-D coordinate decomposed from it (sizes are kernel arguments, divisions by runtime
// values -- the copy is memory-bound).
#include "common.h"
#include "kernels.h"

namespace smpk {
namespace {

struct Copy4 {
  int64_t n0, n1, n2, n3;  // sizes (n3 counted in vectors for the vector path)
  int64_t s0, s1, s2, s3;  // src strides (elements or vectors)
  int64_t d0, d1, d2, d3;  // dst strides
};

template <typename V>
__global__ void __launch_bounds__(256) strided_copy4_kernel(const V* __restrict__ src, V* __restrict__ dst, Copy4 c,
                                                            int64_t total) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += step) {
    int64_t r = i;
    const int64_t i3 = r % c.n3;
    r /= c.n3;
    const int64_t i2 = r % c.n2;
    r /= c.n2;
    const int64_t i1 = r % c.n1;
    const int64_t i0 = r / c.n1;
    dst[i0 * c.d0 + i1 * c.d1 + i2 * c.d2 + i3 * c.d3] = src[i0 * c.s0 + i1 * c.s1 + i2 * c.s2 + i3 * c.s3];
  }
}

template <typename V>
int launch(const void* src, void* dst, Copy4 c, hipStream_t s) {
  const int64_t total = c.n0 * c.n1 * c.n2 * c.n3;
  if (total == 0) return 0;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  strided_copy4_kernel<V><<<static_cast<unsigned>(blocks), 256, 0, s>>>(static_cast<const V*>(src),
                                                                         static_cast<V*>(dst), c, total);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int strided_copy4(int elem_bytes, const void* src, void* dst, const int64_t* sizes, const int64_t* ss,
                  const int64_t* ds, hipStream_t s) {
  Copy4 c{sizes[0], sizes[1], sizes[2], sizes[3], ss[0], ss[1], ss[2], ss[3], ds[0], ds[1], ds[2], ds[3]};
  // 16-byte vectors when the innermost run is contiguous on both sides and every row start
  // stays 16-byte aligned
  const int per = 16 / elem_bytes;
  const bool vec = ss[3] == 1 && ds[3] == 1 && sizes[3] % per == 0 &&
                   ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0 &&
                   ss[0] % per == 0 && ss[1] % per == 0 && ss[2] % per == 0 && ds[0] % per == 0 &&
                   ds[1] % per == 0 && ds[2] % per == 0;
  if (vec) {
    Copy4 v{c.n0, c.n1, c.n2, c.n3 / per, c.s0 / per, c.s1 / per, c.s2 / per, 1, c.d0 / per, c.d1 / per, c.d2 / per, 1};
    return launch<uint4>(src, dst, v, s);
  }
  switch (elem_bytes) {
    case 1: return launch<uint8_t>(src, dst, c, s);
    case 2: return launch<uint16_t>(src, dst, c, s);
    case 4: return launch<uint32_t>(src, dst, c, s);
    case 8: return launch<uint64_t>(src, dst, c, s);
    default: return -3;
  }
}

namespace {
// grid-stride copy of n16 16-byte vectors, then the byte tail by the first block
__global__ void __launch_bounds__(256) device_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int64_t n16, const uint8_t* __restrict__ tsrc,
                                                          uint8_t* __restrict__ tdst, int tail) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && static_cast<int>(threadIdx.x) < tail) tdst[threadIdx.x] = tsrc[threadIdx.x];
}

__global__ void __launch_bounds__(256) device_copy_bytes_kernel(const uint8_t* __restrict__ src,
                                                                uint8_t* __restrict__ dst, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}
}  // namespace

int device_copy(void* dst, const void* src, int64_t nbytes, hipStream_t s) {
  if (nbytes <= 0) return 0;
  const bool aligned = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  if (aligned) {
    const int64_t n16 = nbytes / 16;
    const int tail = static_cast<int>(nbytes - n16 * 16);
    // enough workgroups to fill the chip (2048 x 256 threads), grid-stride beyond
    const int64_t want = (n16 + 255) / 256;
    const unsigned grid = static_cast<unsigned>(want < 1 ? 1 : (want > 2048 ? 2048 : want));
    device_copy_kernel<<<grid, 256, 0, s>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16,
                                            static_cast<const uint8_t*>(src) + n16 * 16,
                                            static_cast<uint8_t*>(dst) + n16 * 16, tail);
  } else {
    const int64_t want = (nbytes + 255) / 256;
    const unsigned grid = static_cast<unsigned>(want > 2048 ? 2048 : want);
    device_copy_bytes_kernel<<<grid, 256, 0, s>>>(static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst),
                                                  nbytes);
  }
  return static_cast<int>(hipGetLastError());
}

}  // namespace smpk
