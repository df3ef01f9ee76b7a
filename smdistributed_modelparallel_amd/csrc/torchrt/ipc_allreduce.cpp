// IpcAllReduce: one-shot all-reduce for small tensor-parallel messages over hipIpc mappings.
//
// Reference: the TP all-reduces of `smp/torch/nn/utils.py:548,570` (f/g collectives),
// `nn/layer_norm.py:41-79` (distributed-LN statistics) and `nn/cross_entropy.py:34-66`
// (vocab-parallel CE max / sum-exp / target logit) all go to NCCL, whose ring all-reduce
// is latency-bound at these sizes (KBs to ~1 MB: [B, s] statistics, small-batch
// activations).  SURVEY §5.8 asks for a one-shot path for TP groups of <= 4-8 GPUs.
//
// MI355X design (ours): every rank owns a registered buffer of 2 x max_bytes (double-
// buffered data slots) and a flag array, both exported by hipIpc and mapped by every peer of
// the group once.  One kernel per call, one workgroup per contiguous chunk:
//   1. copy the chunk of the input into this rank's data slot (epoch parity),
//   2. system-scope release, then PUSH the epoch into every peer's flag array
//      (flag[src rank][chunk]) -- remote stores over xGMI,
//   3. poll the LOCAL flag array (peers pushed into it) until every peer's epoch arrived,
//      bounded by a wall-clock timeout,
//   4. read the chunk from every peer's slot (xGMI) and reduce in rank order 0..world-1 in
//      fp32 -- bitwise the same result on every rank, as TP requires.
// Failure is never silent: a timeout (a peer skipped a call, died or drifted past the
// timeout) writes the error word in host-mapped pinned memory (the host reads it without any
// synchronisation at step end and raises), pushes an ABORT word into every peer's flag array
// (their next or current kernels fail too, so the error surfaces on every rank), and the
// kernel writes NaN -- not the stale slots -- into its output.  Once an instance has failed,
// every later call on it fails the same way.
// Slot reuse is safe with two slots: a rank writes slot (e % 2) at epoch e + 2 only after
// every peer's chunk pushed epoch e + 1, which a peer does after its epoch-e kernel finished
// reading.  All calls of one instance must be issued in the same order on every rank, on
// one stream per rank (the TP collectives run on the compute stream).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <cstring>
#include <string>
#include <vector>

namespace py = pybind11;

namespace smprt_torch {

namespace {

constexpr int kMaxRanks = 8;
// One wave per workgroup and at most 64 workgroups (a quarter of the CUs): the spinning waits
// of a call hold no LDS and few wave slots, so they never keep a full-LDS GEMM workgroup off
// the CUs they sit on (with 128 x 256-thread workgroups each taking an LDS
// word, a TP rank's spinning one-shot kernel could starve a co-resident rank's GEMM when the
// ranks share a GPU).
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 64;
constexpr int kAbortWord = kMaxRanks * kMaxBlocks;  // index of the abort word in a flag array
constexpr int kFlagWords = kAbortWord + 64;          // the abort word on a line of its own

void ar_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "IpcAllReduce: ", what, " failed: ", hipGetErrorString(e));
}

struct ArParams {
  const void* in;
  void* out;
  int64_t n;       // elements
  int64_t chunk;   // elements per workgroup (multiple of 8)
  const char* slot[kMaxRanks];      // data slot of every rank for this epoch (own included)
  uint32_t* peer_flags[kMaxRanks];  // flag array of every rank (mapped)
  uint32_t* my_flags;
  int* err;  // host-mapped pinned word
  int rank, world, op;  // op 0 = sum, 1 = max
  uint32_t epoch;
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
};

template <typename T>
__device__ __forceinline__ float ld_f(const T* p) { return static_cast<float>(p[0]); }
template <>
__device__ __forceinline__ float ld_f<__hip_bfloat16>(const __hip_bfloat16* p) { return __bfloat162float(p[0]); }
template <>
__device__ __forceinline__ float ld_f<__half>(const __half* p) { return __half2float(p[0]); }

template <typename T>
__device__ __forceinline__ T from_f(float x) { return static_cast<T>(x); }
template <>
__device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float x) { return __float2bfloat16(x); }
template <>
__device__ __forceinline__ __half from_f<__half>(float x) { return __float2half(x); }

template <typename T>
__global__ void __launch_bounds__(kThreads) oneshot_allreduce_kernel(ArParams p) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t lo = static_cast<int64_t>(b) * p.chunk;
  const int64_t hi = lo + p.chunk < p.n ? lo + p.chunk : p.n;
  constexpr int V = 16 / sizeof(T);  // elements per 16-byte vector
  const int64_t vlo = lo / V, vhi = hi / V;  // lo is a multiple of 8 >= V
  // 1. input chunk -> own slot
  {
    const uint4* src = static_cast<const uint4*>(p.in);
    uint4* dst = reinterpret_cast<uint4*>(const_cast<char*>(p.slot[p.rank]));
    for (int64_t i = vlo + tid; i < vhi; i += kThreads) dst[i] = src[i];
    const T* s1 = static_cast<const T*>(p.in);
    T* d1 = reinterpret_cast<T*>(const_cast<char*>(p.slot[p.rank]));
    for (int64_t i = vhi * V + tid; i < hi; i += kThreads) d1[i] = s1[i];
  }
  // 2. publish: the wave's stores visible at system scope (one wave: the fence orders all of
  // them before the pushes), then push the epoch
  __threadfence_system();
  if (tid < p.world && tid != p.rank) {
    __hip_atomic_store(p.peer_flags[tid] + p.rank * kMaxBlocks + b, p.epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every peer's chunk (bounded; a peer's abort ends the wait too)
  bool fail = false;
  if (tid < p.world && tid != p.rank) {
    const uint32_t* f = p.my_flags + tid * kMaxBlocks + b;
    const uint32_t* ab = p.my_flags + kAbortWord;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    fail = __hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    while (!fail &&
           static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - p.epoch) < 0) {
      if (__hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        fail = true;
      } else if (__builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
        fail = true;
        // tell every peer: their pending and future calls on this group fail as well
        for (int r = 0; r < p.world; ++r)
          __hip_atomic_store(p.peer_flags[r] + kAbortWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (fail) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // the polling lanes' verdict reaches the whole wave by a vote (no LDS)
  const bool any_fail = __any(fail);
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // (system-scope acquire by the polling lanes above)
  if (any_fail) {  // never reduce stale slots: the output is poisoned, the host raises at step end
    T* out = static_cast<T*>(p.out);
    const T nan = from_f<T>(__builtin_nanf(""));
    for (int64_t i = lo + tid; i < hi; i += kThreads) out[i] = nan;
    return;
  }
  // 4. reduce in rank order (identical on every rank)
  T* out = static_cast<T*>(p.out);
  for (int64_t i = vlo + tid; i < vhi; i += kThreads) {
    float acc[V];
    {
      const uint4 v = reinterpret_cast<const uint4*>(p.slot[0])[i];
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = ld_f<T>(e + j);
    }
    for (int r = 1; r < p.world; ++r) {
      const uint4 v = reinterpret_cast<const uint4*>(p.slot[r])[i];
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = p.op == 0 ? acc[j] + ld_f<T>(e + j) : fmaxf(acc[j], ld_f<T>(e + j));
    }
    uint4 o;
    T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int j = 0; j < V; ++j) oe[j] = from_f<T>(acc[j]);
    reinterpret_cast<uint4*>(out)[i] = o;
  }
  for (int64_t i = vhi * V + tid; i < hi; i += kThreads) {
    float acc = ld_f<T>(reinterpret_cast<const T*>(p.slot[0]) + i);
    for (int r = 1; r < p.world; ++r) {
      const float x = ld_f<T>(reinterpret_cast<const T*>(p.slot[r]) + i);
      acc = p.op == 0 ? acc + x : fmaxf(acc, x);
    }
    out[i] = from_f<T>(acc);
  }
}

}  // namespace

class IpcAllReduce {
 public:
  IpcAllReduce(int device, int rank, int world, int64_t max_bytes)
      : device_(device), rank_(rank), world_(world), max_bytes_((max_bytes + 255) / 256 * 256) {
    TORCH_CHECK(world >= 1 && world <= kMaxRanks, "IpcAllReduce: group size must be 1..", kMaxRanks);
    TORCH_CHECK(rank >= 0 && rank < world, "IpcAllReduce: bad rank");
    ar_check(hipSetDevice(device_), "hipSetDevice");
    ar_check(hipMalloc(&data_, 2 * max_bytes_), "hipMalloc(data)");
    const size_t fbytes = sizeof(uint32_t) * kFlagWords;
    // flags: uncached device memory (peers' pushes land in HBM, the poll reads HBM);
    // plain device memory if this allocation kind cannot be exported
    uncached_flags_ = hipExtMallocWithFlags(&flags_, fbytes, hipDeviceMallocUncached) == hipSuccess;
    if (uncached_flags_) {
      hipIpcMemHandle_t h;
      if (hipIpcGetMemHandle(&h, flags_) != hipSuccess) {
        (void)hipGetLastError();
        hipFree(flags_);
        uncached_flags_ = false;
      }
    } else {
      (void)hipGetLastError();
    }
    if (!uncached_flags_) ar_check(hipMalloc(&flags_, fbytes), "hipMalloc(flags)");
    ar_check(hipMemset(flags_, 0, fbytes), "hipMemset(flags)");
    // error word in host-mapped pinned memory: kernels store into it, the host polls it with
    // a plain load (no stream or device synchronisation on the step path)
    ar_check(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(int), hipHostMallocMapped | hipHostMallocCoherent),
             "hipHostMalloc(err)");
    *err_host_ = 0;
    ar_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_), err_host_, 0), "hipHostGetDevicePointer(err)");
    ar_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    peer_data_.assign(world_, nullptr);
    peer_flags_.assign(world_, nullptr);
    peer_data_[rank_] = static_cast<char*>(data_);
    peer_flags_[rank_] = static_cast<uint32_t*>(flags_);
  }

  ~IpcAllReduce() { close(); }

  // (data handle bytes, flags handle bytes) to be exchanged within the group
  py::tuple handles() {
    hipIpcMemHandle_t hd, hf;
    ar_check(hipIpcGetMemHandle(&hd, data_), "hipIpcGetMemHandle(data)");
    ar_check(hipIpcGetMemHandle(&hf, flags_), "hipIpcGetMemHandle(flags)");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&hd), sizeof(hd)),
                          py::bytes(reinterpret_cast<const char*>(&hf), sizeof(hf)));
  }

  // handles[r] = (data, flags) of group rank r (own entry ignored)
  void open(const std::vector<std::pair<py::bytes, py::bytes>>& handles) {
    TORCH_CHECK(static_cast<int>(handles.size()) == world_, "IpcAllReduce.open: need one handle pair per rank");
    ar_check(hipSetDevice(device_), "hipSetDevice");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      std::string d = handles[r].first, f = handles[r].second;
      TORCH_CHECK(d.size() == sizeof(hipIpcMemHandle_t) && f.size() == sizeof(hipIpcMemHandle_t),
                  "IpcAllReduce.open: malformed handle");
      hipIpcMemHandle_t hd, hf;
      std::memcpy(&hd, d.data(), sizeof(hd));
      std::memcpy(&hf, f.data(), sizeof(hf));
      void *pd = nullptr, *pf = nullptr;
      ar_check(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(data)");
      ar_check(hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(flags)");
      peer_data_[r] = static_cast<char*>(pd);
      peer_flags_[r] = static_cast<uint32_t*>(pf);
      opened_.push_back(pd);
      opened_.push_back(pf);
    }
    ready_ = true;
  }

  bool fits(const at::Tensor& t) const {
    return t.is_cuda() && t.is_contiguous() && t.numel() * t.element_size() <= max_bytes_ &&
           (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf || t.scalar_type() == at::kFloat) &&
           reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  }

  // in-place (out may alias in) all-reduce of `t` on the current stream; op: 0 sum, 1 max
  void all_reduce(const at::Tensor& in, at::Tensor out, int op, double timeout_s) {
    TORCH_CHECK(ready_, "IpcAllReduce: open() was not called");
    TORCH_CHECK(fits(in), "IpcAllReduce: tensor does not fit (contiguous bf16/f16/f32, 16-B aligned, <= ",
                max_bytes_, " B)");
    TORCH_CHECK(out.is_contiguous() && out.numel() == in.numel() && out.scalar_type() == in.scalar_type() &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "IpcAllReduce: output must match the input (contiguous, 16-B aligned)");
    TORCH_CHECK(op == 0 || op == 1, "IpcAllReduce: op must be 0 (sum) or 1 (max)");
    const int64_t n = in.numel();
    if (n == 0) return;
    ++epoch_;
    ArParams p{};
    p.in = in.data_ptr();
    p.out = out.data_ptr();
    p.n = n;
    // chunks of >= 2 KB, multiples of 8 elements, at most kMaxBlocks of them
    const int64_t min_chunk = 2048 / in.element_size();
    int64_t chunk = (n + kMaxBlocks - 1) / kMaxBlocks;
    chunk = chunk < min_chunk ? min_chunk : chunk;
    chunk = (chunk + 7) / 8 * 8;
    p.chunk = chunk;
    const int blocks = static_cast<int>((n + chunk - 1) / chunk);
    const int64_t slot_off = (epoch_ & 1) ? max_bytes_ : 0;
    for (int r = 0; r < world_; ++r) {
      p.slot[r] = peer_data_[r] + slot_off;
      p.peer_flags[r] = peer_flags_[r];
    }
    p.my_flags = static_cast<uint32_t*>(flags_);
    p.err = err_;
    p.rank = rank_;
    p.world = world_;
    p.op = op;
    p.epoch = epoch_;
    p.timeout_ticks = static_cast<uint64_t>(timeout_s * 1e8);
    hipStream_t s = at::hip::getCurrentHIPStream(device_).stream();
    switch (in.scalar_type()) {
      case at::kBFloat16:
        hipLaunchKernelGGL(oneshot_allreduce_kernel<__hip_bfloat16>, dim3(blocks), dim3(kThreads), 0, s, p);
        break;
      case at::kHalf:
        hipLaunchKernelGGL(oneshot_allreduce_kernel<__half>, dim3(blocks), dim3(kThreads), 0, s, p);
        break;
      default:
        hipLaunchKernelGGL(oneshot_allreduce_kernel<float>, dim3(blocks), dim3(kThreads), 0, s, p);
    }
    ar_check(hipGetLastError(), "oneshot_allreduce_kernel launch");
    calls_++;
  }

  // 1 if a kernel of this instance failed (own timeout or a peer's abort).  Non-blocking: a
  // plain read of the host-mapped error word; kernels still running are seen by a later call.
  int error(bool reset) {
    const int h = __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
    if (reset && h) __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE);
    return h;
  }

  // Test hook: this rank behaves as if its kernel had timed out (own error + abort pushed to
  // every peer's flag array); used to exercise the failure path without a 10-minute wait.
  void inject_abort() {
    ar_check(hipSetDevice(device_), "hipSetDevice");
    const uint32_t one = 1;
    for (int r = 0; r < world_; ++r)
      ar_check(hipMemcpy(peer_flags_[r] + kAbortWord, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy(abort)");
    __atomic_store_n(err_host_, 1, __ATOMIC_RELEASE);
  }

  void close() {
    if (data_ == nullptr) return;
    hipSetDevice(device_);
    hipDeviceSynchronize();
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    hipFree(data_);
    hipFree(flags_);
    hipHostFree(err_host_);
    err_host_ = nullptr;
    err_ = nullptr;
    data_ = nullptr;
    ready_ = false;
  }

  py::dict stats() const {
    py::dict d;
    d["calls"] = calls_;
    d["epoch"] = static_cast<int64_t>(epoch_);
    d["max_bytes"] = max_bytes_;
    d["uncached_flags"] = uncached_flags_;
    return d;
  }

  int64_t max_bytes() const { return max_bytes_; }

 private:
  int device_, rank_, world_;
  int64_t max_bytes_;
  void* data_ = nullptr;
  void* flags_ = nullptr;
  int* err_ = nullptr;       // device view of err_host_
  int* err_host_ = nullptr;  // hipHostMalloc'd, mapped + coherent
  bool uncached_flags_ = false;
  bool ready_ = false;
  uint32_t epoch_ = 0;
  int64_t calls_ = 0;
  std::vector<char*> peer_data_;
  std::vector<uint32_t*> peer_flags_;
  std::vector<void*> opened_;
};

void register_ipc_allreduce(py::module& m) {
  py::class_<IpcAllReduce>(m, "IpcAllReduce")
      .def(py::init<int, int, int, int64_t>(), py::arg("device"), py::arg("rank"), py::arg("world"),
           py::arg("max_bytes"))
      .def("handles", &IpcAllReduce::handles)
      .def("open", &IpcAllReduce::open)
      .def("fits", &IpcAllReduce::fits)
      .def("all_reduce", &IpcAllReduce::all_reduce, py::arg("input"), py::arg("output"), py::arg("op") = 0,
           py::arg("timeout_s") = 5.0)
      .def("error", &IpcAllReduce::error, py::arg("reset") = true)
      .def("inject_abort", &IpcAllReduce::inject_abort)
      .def("close", &IpcAllReduce::close)
      .def("stats", &IpcAllReduce::stats)
      .def_property_readonly("max_bytes", &IpcAllReduce::max_bytes);
}

}  // namespace smprt_torch
