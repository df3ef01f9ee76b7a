// IpcP2P: device-to-device pipeline tensor transport over hipIpc mappings (N1c).
//
// Reference: the native D2D engine behind smp_torch_send/recv (smp/torch/ops.py:34-123,
// server_comm.py:260-302) -- CUDA IPC intra-node with an RMM receive pool.
//
// MI355X design (ours):
//  * export(t): the sender publishes the allocation that holds `t` (hipIpcGetMemHandle of
//    the caching-allocator segment, cached per segment and invalidated when the allocator
//    returns the segment to the driver).  Nothing is copied on the sender.
//  * record_event(): one plain HIP event per control message, recorded on the sender's
//    compute stream right after the producer kernels.  The control message is handed to the
//    native mailbox as a GATED send (`csrc/runtime/mailbox.h`): the destination's sender
//    thread releases it (and everything queued after it for that peer, FIFO) only once this
//    event has completed -- `gate_fn()` is the hipEventQuery predicate it calls.  So when a
//    receiver sees the message, the bytes are final: no cross-process device wait (inter-
//    process events) is ever needed.  The sender's host does not block, and neither does the
//    receiver's.
//  * import_copy(dst, ...): the receiver maps the segment once (hipIpcOpenMemHandle with
//    lazy peer enable -- over xGMI when the ranks own different GPUs, plain HBM when they
//    share one) and pulls the bytes with one hipMemcpyAsync D2D on its current stream (the
//    transport's communication stream).  No receive pool is needed because the destination
//    is an ordinary caching-allocator tensor of the receiver.
//  * pull engine, chosen per mapping (SMP_P2P_PULL_ENGINE = auto | kernel | sdma): when the
//    mapped segment lives on ANOTHER GPU (hipPointerGetAttributes), hipMemcpyAsync -- the
//    copy engines (SDMA) move the bytes over xGMI and no CU is taken from the compute kernels
//    the pull overlaps; when both stages share ONE GPU, a copy kernel (smpk::device_copy):
//    there, >= 100 MB hipMemcpyAsync pulls blocked the host thread with four processes
//    time-sharing the GPU (profiles/r4/pp4_hang_root_cause.md).
//  * lifetime: the sender keeps the source tensors and the event slot until the receiver
//    reports (release message, Python side) that its copy has completed.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>

#include "../kernels/kernels.h"
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace smprt_torch {

namespace {

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "IpcP2P: ", what, " failed: ", hipGetErrorString(e));
}

struct SegmentExport {
  size_t size = 0;
  int64_t gen = 0;
  hipIpcMemHandle_t handle;
};

// Segments returned to the driver since the last export lookup (filled by the caching
// allocator's trace tracker, drained under the P2P lock).
std::mutex g_freed_mu;
std::vector<uintptr_t> g_freed;
bool g_tracker_attached = false;

}  // namespace

class IpcP2P {
 public:
  explicit IpcP2P(int device) : device_(device) {
    std::lock_guard<std::mutex> g(g_freed_mu);
    if (!g_tracker_attached) {
      c10::hip::HIPCachingAllocator::attachAllocatorTraceTracker(
          [](const c10::hip::HIPCachingAllocator::TraceEntry& te) {
            if (te.action_ == c10::hip::HIPCachingAllocator::TraceEntry::SEGMENT_FREE ||
                te.action_ == c10::hip::HIPCachingAllocator::TraceEntry::SEGMENT_UNMAP) {
              std::lock_guard<std::mutex> g2(g_freed_mu);
              g_freed.push_back(static_cast<uintptr_t>(te.addr_));
            }
          });
      g_tracker_attached = true;
    }
  }

  ~IpcP2P() { close(); }

  // -> (segment_base, generation, mem_handle_bytes, offset, nbytes)
  py::tuple export_tensor(const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda(), "IpcP2P.export: tensor must be on the GPU");
    TORCH_CHECK(t.is_contiguous(), "IpcP2P.export: tensor must be contiguous");
    int64_t b_out = 0, gen_out = 0, offset = 0, nbytes = 0;
    hipIpcMemHandle_t handle;
    {
      // HIP runtime calls without the GIL (a blocked call must not freeze the process's other
      // Python threads -- the watchdog among them)
      py::gil_scoped_release nogil;
      export_locked_impl(t, b_out, gen_out, handle, offset, nbytes);
    }
    return py::make_tuple(b_out, gen_out, py::bytes(reinterpret_cast<const char*>(&handle), sizeof(hipIpcMemHandle_t)),
                          offset, nbytes);
  }

  void export_locked_impl(const at::Tensor& t, int64_t& b_out, int64_t& gen_out, hipIpcMemHandle_t& handle,
                          int64_t& offset_out, int64_t& nbytes_out) {
    std::lock_guard<std::mutex> g(mu_);
    drain_freed_locked();
    char* ptr = static_cast<char*>(t.data_ptr());
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)), "hipMemGetAddressRange");
    if (size > kMaxExportSegment) {
      // the tensor sits in a huge caching-allocator segment (e.g. a freed multi-GB logits
      // block reused for a gradient): opening such a segment's IPC handle in the peer blocked
      // indefinitely on this driver (3.5 GB hung, 1 GB worked: tools/ipc_size_probe.py), so
      // the bytes go out through a pooled, separately allocated staging buffer instead --
      // one D2D copy on the producer's stream, before the message's readiness event
      const int64_t nb = static_cast<int64_t>(t.numel() * t.element_size());
      const int si = acquire_staging_locked(static_cast<size_t>(nb));
      Staging& st = staging_[si];
      hip_check(static_cast<hipError_t>(
                    smpk::device_copy(st.ptr, ptr, nb, at::hip::getCurrentHIPStream(device_).stream())),
                "device_copy (staging)");
      staging_pending_.push_back(si);
      stats_staged_++;
      stats_exports_++;
      stats_bytes_out_ += nb;
      b_out = static_cast<int64_t>(reinterpret_cast<uintptr_t>(st.ptr));
      gen_out = st.gen;
      handle = st.handle;
      offset_out = 0;
      nbytes_out = nb;
      return;
    }
    uintptr_t b = reinterpret_cast<uintptr_t>(base);
    auto it = exports_.find(b);
    if (it == exports_.end() || it->second.size != size) {
      SegmentExport se;
      se.size = size;
      se.gen = ++gen_counter_;
      hip_check(hipIpcGetMemHandle(&se.handle, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
      exports_[b] = se;
      it = exports_.find(b);
      stats_exports_new_++;
    }
    offset_out = static_cast<int64_t>(reinterpret_cast<uintptr_t>(ptr) - b);
    nbytes_out = static_cast<int64_t>(t.numel() * t.element_size());
    stats_exports_++;
    stats_bytes_out_ += nbytes_out;
    b_out = static_cast<int64_t>(b);
    gen_out = it->second.gen;
    handle = it->second.handle;
  }

  // Sender side: record the readiness event of one control message on the current stream.
  // -> (slot, gate context for gate_fn)
  py::tuple record_event() {
    std::lock_guard<std::mutex> g(mu_);
    int slot = acquire_event_locked();
    // the staging buffers of this message are free again once its receiver releases the slot
    staging_by_slot_[slot].swap(staging_pending_);
    staging_pending_.clear();
    hip_check(hipEventRecord(events_[slot].ev, at::hip::getCurrentHIPStream(device_).stream()), "hipEventRecord");
    return py::make_tuple(slot, static_cast<uint64_t>(reinterpret_cast<uintptr_t>(events_[slot].ev)));
  }

  // hipEventQuery predicate for the mailbox's gated sends: 1 done, 0 pending, -1 error.
  static int event_gate(uintptr_t ctx) {
    const hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(ctx));
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return -1;
  }
  static uint64_t gate_fn() { return static_cast<uint64_t>(reinterpret_cast<uintptr_t>(&IpcP2P::event_gate)); }

  // Sender side: the peer's copy out of `slot` completed (release message).
  void release_event(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(slot >= 0 && slot < static_cast<int>(events_.size()), "IpcP2P.release_event: bad slot");
    if (events_[slot].busy) {
      events_[slot].busy = false;
      free_slots_.push_back(slot);
    }
    auto sb = staging_by_slot_.find(slot);
    if (sb != staging_by_slot_.end()) {
      for (int si : sb->second) staging_free_.push_back(si);
      staging_by_slot_.erase(sb);
    }
  }

  // Receiver side: enqueue one D2D pull of nbytes into dst on the current stream.  The
  // message that carried the handle was gated on the producer's completion, so the bytes
  // are final.
  void import_copy(at::Tensor dst, int src, int64_t base, int64_t gen, py::bytes mem_handle, int64_t offset,
                   int64_t nbytes) {
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "IpcP2P.import: dst must be a contiguous GPU tensor");
    TORCH_CHECK(dst.numel() * dst.element_size() == nbytes, "IpcP2P.import: size mismatch (dst ",
                dst.numel() * dst.element_size(), " B, message ", nbytes, " B)");
    std::string mh = mem_handle;
    TORCH_CHECK(mh.size() == sizeof(hipIpcMemHandle_t), "IpcP2P.import: malformed handle");
    py::gil_scoped_release nogil;  // HIP calls below: no GIL held while they run
    std::lock_guard<std::mutex> g(mu_);
    // ---- mapping of the sender's segment
    auto key = std::make_pair(src, base);
    auto it = imports_.find(key);
    if (it != imports_.end() && it->second.gen != gen) {
      hipIpcCloseMemHandle(it->second.ptr);
      imports_.erase(it);
      it = imports_.end();
    }
    if (it == imports_.end()) {
      if (imports_.size() >= kMaxImports) evict_lru_locked();
      hipIpcMemHandle_t h;
      std::memcpy(&h, mh.data(), sizeof(h));
      void* p = nullptr;
      hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      bool remote = false;
      hipPointerAttribute_t attr;
      if (hipPointerGetAttributes(&attr, p) == hipSuccess) remote = attr.device >= 0 && attr.device != device_;
      (void)hipGetLastError();
      imports_[key] = Mapping{gen, p, 0, remote};
      it = imports_.find(key);
      stats_maps_++;
    }
    it->second.last_use = ++use_clock_;
    hipStream_t s = at::hip::getCurrentHIPStream(device_).stream();
    if (nbytes > 0) {
      const char* srcp = static_cast<char*>(it->second.ptr) + offset;
      const bool sdma = engine_ == kEngineSdma || (engine_ == kEngineAuto && it->second.remote);
      if (sdma) {
        hip_check(hipMemcpyAsync(dst.data_ptr(), srcp, static_cast<size_t>(nbytes), hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync (pull)");
        stats_pulls_sdma_++;
      } else {
        // same GPU: a copy kernel on the pull stream, not hipMemcpyAsync -- with four processes
        // time-sharing one GPU, >= 100 MB hipMemcpyAsync pulls blocked the host thread
        // indefinitely (PP=4 micro-batch 16 rehearsal, tools/gpu_pp_hang.sh)
        hip_check(static_cast<hipError_t>(smpk::device_copy(dst.data_ptr(), srcp, nbytes, s)), "device_copy");
        stats_pulls_kernel_++;
      }
    }
    stats_imports_++;
    stats_bytes_in_ += nbytes;
  }

  // test hook: a small cap makes every pull of a new segment evict (tests/workers/pp_gpu.py)
  void set_max_imports(int64_t n) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(n >= 1, "IpcP2P.set_max_imports: need >= 1");
    kMaxImports = static_cast<size_t>(n);
  }

  void close() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : imports_) hipIpcCloseMemHandle(kv.second.ptr);
    imports_.clear();
    for (auto& e : events_) hipEventDestroy(e.ev);
    events_.clear();
    free_slots_.clear();
    exports_.clear();
    if (!staging_.empty()) {
      hipDeviceSynchronize();  // a staging copy may still be queued
      for (auto& st : staging_) hipFree(st.ptr);
    }
    staging_.clear();
    staging_free_.clear();
    staging_pending_.clear();
    staging_by_slot_.clear();
  }

  py::dict stats() {
    py::dict d;
    // never blocks: the watchdog reads this while the main thread may be stuck inside a HIP
    // call that holds mu_ (that itself is the diagnostic)
    std::unique_lock<std::mutex> g(mu_, std::try_to_lock);
    if (!g.owns_lock()) {
      d["locked_by_hip_call"] = true;
      return d;
    }
    d["exports"] = stats_exports_;
    d["segment_exports"] = stats_exports_new_;
    d["imports"] = stats_imports_;
    d["mappings"] = stats_maps_;
    d["mappings_open"] = static_cast<int64_t>(imports_.size());
    d["mappings_evicted"] = stats_evicted_;
    d["staged_exports"] = stats_staged_;
    d["pull_engine"] = engine_ == kEngineSdma ? "sdma" : engine_ == kEngineKernel ? "kernel" : "auto";
    d["pulls_sdma"] = stats_pulls_sdma_;
    d["pulls_kernel"] = stats_pulls_kernel_;
    int64_t remote_maps = 0;
    for (auto& kv : imports_) remote_maps += kv.second.remote ? 1 : 0;
    d["mappings_remote_gpu"] = remote_maps;
    d["staging_buffers"] = static_cast<int64_t>(staging_.size());
    d["bytes_out"] = stats_bytes_out_;
    d["bytes_in"] = stats_bytes_in_;
    d["event_slots"] = static_cast<int64_t>(events_.size());
    int64_t busy = 0;
    for (auto& e : events_) busy += e.busy ? 1 : 0;
    d["event_slots_busy"] = busy;
    return d;
  }

 private:
  struct LocalEvent {
    hipEvent_t ev;
    bool busy;
  };
  struct Mapping {
    int64_t gen;
    void* ptr;
    uint64_t last_use;
    bool remote;  // the segment lives on another GPU (pull over xGMI)
  };
  static constexpr int kEngineAuto = 0, kEngineKernel = 1, kEngineSdma = 2;
  static int engine_from_env() {
    const char* e = getenv("SMP_P2P_PULL_ENGINE");
    if (e == nullptr) return kEngineAuto;
    if (strcmp(e, "kernel") == 0) return kEngineKernel;
    if (strcmp(e, "sdma") == 0) return kEngineSdma;
    return kEngineAuto;
  }
  int engine_ = engine_from_env();

  // largest caching-allocator segment exported in place
  static constexpr size_t kMaxExportSegment = size_t(1) << 30;
  struct Staging {
    void* ptr;
    size_t cap;
    int64_t gen;
    hipIpcMemHandle_t handle;
  };
  // best-fitting free staging buffer, or a new one (2 MB-rounded hipMalloc: its own segment,
  // exported once -- receivers keep the mapping across steps)
  int acquire_staging_locked(size_t nbytes) {
    int best = -1;
    for (size_t i = 0; i < staging_free_.size(); ++i) {
      const int si = staging_free_[i];
      if (staging_[si].cap >= nbytes && (best < 0 || staging_[si].cap < staging_[staging_free_[best]].cap))
        best = static_cast<int>(i);
    }
    if (best >= 0) {
      const int si = staging_free_[best];
      staging_free_.erase(staging_free_.begin() + best);
      return si;
    }
    Staging st;
    st.cap = (nbytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipMalloc(&st.ptr, st.cap), "hipMalloc (IPC staging)");
    hip_check(hipIpcGetMemHandle(&st.handle, st.ptr), "hipIpcGetMemHandle (IPC staging)");
    st.gen = ++gen_counter_;
    staging_.push_back(st);
    return static_cast<int>(staging_.size()) - 1;
  }
  std::vector<Staging> staging_;
  std::vector<int> staging_free_, staging_pending_;
  std::map<int, std::vector<int>> staging_by_slot_;

  // A receiver never learns that a sender freed a segment (only a new generation at the same
  // base replaces a mapping), so under allocator churn mappings of dead segments -- and the
  // sender memory they pin -- would accumulate.  The import table is bounded: past
  // kMaxImports mappings the least recently used one is closed, after the pull stream has
  // drained (a pending copy may still read it; eviction is rare, so the sync is cheap).
  static constexpr size_t kMaxImportsDefault = 256;
  size_t kMaxImports = kMaxImportsDefault;
  void evict_lru_locked() {
    auto lru = imports_.begin();
    for (auto i = imports_.begin(); i != imports_.end(); ++i)
      if (i->second.last_use < lru->second.last_use) lru = i;
    if (lru == imports_.end()) return;
    hip_check(hipStreamSynchronize(at::hip::getCurrentHIPStream(device_).stream()), "hipStreamSynchronize");
    hipIpcCloseMemHandle(lru->second.ptr);
    imports_.erase(lru);
    stats_evicted_++;
  }

  int acquire_event_locked() {
    if (free_slots_.empty()) {
      LocalEvent e;
      hip_check(hipSetDevice(device_), "hipSetDevice");
      hip_check(hipEventCreateWithFlags(&e.ev, hipEventDisableTiming), "hipEventCreateWithFlags");
      e.busy = false;
      events_.push_back(e);
      free_slots_.push_back(static_cast<int>(events_.size()) - 1);
    }
    int slot = free_slots_.back();
    free_slots_.pop_back();
    events_[slot].busy = true;
    return slot;
  }

  void drain_freed_locked() {
    std::vector<uintptr_t> freed;
    {
      std::lock_guard<std::mutex> g(g_freed_mu);
      freed.swap(g_freed);
    }
    for (uintptr_t b : freed) exports_.erase(b);
  }

  int device_;
  std::mutex mu_;
  std::unordered_map<uintptr_t, SegmentExport> exports_;
  int64_t gen_counter_ = 0;
  std::vector<LocalEvent> events_;
  std::vector<int> free_slots_;
  std::map<std::pair<int, int64_t>, Mapping> imports_;
  uint64_t use_clock_ = 0;
  int64_t stats_exports_ = 0, stats_exports_new_ = 0, stats_imports_ = 0, stats_maps_ = 0, stats_evicted_ = 0;
  int64_t stats_staged_ = 0, stats_pulls_sdma_ = 0, stats_pulls_kernel_ = 0;
  int64_t stats_bytes_out_ = 0, stats_bytes_in_ = 0;
};

void register_ipc_p2p(py::module& m) {
  py::class_<IpcP2P>(m, "IpcP2P")
      .def(py::init<int>(), py::arg("device"))
      .def("export_tensor", &IpcP2P::export_tensor)
      .def("record_event", &IpcP2P::record_event)
      .def_static("gate_fn", &IpcP2P::gate_fn)
      .def("import_copy", &IpcP2P::import_copy, py::arg("dst"), py::arg("src"), py::arg("base"), py::arg("gen"),
           py::arg("mem_handle"), py::arg("offset"), py::arg("nbytes"))
      .def("release_event", &IpcP2P::release_event)
      .def("set_max_imports", &IpcP2P::set_max_imports)
      .def("close", &IpcP2P::close)
      .def("stats", &IpcP2P::stats);
}

// Page-locks the storage of an ordinary CPU tensor in place (hipHostRegister): exact-size
// pinned host memory for large optimizer-state arrays -- the caching pinned allocator rounds
// every block up to a power of two, which at hundreds of GB costs tens of GB of host RAM.
void host_register(const at::Tensor& t) {
  TORCH_CHECK(t.device().is_cpu() && t.is_contiguous(), "host_register: a contiguous CPU tensor is required");
  const size_t bytes = static_cast<size_t>(t.numel()) * t.element_size();
  if (bytes == 0) return;
  hip_check(hipHostRegister(t.data_ptr(), bytes, hipHostRegisterDefault), "hipHostRegister");
}

void host_unregister_ptr(uint64_t ptr) {
  if (ptr != 0) (void)hipHostUnregister(reinterpret_cast<void*>(static_cast<uintptr_t>(ptr)));
}

void register_grad_tracker(py::module& m);
void register_ipc_allreduce(py::module& m);

void register_bindings(py::module& m) {
  m.def("host_register", &host_register);
  m.def("host_unregister_ptr", &host_unregister_ptr);
  register_grad_tracker(m);
  register_ipc_p2p(m);
  register_ipc_allreduce(m);
}

}  // namespace smprt_torch
