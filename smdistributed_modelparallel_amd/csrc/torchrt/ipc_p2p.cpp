// IpcP2P: device-to-device pipeline tensor transport over hipIpc mappings (N1c).
//
// Reference: the native D2D engine behind smp_torch_send/recv (smp/torch/ops.py:34-123,
// server_comm.py:260-302) -- CUDA IPC intra-node with an RMM receive pool.
//
// MI355X design (ours):
//  * export(t): the sender publishes the allocation that holds `t` (hipIpcGetMemHandle of
//    the caching-allocator segment, cached per segment and invalidated when the allocator
//    returns the segment to the driver) and records an inter-process event on its compute
//    stream right after the producer kernels.  Nothing is copied on the sender.
//  * import_copy(dst, ...): the receiver maps the segment once (hipIpcOpenMemHandle with
//    lazy peer enable -- over xGMI when the ranks own different GPUs, plain HBM when they
//    share one), makes its compute stream wait on the sender's event (device-side, no host
//    blocking) and pulls the bytes with one hipMemcpyAsync D2D on that stream.  The copy
//    is enqueued the moment the control message arrives, i.e. the "receive" is posted as
//    early as the data can exist; no receive pool is needed because the destination is an
//    ordinary caching-allocator tensor of the receiver.
//  * lifetime: the sender keeps the source tensor and the event slot until the receiver
//    reports (release message, Python side) that its copy has completed; event slots are
//    therefore never re-recorded while a peer may still wait on them (re-recording a slot
//    a peer has not waited on yet could create a cross-process wait cycle).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

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

  // -> (segment_base, generation, mem_handle_bytes, offset, nbytes, event_slot, event_handle_bytes)
  py::tuple export_tensor(const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda(), "IpcP2P.export: tensor must be on the GPU");
    TORCH_CHECK(t.is_contiguous(), "IpcP2P.export: tensor must be contiguous");
    std::lock_guard<std::mutex> g(mu_);
    drain_freed_locked();
    char* ptr = static_cast<char*>(t.data_ptr());
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)), "hipMemGetAddressRange");
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
    const int64_t offset = static_cast<int64_t>(reinterpret_cast<uintptr_t>(ptr) - b);
    const int64_t nbytes = static_cast<int64_t>(t.numel() * t.element_size());
    int slot = acquire_event_locked();
    hip_check(hipEventRecord(events_[slot].ev, at::hip::getCurrentHIPStream(device_).stream()), "hipEventRecord");
    stats_exports_++;
    stats_bytes_out_ += nbytes;
    return py::make_tuple(static_cast<int64_t>(b), it->second.gen,
                          py::bytes(reinterpret_cast<const char*>(&it->second.handle), sizeof(hipIpcMemHandle_t)),
                          offset, nbytes, slot,
                          py::bytes(reinterpret_cast<const char*>(&events_[slot].handle), sizeof(hipIpcEventHandle_t)));
  }

  // Sender side: the peer's copy out of `slot` completed (release message).
  void release_event(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(slot >= 0 && slot < static_cast<int>(events_.size()), "IpcP2P.release_event: bad slot");
    if (events_[slot].busy) {
      events_[slot].busy = false;
      free_slots_.push_back(slot);
    }
  }

  // Receiver side: enqueue (wait sender event) + (copy nbytes into dst) on the current stream.
  void import_copy(at::Tensor dst, int src, int64_t base, int64_t gen, py::bytes mem_handle, int64_t offset,
                   int64_t nbytes, int slot, py::bytes ev_handle) {
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "IpcP2P.import: dst must be a contiguous GPU tensor");
    TORCH_CHECK(dst.numel() * dst.element_size() == nbytes, "IpcP2P.import: size mismatch (dst ",
                dst.numel() * dst.element_size(), " B, message ", nbytes, " B)");
    std::string mh = mem_handle;
    std::string eh = ev_handle;
    TORCH_CHECK(mh.size() == sizeof(hipIpcMemHandle_t) && eh.size() == sizeof(hipIpcEventHandle_t),
                "IpcP2P.import: malformed handles");
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
      hipIpcMemHandle_t h;
      std::memcpy(&h, mh.data(), sizeof(h));
      void* p = nullptr;
      hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      imports_[key] = Mapping{gen, p};
      it = imports_.find(key);
      stats_maps_++;
    }
    // ---- the sender's event slot
    auto ek = std::make_pair(src, slot);
    auto eit = peer_events_.find(ek);
    if (eit == peer_events_.end() || eit->second.handle_bytes != eh) {
      if (eit != peer_events_.end()) hipEventDestroy(eit->second.ev);
      hipIpcEventHandle_t h;
      std::memcpy(&h, eh.data(), sizeof(h));
      hipEvent_t ev;
      hip_check(hipIpcOpenEventHandle(&ev, h), "hipIpcOpenEventHandle");
      peer_events_[ek] = PeerEvent{ev, eh};
      eit = peer_events_.find(ek);
    }
    hipStream_t s = at::hip::getCurrentHIPStream(device_).stream();
    hip_check(hipStreamWaitEvent(s, eit->second.ev, 0), "hipStreamWaitEvent");
    if (nbytes > 0) {
      hip_check(hipMemcpyAsync(dst.data_ptr(), static_cast<char*>(it->second.ptr) + offset, nbytes,
                               hipMemcpyDeviceToDevice, s),
                "hipMemcpyAsync");
    }
    stats_imports_++;
    stats_bytes_in_ += nbytes;
  }

  void close() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : imports_) hipIpcCloseMemHandle(kv.second.ptr);
    imports_.clear();
    for (auto& kv : peer_events_) hipEventDestroy(kv.second.ev);
    peer_events_.clear();
    for (auto& e : events_) hipEventDestroy(e.ev);
    events_.clear();
    free_slots_.clear();
    exports_.clear();
  }

  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    d["exports"] = stats_exports_;
    d["segment_exports"] = stats_exports_new_;
    d["imports"] = stats_imports_;
    d["mappings"] = stats_maps_;
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
    hipIpcEventHandle_t handle;
    bool busy;
  };
  struct Mapping {
    int64_t gen;
    void* ptr;
  };
  struct PeerEvent {
    hipEvent_t ev;
    std::string handle_bytes;
  };

  int acquire_event_locked() {
    if (free_slots_.empty()) {
      LocalEvent e;
      hip_check(hipSetDevice(device_), "hipSetDevice");
      hip_check(hipEventCreateWithFlags(&e.ev, hipEventInterprocess | hipEventDisableTiming),
                "hipEventCreateWithFlags(interprocess)");
      hip_check(hipIpcGetEventHandle(&e.handle, e.ev), "hipIpcGetEventHandle");
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
  std::map<std::pair<int, int>, PeerEvent> peer_events_;
  int64_t stats_exports_ = 0, stats_exports_new_ = 0, stats_imports_ = 0, stats_maps_ = 0;
  int64_t stats_bytes_out_ = 0, stats_bytes_in_ = 0;
};

void register_ipc_p2p(py::module& m) {
  py::class_<IpcP2P>(m, "IpcP2P")
      .def(py::init<int>(), py::arg("device"))
      .def("export_tensor", &IpcP2P::export_tensor)
      .def("import_copy", &IpcP2P::import_copy, py::arg("dst"), py::arg("src"), py::arg("base"), py::arg("gen"),
           py::arg("mem_handle"), py::arg("offset"), py::arg("nbytes"), py::arg("slot"), py::arg("ev_handle"))
      .def("release_event", &IpcP2P::release_event)
      .def("close", &IpcP2P::close)
      .def("stats", &IpcP2P::stats);
}

void register_grad_tracker(py::module& m);
void register_ipc_allreduce(py::module& m);

void register_bindings(py::module& m) {
  register_grad_tracker(m);
  register_ipc_p2p(m);
  register_ipc_allreduce(m);
}

}  // namespace smprt_torch
