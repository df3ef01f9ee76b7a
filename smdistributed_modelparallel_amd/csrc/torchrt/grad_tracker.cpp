// GradTracker: when is a parameter's gradient final for the step? (N1g)
//
// Reference semantics (smp/torch/patches/execution.py:131-162,165-258 with
// allreduce/reducer.py:92 and server.py:410,455): every time a backward *segment* is
// registered (the tensors whose gradients will later arrive from another pipeline stage,
// or the loss on stage 0), the parameters reachable from those tensors through the
// autograd graph each expect one more gradient accumulation.  A parameter is final once
// every microbatch has finished its forward pass (the expected count can no longer grow)
// and the accumulations seen match the expected count.
//
// Our design: the graph walk runs here in C++ over torch::autograd::Node edges (a GPT-2 XL
// stage has thousands of nodes per segment -- a Python walk over grad_fn.next_functions
// would cost milliseconds per microbatch), parameters are addressed by dense indices, and
// walks can be memoised per segment signature by the caller (add_expected()).
#include <ATen/ATen.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/accumulate_grad.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/extension.h>

#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace smprt_torch {

class GradTracker {
 public:
  GradTracker(const std::vector<at::Tensor>& params, int num_mb) {
    for (size_t i = 0; i < params.size(); ++i) index_[params[i].unsafeGetTensorImpl()] = static_cast<int64_t>(i);
    expected_.assign(params.size(), 0);
    seen_.assign(params.size(), 0);
    reported_.assign(params.size(), 0);
    reset(num_mb);
  }

  void reset(int num_mb) {
    std::fill(expected_.begin(), expected_.end(), 0);
    std::fill(seen_.begin(), seen_.end(), 0);
    std::fill(reported_.begin(), reported_.end(), 0);
    num_mb_ = num_mb;
    fwd_done_.assign(num_mb, 0);
    fwd_done_count_ = 0;
  }

  // Walk the autograd graph from `roots`; every registered parameter reached (through its
  // AccumulateGrad node, or as a root leaf) expects one more gradient.  Returns the
  // parameter indices found (sorted, unique) so the caller can memoise the segment.
  std::vector<int64_t> add_segment(const std::vector<at::Tensor>& roots) {
    std::vector<int64_t> found = reachable(roots);
    add_expected(found);
    return found;
  }

  std::vector<int64_t> reachable(const std::vector<at::Tensor>& roots) const {
    using torch::autograd::AccumulateGrad;
    using torch::autograd::Node;
    std::unordered_set<const Node*> seen;
    std::vector<Node*> stack;
    std::unordered_set<int64_t> hit;
    for (const auto& r : roots) {
      if (!r.defined() || !r.requires_grad()) continue;
      const auto& fn = r.grad_fn();
      if (!fn) {
        auto it = index_.find(r.unsafeGetTensorImpl());
        if (it != index_.end()) hit.insert(it->second);
        continue;
      }
      if (seen.insert(fn.get()).second) stack.push_back(fn.get());
    }
    while (!stack.empty()) {
      Node* n = stack.back();
      stack.pop_back();
      if (auto* acc = dynamic_cast<AccumulateGrad*>(n)) {
        auto it = index_.find(acc->variable.unsafeGetTensorImpl());
        if (it != index_.end()) hit.insert(it->second);
        continue;
      }
      for (const auto& e : n->next_edges()) {
        if (e.function && seen.insert(e.function.get()).second) stack.push_back(e.function.get());
      }
    }
    std::vector<int64_t> out(hit.begin(), hit.end());
    std::sort(out.begin(), out.end());
    return out;
  }

  void add_expected(const std::vector<int64_t>& idx) {
    for (int64_t i : idx) {
      TORCH_CHECK(i >= 0 && i < static_cast<int64_t>(expected_.size()), "GradTracker: bad index");
      expected_[i]++;
    }
  }

  // One gradient accumulation into parameter i.  True when that made it final.
  bool mark_grad(int64_t i) {
    TORCH_CHECK(i >= 0 && i < static_cast<int64_t>(seen_.size()), "GradTracker: bad index");
    seen_[i]++;
    if (!reported_[i] && final_(i)) {
      reported_[i] = 1;
      return true;
    }
    return false;
  }

  // Microbatch `mb` finished its forward on this stage.  Returns parameters that became
  // final because the last forward just completed.
  std::vector<int64_t> mark_fwd_done(int mb) {
    std::vector<int64_t> out;
    TORCH_CHECK(mb >= 0 && mb < num_mb_, "GradTracker: bad microbatch ", mb);
    if (!fwd_done_[mb]) {
      fwd_done_[mb] = 1;
      fwd_done_count_++;
      if (fwd_done_count_ == num_mb_) {
        for (size_t i = 0; i < expected_.size(); ++i) {
          if (!reported_[i] && final_(static_cast<int64_t>(i))) {
            reported_[i] = 1;
            out.push_back(static_cast<int64_t>(i));
          }
        }
      }
    }
    return out;
  }

  bool is_final(int64_t i) const { return final_(i); }
  bool all_forwards_done() const { return fwd_done_count_ == num_mb_; }
  int64_t expected(int64_t i) const { return expected_.at(i); }
  int64_t seen(int64_t i) const { return seen_.at(i); }
  int64_t num_params() const { return static_cast<int64_t>(expected_.size()); }

 private:
  bool final_(int64_t i) const {
    return fwd_done_count_ == num_mb_ && expected_[i] > 0 && seen_[i] >= expected_[i];
  }

  std::unordered_map<const c10::TensorImpl*, int64_t> index_;
  std::vector<int64_t> expected_, seen_;
  std::vector<char> reported_, fwd_done_;
  int num_mb_ = 1;
  int fwd_done_count_ = 0;
};

// Graph validation (reference `patches/execution.py:57-72`): for every target tensor, does
// the autograd graph of `roots` reach it?  A target with a grad_fn (a RemoteOutput result)
// is matched by that node, a leaf target (an input leaf of a remote request) by its
// AccumulateGrad node or by being a root itself.  `bridges[i]` continue the walk once
// target i is hit: a RemoteOutput's graph goes on, through the remote stage, at the
// tensors that were sent in that call.  The walk stops once every target is hit.
std::vector<bool> graph_reaches(const std::vector<at::Tensor>& roots, const std::vector<at::Tensor>& targets,
                                const std::vector<std::vector<at::Tensor>>& bridges) {
  using torch::autograd::Node;
  std::unordered_map<const Node*, std::vector<size_t>> by_node;
  std::unordered_map<const c10::TensorImpl*, std::vector<size_t>> by_leaf;
  std::vector<bool> hit(targets.size(), false);
  size_t remaining = 0;
  for (size_t i = 0; i < targets.size(); ++i) {
    const auto& t = targets[i];
    if (!t.defined() || !t.requires_grad()) continue;
    ++remaining;
    by_leaf[t.unsafeGetTensorImpl()].push_back(i);
    if (const auto& fn = t.grad_fn()) {
      by_node[fn.get()].push_back(i);
    } else if (auto acc = torch::autograd::impl::try_get_grad_accumulator(t)) {
      by_node[acc.get()].push_back(i);
    }
  }
  std::unordered_set<const Node*> seen;
  std::vector<Node*> stack;
  std::vector<const at::Tensor*> pending;
  auto mark = [&](const std::vector<size_t>& idx) {
    for (size_t i : idx)
      if (!hit[i]) {
        hit[i] = true;
        --remaining;
        if (i < bridges.size())
          for (const auto& b : bridges[i]) pending.push_back(&b);
      }
  };
  auto push_root = [&](const at::Tensor& r) {
    if (!r.defined() || !r.requires_grad()) return;
    auto lt = by_leaf.find(r.unsafeGetTensorImpl());
    if (lt != by_leaf.end()) mark(lt->second);
    const auto& fn = r.grad_fn();
    if (fn && seen.insert(fn.get()).second) stack.push_back(fn.get());
  };
  for (const auto& r : roots) push_root(r);
  while (remaining > 0 && (!stack.empty() || !pending.empty())) {
    while (!pending.empty()) {
      const at::Tensor* t = pending.back();
      pending.pop_back();
      push_root(*t);
    }
    if (stack.empty()) continue;
    Node* n = stack.back();
    stack.pop_back();
    auto it = by_node.find(n);
    if (it != by_node.end()) mark(it->second);
    for (const auto& e : n->next_edges()) {
      if (e.function && seen.insert(e.function.get()).second) stack.push_back(e.function.get());
    }
  }
  return hit;
}

void register_grad_tracker(py::module& m) {
  m.def("graph_reaches", &graph_reaches, py::arg("roots"), py::arg("targets"),
        py::arg("bridges") = std::vector<std::vector<at::Tensor>>());
  py::class_<GradTracker>(m, "GradTracker")
      .def(py::init<const std::vector<at::Tensor>&, int>(), py::arg("params"), py::arg("num_microbatches"))
      .def("reset", &GradTracker::reset)
      .def("add_segment", &GradTracker::add_segment)
      .def("reachable", &GradTracker::reachable)
      .def("add_expected", &GradTracker::add_expected)
      .def("mark_grad", &GradTracker::mark_grad)
      .def("mark_fwd_done", &GradTracker::mark_fwd_done)
      .def("is_final", &GradTracker::is_final)
      .def("all_forwards_done", &GradTracker::all_forwards_done)
      .def("expected", &GradTracker::expected)
      .def("seen", &GradTracker::seen)
      .def_property_readonly("num_params", &GradTracker::num_params);
}

}  // namespace smprt_torch
