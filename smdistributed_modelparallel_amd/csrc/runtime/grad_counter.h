// Per-parameter gradient arrival accounting across microbatches (N1g, SURVEY §2.1;
// reference call sites smp/torch/model.py:401-403, patches/execution.py:156,220,
// allreduce/reducer.py:92, server.py:410,455, worker.py:406-417, state_mod.py:317).
//
// A parameter's gradient is *final* for the step once the forward passes of all
// microbatches have finished (so the expected count can no longer grow) and the number
// of accumulations seen equals the number of uses recorded during forward.  The reducer
// launches a bucket's all-reduce exactly when every parameter in it becomes final.
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace smprt {

class GradCounter {
 public:
  GradCounter(const std::vector<std::string>& names, int num_microbatches);

  void increment_expected_num_grads(int mb, const std::vector<std::string>& names);
  // Returns true when this call made the parameter's gradient final.
  bool mark_grad_computed(const std::string& name);
  // Returns the names whose gradients became final because forward finished.
  std::vector<std::string> mark_fwd_pass_done(int mb);
  bool is_grad_ready(const std::string& name);
  bool all_forwards_done();
  int64_t get_param_grad_count(const std::string& name);
  int64_t get_seen_grad_count(const std::string& name);
  void set_microbatch(int mb) { current_mb_ = mb; }
  int microbatch() const { return current_mb_; }
  void clear_minibatch_state();
  int num_params() const { return static_cast<int>(names_.size()); }

 private:
  int index(const std::string& name);
  bool final_locked(int i) const;

  std::vector<std::string> names_;
  std::unordered_map<std::string, int> idx_;
  std::vector<int64_t> expected_, seen_;
  std::vector<char> reported_;
  std::vector<char> fwd_done_;
  int num_mb_;
  int fwd_done_count_ = 0;
  int current_mb_ = 0;
  std::mutex mu_;
};

}  // namespace smprt
