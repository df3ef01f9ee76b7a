#include "grad_counter.h"

#include <stdexcept>

namespace smprt {

GradCounter::GradCounter(const std::vector<std::string>& names, int num_microbatches)
    : names_(names),
      expected_(names.size(), 0),
      seen_(names.size(), 0),
      reported_(names.size(), 0),
      fwd_done_(num_microbatches, 0),
      num_mb_(num_microbatches) {
  for (size_t i = 0; i < names.size(); ++i) idx_[names[i]] = static_cast<int>(i);
}

int GradCounter::index(const std::string& name) {
  auto it = idx_.find(name);
  if (it == idx_.end()) throw std::out_of_range("GradCounter: unknown parameter " + name);
  return it->second;
}

bool GradCounter::final_locked(int i) const {
  return fwd_done_count_ == num_mb_ && seen_[i] >= expected_[i] && expected_[i] > 0;
}

void GradCounter::increment_expected_num_grads(int /*mb*/, const std::vector<std::string>& names) {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& n : names) expected_[index(n)]++;
}

bool GradCounter::mark_grad_computed(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  int i = index(name);
  seen_[i]++;
  if (!reported_[i] && final_locked(i)) {
    reported_[i] = 1;
    return true;
  }
  return false;
}

std::vector<std::string> GradCounter::mark_fwd_pass_done(int mb) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  if (mb < 0 || mb >= num_mb_) throw std::out_of_range("GradCounter: bad microbatch");
  if (!fwd_done_[mb]) {
    fwd_done_[mb] = 1;
    fwd_done_count_++;
  }
  if (fwd_done_count_ == num_mb_) {
    for (size_t i = 0; i < names_.size(); ++i) {
      if (!reported_[i] && final_locked(static_cast<int>(i))) {
        reported_[i] = 1;
        out.push_back(names_[i]);
      }
    }
  }
  return out;
}

bool GradCounter::is_grad_ready(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  return final_locked(index(name));
}

bool GradCounter::all_forwards_done() {
  std::lock_guard<std::mutex> g(mu_);
  return fwd_done_count_ == num_mb_;
}

int64_t GradCounter::get_param_grad_count(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  return expected_[index(name)];
}

int64_t GradCounter::get_seen_grad_count(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  return seen_[index(name)];
}

void GradCounter::clear_minibatch_state() {
  std::lock_guard<std::mutex> g(mu_);
  std::fill(expected_.begin(), expected_.end(), 0);
  std::fill(seen_.begin(), seen_.end(), 0);
  std::fill(reported_.begin(), reported_.end(), 0);
  std::fill(fwd_done_.begin(), fwd_done_.end(), 0);
  fwd_done_count_ = 0;
  current_mb_ = 0;
}

}  // namespace smprt
