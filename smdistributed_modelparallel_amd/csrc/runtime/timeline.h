// Pipeline timeline tracer (N1h; reference call sites
// smp/backend/core.py:290,524-536, smp/torch/server.py:366-478, step.py:254,269).
//
// Records per-step, per-microbatch pipeline events and writes Chrome-trace JSON
// (chrome://tracing / Perfetto).  When SMP_ROCTX=1 and libroctx64 is loadable, every
// event is also emitted as a roctx range so it shows up in rocprofv3 marker traces.
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace smprt {

class Timeline {
 public:
  explicit Timeline(int rank);
  ~Timeline();
  void set_output(const std::string& path);
  bool enabled() const { return !path_.empty(); }
  bool roctx_enabled() const { return roctx_push_ != nullptr; }
  void start_step(int64_t step);
  void end_step();
  // Instant-with-duration event: [begin, end) of a pipeline task on microbatch `mb`.
  void record(int mb, const std::string& label, double begin_us, double end_us);
  // Mark: zero-duration event at now.
  void mark(int mb, const std::string& label);
  void range_push(const std::string& label);
  void range_pop();
  double now_us() const;
  void flush();

 private:
  struct Event {
    std::string name;
    int mb;
    double ts, dur;
    int64_t step;
  };
  int rank_;
  std::string path_;
  int64_t step_ = -1;
  double step_begin_ = 0;
  std::vector<Event> events_;
  std::mutex mu_;
  void* roctx_ = nullptr;
  int (*roctx_push_)(const char*) = nullptr;
  int (*roctx_pop_)() = nullptr;
};

}  // namespace smprt
