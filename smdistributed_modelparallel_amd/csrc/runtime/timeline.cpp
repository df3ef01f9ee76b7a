#include "timeline.h"

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace smprt {

static std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

Timeline::Timeline(int rank) : rank_(rank) {
  const char* r = getenv("SMP_ROCTX");
  if (r && strcmp(r, "1") == 0) {
    roctx_ = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (roctx_) {
      roctx_push_ = reinterpret_cast<int (*)(const char*)>(dlsym(roctx_, "roctxRangePushA"));
      roctx_pop_ = reinterpret_cast<int (*)()>(dlsym(roctx_, "roctxRangePop"));
    }
  }
}

Timeline::~Timeline() { flush(); }

void Timeline::set_output(const std::string& path) { path_ = path; }

double Timeline::now_us() const {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void Timeline::start_step(int64_t step) {
  std::lock_guard<std::mutex> g(mu_);
  step_ = step;
  step_begin_ = now_us();
}

void Timeline::end_step() {
  double t = now_us();
  std::lock_guard<std::mutex> g(mu_);
  if (!path_.empty()) events_.push_back({"step " + std::to_string(step_), -1, step_begin_, t - step_begin_, step_});
}

void Timeline::record(int mb, const std::string& label, double begin_us, double end_us) {
  if (path_.empty()) return;
  std::lock_guard<std::mutex> g(mu_);
  events_.push_back({label, mb, begin_us, end_us - begin_us, step_});
}

void Timeline::mark(int mb, const std::string& label) {
  if (path_.empty()) return;
  double t = now_us();
  std::lock_guard<std::mutex> g(mu_);
  events_.push_back({label, mb, t, 0.0, step_});
}

void Timeline::range_push(const std::string& label) {
  if (roctx_push_) roctx_push_(label.c_str());
}

void Timeline::range_pop() {
  if (roctx_pop_) roctx_pop_();
}

void Timeline::flush() {
  std::lock_guard<std::mutex> g(mu_);
  if (path_.empty() || events_.empty()) return;
  FILE* f = fopen(path_.c_str(), "w");
  if (!f) return;
  fprintf(f, "{\"traceEvents\":[\n");
  for (size_t i = 0; i < events_.size(); ++i) {
    const Event& e = events_[i];
    // One Perfetto "thread" per microbatch (tid = mb + 1; step rows at tid 0).
    fprintf(f,
            "{\"name\":\"%s\",\"ph\":\"%s\",\"pid\":%d,\"tid\":%d,\"ts\":%.3f,\"dur\":%.3f,"
            "\"args\":{\"step\":%lld,\"mb\":%d}}%s\n",
            json_escape(e.name).c_str(), e.dur > 0 ? "X" : "i", rank_, e.mb + 1, e.ts, e.dur,
            static_cast<long long>(e.step), e.mb, i + 1 < events_.size() ? "," : "");
  }
  fprintf(f, "],\"displayTimeUnit\":\"ms\"}\n");
  fclose(f);
}

}  // namespace smprt
