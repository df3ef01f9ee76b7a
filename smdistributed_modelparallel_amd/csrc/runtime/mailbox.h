// Control-plane transport of the runtime: a full-mesh TCP mailbox.
//
// Replaces the reference's MPI object channel + listener thread (N1b/N1d in SURVEY §2.1;
// call sites smp/backend/collectives.py:237-324 and smp/torch/server_comm.py:60-348).
//
// Every message carries (src, transaction id, channel). Channel USER messages are
// matched by (src, tid) against explicit receives; channel SERVER messages are
// unsolicited and go to a FIFO the pipeline server drains (the reference's
// "server=True" routing).  One receiver thread multiplexes all peer sockets with
// poll(2); one sender thread per peer drains an outgoing queue so a Python send never
// blocks the caller on a slow peer (async send semantics of smp_async_send).
//
// Coordinated shutdown (reference smp_shutdown(success), smp/backend/core.py:227-259):
// shutdown() sends every peer a CONTROL frame -- GOODBYE on success, ABORT on failure --
// before closing.  A peer that receives ABORT, or sees a connection close without a
// GOODBYE (the process died), records the failure: every blocked or later receive then
// throws instead of waiting forever, and wait_error() wakes the watchdog thread.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

namespace smprt {

enum Channel : uint8_t { USER = 0, SERVER = 1, CONTROL = 2 };
enum ControlTid : int64_t { GOODBYE = 0, ABORT = 1 };

struct Message {
  int32_t src = -1;
  int64_t tid = 0;
  uint8_t channel = USER;
  std::string payload;
};

struct TransportStats {
  uint64_t msgs_sent = 0, msgs_recv = 0, bytes_sent = 0, bytes_recv = 0;
  uint64_t gated_sent = 0;      // messages that waited for a readiness gate
  uint64_t gate_wait_us = 0;    // total time the peer sender threads spent on gates
};

// Readiness gate of a gated send: returns 1 when the message may go out, 0 while it must
// wait, < 0 on error (the message then goes out anyway and the error is recorded).  Called
// from the destination's sender thread, never under a lock.  The pipeline transport passes
// a HIP event query here (`csrc/torchrt/ipc_p2p.cpp`): a control message describing device
// tensors leaves only once the kernels that produced them have completed, so the receiver
// can pull the bytes without any device-side cross-process wait.
using GateFn = int (*)(uintptr_t ctx);

class Mailbox {
 public:
  Mailbox(int rank, int world);
  ~Mailbox();

  // Bind a listening socket on `host` (port chosen by the kernel); returns the port.
  int listen(const std::string& host);
  // Connect the full mesh. `hosts`/`ports` are indexed by rank.
  void connect(const std::vector<std::string>& hosts, const std::vector<int>& ports,
               double timeout_s);

  void send(int dst, int64_t tid, uint8_t channel, std::string payload);
  // FIFO per destination like send(): this message and every later one to `dst` wait until
  // gate(ctx) reports ready.
  void send_gated(int dst, int64_t tid, uint8_t channel, std::string payload, GateFn gate, uintptr_t ctx);
  // Multi-destination send of one payload (smp_async_bcast).
  void broadcast(const std::vector<int>& dsts, int64_t tid, uint8_t channel,
                 const std::string& payload);

  // Matched receive. timeout_s < 0 waits forever. Throws on timeout/shutdown.
  std::string recv(int src, int64_t tid, double timeout_s);
  bool poll(int src, int64_t tid);

  // Unsolicited (server channel) messages.
  bool has_server_message();
  // Returns false on timeout.
  bool next_server_message(Message* out, double timeout_s);

  // Wait until every queued outgoing message has been written to its socket.
  void flush();
  // success=false tells every peer that this rank failed (ABORT).
  void shutdown(bool success = true);
  // First recorded transport failure ("" if none).
  std::string error();
  // Rank that aborted or vanished (-1 if none / unknown).
  int failed_rank();
  // Block until a failure is recorded or the mailbox stops; returns error() ("" on
  // timeout or orderly stop).  timeout_s < 0 waits forever.
  std::string wait_error(double timeout_s);
  TransportStats stats();
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  struct OutMsg {
    std::shared_ptr<const std::string> frame;
    GateFn gate = nullptr;
    uintptr_t ctx = 0;
  };
  struct Peer {
    int fd = -1;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<OutMsg> outq;  // framed messages (optionally gated)
    std::thread sender;
    bool writing = false;
  };

  void recv_loop();
  void send_loop(int peer);
  void deliver(Message&& m);
  void record_failure(int rank, const std::string& what);
  std::shared_ptr<const std::string> frame(int64_t tid, uint8_t channel, const std::string& p);

  int rank_, world_;
  int listen_fd_ = -1;
  std::vector<std::unique_ptr<Peer>> peers_;
  std::thread receiver_;
  std::atomic<bool> stop_{false};
  int wake_pipe_[2] = {-1, -1};

  std::mutex in_mu_;
  std::condition_variable in_cv_;
  std::map<std::pair<int, int64_t>, std::deque<std::string>> matched_;
  std::deque<Message> server_q_;
  std::string error_;
  int failed_rank_ = -1;
  std::vector<uint8_t> goodbye_;  // peer said GOODBYE (orderly close follows)

  std::mutex stats_mu_;
  TransportStats stats_;
};

}  // namespace smprt
