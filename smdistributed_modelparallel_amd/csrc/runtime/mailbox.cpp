#include "mailbox.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace smprt {

namespace {

constexpr uint32_t kMagic = 0x534d5031;  // "SMP1"

#pragma pack(push, 1)
struct FrameHeader {
  uint32_t magic;
  int32_t src;
  int64_t tid;
  uint64_t len;
  uint8_t channel;
  uint8_t pad[7];
};
#pragma pack(pop)
static_assert(sizeof(FrameHeader) == 32, "frame header layout");

void write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("mailbox send failed: ") + strerror(errno));
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
}

// Returns false on EOF before any byte was read -- an orderly close, or a reset (a peer that
// exits with unread bytes in its receive queue sends RST instead of FIN): both are "the peer
// left", and the caller tells a shutdown from a death by the goodbye it did or did not send.
bool read_all(int fd, char* p, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::recv(fd, p + got, n - got, 0);
    if (r == 0) {
      if (got == 0) return false;
      throw std::runtime_error("mailbox peer closed mid-frame");
    }
    if (r < 0) {
      if (errno == EINTR) continue;
      if (errno == ECONNRESET && got == 0) return false;
      throw std::runtime_error(std::string("mailbox recv failed: ") + strerror(errno));
    }
    got += static_cast<size_t>(r);
  }
  return true;
}

void tune_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

Mailbox::Mailbox(int rank, int world) : rank_(rank), world_(world) {
  peers_.resize(world);
  for (int i = 0; i < world; ++i) peers_[i] = std::make_unique<Peer>();
  goodbye_.assign(world, 0);
}

Mailbox::~Mailbox() {
  try {
    shutdown();
  } catch (...) {
  }
}

int Mailbox::listen(const std::string& host) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("mailbox: socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = 0;
  if (host.empty() || host == "0.0.0.0") {
    addr.sin_addr.s_addr = INADDR_ANY;
  } else if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    addr.sin_addr.s_addr = INADDR_ANY;
  }
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
    throw std::runtime_error(std::string("mailbox: bind failed: ") + strerror(errno));
  if (::listen(listen_fd_, world_ + 8) != 0) throw std::runtime_error("mailbox: listen failed");
  socklen_t len = sizeof(addr);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  return ntohs(addr.sin_port);
}

void Mailbox::connect(const std::vector<std::string>& hosts, const std::vector<int>& ports,
                      double timeout_s) {
  const double deadline = now_s() + timeout_s;
  // Lower ranks accept, higher ranks dial.  Dial first to all lower ranks.
  for (int peer = 0; peer < rank_; ++peer) {
    int fd = -1;
    while (true) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      std::string port = std::to_string(ports[peer]);
      if (getaddrinfo(hosts[peer].c_str(), port.c_str(), &hints, &res) == 0 && res) {
        fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
          freeaddrinfo(res);
          break;
        }
        ::close(fd);
        fd = -1;
        freeaddrinfo(res);
      }
      if (now_s() > deadline) throw std::runtime_error("mailbox: connect timeout");
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    tune_socket(fd);
    int32_t me = rank_;
    write_all(fd, reinterpret_cast<const char*>(&me), sizeof(me));
    peers_[peer]->fd = fd;
  }
  for (int n = rank_ + 1; n < world_; ++n) {
    pollfd pfd{listen_fd_, POLLIN, 0};
    int rem_ms = static_cast<int>((deadline - now_s()) * 1000);
    if (rem_ms <= 0 || ::poll(&pfd, 1, rem_ms) <= 0) throw std::runtime_error("mailbox: accept timeout");
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) throw std::runtime_error("mailbox: accept failed");
    tune_socket(fd);
    int32_t who = -1;
    if (!read_all(fd, reinterpret_cast<char*>(&who), sizeof(who)) || who <= rank_ || who >= world_)
      throw std::runtime_error("mailbox: bad handshake");
    peers_[who]->fd = fd;
  }
  ::close(listen_fd_);
  listen_fd_ = -1;
  // The wake pipe exists before any thread that reads or writes it starts.
  if (::pipe(wake_pipe_) != 0) throw std::runtime_error("mailbox: pipe() failed");
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    peers_[p]->sender = std::thread(&Mailbox::send_loop, this, p);
  }
  receiver_ = std::thread(&Mailbox::recv_loop, this);
}

std::shared_ptr<const std::string> Mailbox::frame(int64_t tid, uint8_t channel, const std::string& p) {
  FrameHeader h{};
  h.magic = kMagic;
  h.src = rank_;
  h.tid = tid;
  h.len = p.size();
  h.channel = channel;
  auto buf = std::make_shared<std::string>();
  buf->reserve(sizeof(h) + p.size());
  buf->append(reinterpret_cast<const char*>(&h), sizeof(h));
  buf->append(p);
  return buf;
}

void Mailbox::send(int dst, int64_t tid, uint8_t channel, std::string payload) {
  if (dst < 0 || dst >= world_) throw std::runtime_error("mailbox: bad destination rank");
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.msgs_sent++;
    stats_.bytes_sent += payload.size();
  }
  if (dst == rank_) {
    Message m;
    m.src = rank_;
    m.tid = tid;
    m.channel = channel;
    m.payload = std::move(payload);
    deliver(std::move(m));
    return;
  }
  auto f = frame(tid, channel, payload);
  Peer& p = *peers_[dst];
  {
    std::lock_guard<std::mutex> g(p.mu);
    p.outq.push_back(OutMsg{std::move(f), nullptr, 0});
  }
  p.cv.notify_all();
}

void Mailbox::send_gated(int dst, int64_t tid, uint8_t channel, std::string payload, GateFn gate, uintptr_t ctx) {
  if (gate == nullptr || dst == rank_) {
    // a message to self is consumed by this process after everything it enqueued so far:
    // wait for the gate here (it only covers this process's own device work)
    if (gate != nullptr) {
      while (gate(ctx) == 0) std::this_thread::yield();
    }
    send(dst, tid, channel, std::move(payload));
    return;
  }
  if (dst < 0 || dst >= world_) throw std::runtime_error("mailbox: bad destination rank");
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.msgs_sent++;
    stats_.bytes_sent += payload.size();
  }
  auto f = frame(tid, channel, payload);
  Peer& p = *peers_[dst];
  {
    std::lock_guard<std::mutex> g(p.mu);
    p.outq.push_back(OutMsg{std::move(f), gate, ctx});
  }
  p.cv.notify_all();
}

void Mailbox::broadcast(const std::vector<int>& dsts, int64_t tid, uint8_t channel,
                        const std::string& payload) {
  std::shared_ptr<const std::string> f;
  for (int d : dsts) {
    if (d == rank_) {
      send(d, tid, channel, payload);
      continue;
    }
    if (!f) f = frame(tid, channel, payload);
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.msgs_sent++;
      stats_.bytes_sent += payload.size();
    }
    Peer& p = *peers_[d];
    {
      std::lock_guard<std::mutex> g(p.mu);
      p.outq.push_back(OutMsg{f, nullptr, 0});
    }
    p.cv.notify_all();
  }
}

void Mailbox::send_loop(int peer) {
  Peer& p = *peers_[peer];
  while (true) {
    OutMsg m;
    {
      std::unique_lock<std::mutex> lk(p.mu);
      p.cv.wait(lk, [&] { return stop_.load() || !p.outq.empty(); });
      if (p.outq.empty()) return;  // stop requested and drained
      m = std::move(p.outq.front());
      p.outq.pop_front();
      p.writing = true;
    }
    if (m.gate != nullptr) {
      // wait (outside every lock) until the device work this message describes is done;
      // later messages to this peer stay queued behind it (per-destination FIFO)
      const auto t0 = std::chrono::steady_clock::now();
      int r;
      int spins = 0;
      while ((r = m.gate(m.ctx)) == 0) {
        if (stop_.load() && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) break;
        if (++spins < 64) {
          std::this_thread::yield();
        } else {
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
      }
      const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0);
      {
        std::lock_guard<std::mutex> g(stats_mu_);
        stats_.gated_sent++;
        stats_.gate_wait_us += static_cast<uint64_t>(us.count());
      }
      if (r <= 0) {
        // the gate failed (r < 0), or shutdown gave up waiting for it (r == 0): the receiver could
        // pull bytes the producer's kernels have not finished writing, so the message is
        // dropped and the failure recorded instead of sending an ungated handle
        {
          std::lock_guard<std::mutex> g(in_mu_);
          if (error_.empty())
            error_ = std::string("mailbox: readiness gate of a message to rank ") + std::to_string(peer) +
                     (r < 0 ? " failed" : " still pending at shutdown (message dropped)");
          in_cv_.notify_all();
        }
        std::lock_guard<std::mutex> g(p.mu);
        p.writing = false;
        p.cv.notify_all();
        continue;
      }
    }
    const std::shared_ptr<const std::string>& f = m.frame;
    try {
      write_all(p.fd, f->data(), f->size());
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(in_mu_);
      if (error_.empty()) error_ = e.what();
      in_cv_.notify_all();
    }
    {
      std::lock_guard<std::mutex> g(p.mu);
      p.writing = false;
    }
    p.cv.notify_all();
  }
}

void Mailbox::recv_loop() {
  std::vector<pollfd> fds;
  std::vector<int> owner;
  for (int p = 0; p < world_; ++p) {
    if (p == rank_ || peers_[p]->fd < 0) continue;
    fds.push_back(pollfd{peers_[p]->fd, POLLIN, 0});
    owner.push_back(p);
  }
  fds.push_back(pollfd{wake_pipe_[0], POLLIN, 0});
  owner.push_back(-1);
  std::vector<bool> closed(fds.size(), false);
  while (!stop_.load()) {
    int n = ::poll(fds.data(), fds.size(), 200);
    if (n <= 0) continue;
    for (size_t i = 0; i < fds.size(); ++i) {
      if (closed[i] || !(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      if (owner[i] < 0) return;  // woken for shutdown
      FrameHeader h{};
      try {
        if (!read_all(fds[i].fd, reinterpret_cast<char*>(&h), sizeof(h))) {
          closed[i] = true;
          fds[i].fd = -1;
          bool orderly;
          {
            std::lock_guard<std::mutex> g(in_mu_);
            orderly = goodbye_[owner[i]] != 0;
          }
          if (!orderly && !stop_.load())
            record_failure(owner[i], "rank " + std::to_string(owner[i]) +
                                         " closed its connection without shutdown (process died?)");
          continue;
        }
        if (h.magic != kMagic) throw std::runtime_error("mailbox: corrupt frame");
        if (h.channel == CONTROL) {
          if (h.tid == ABORT) {
            record_failure(h.src, "rank " + std::to_string(h.src) + " aborted (shutdown with failure)");
          } else {
            std::lock_guard<std::mutex> g(in_mu_);
            goodbye_[h.src] = 1;
          }
          continue;
        }
        Message m;
        m.src = h.src;
        m.tid = h.tid;
        m.channel = h.channel;
        m.payload.resize(h.len);
        if (h.len) read_all(fds[i].fd, &m.payload[0], h.len);
        deliver(std::move(m));
      } catch (const std::exception& e) {
        if (stop_.load()) return;
        closed[i] = true;
        fds[i].fd = -1;
        record_failure(owner[i], e.what());
      }
    }
  }
}

void Mailbox::record_failure(int rank, const std::string& what) {
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (error_.empty()) {
      error_ = what;
      failed_rank_ = rank;
    }
  }
  in_cv_.notify_all();
}

std::string Mailbox::error() {
  std::lock_guard<std::mutex> g(in_mu_);
  return error_;
}

int Mailbox::failed_rank() {
  std::lock_guard<std::mutex> g(in_mu_);
  return failed_rank_;
}

std::string Mailbox::wait_error(double timeout_s) {
  std::unique_lock<std::mutex> lk(in_mu_);
  auto ready = [&] { return !error_.empty() || stop_.load(); };
  if (timeout_s < 0)
    in_cv_.wait(lk, ready);
  else
    in_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready);
  return error_;
}

void Mailbox::deliver(Message&& m) {
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.msgs_recv++;
    stats_.bytes_recv += m.payload.size();
  }
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (m.channel == SERVER) {
      server_q_.push_back(std::move(m));
    } else {
      matched_[{m.src, m.tid}].push_back(std::move(m.payload));
    }
  }
  in_cv_.notify_all();
}

std::string Mailbox::recv(int src, int64_t tid, double timeout_s) {
  std::unique_lock<std::mutex> lk(in_mu_);
  auto key = std::make_pair(src, tid);
  auto ready = [&] {
    auto it = matched_.find(key);
    return (it != matched_.end() && !it->second.empty()) || stop_.load() || !error_.empty();
  };
  if (timeout_s < 0) {
    in_cv_.wait(lk, ready);
  } else if (!in_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready)) {
    throw std::runtime_error("mailbox: recv timeout from rank " + std::to_string(src) +
                             " tid " + std::to_string(tid));
  }
  auto it = matched_.find(key);
  if (it == matched_.end() || it->second.empty()) {
    throw std::runtime_error("mailbox: " + (error_.empty() ? std::string("shut down") : error_));
  }
  std::string out = std::move(it->second.front());
  it->second.pop_front();
  if (it->second.empty()) matched_.erase(it);
  return out;
}

bool Mailbox::poll(int src, int64_t tid) {
  std::lock_guard<std::mutex> g(in_mu_);
  auto it = matched_.find({src, tid});
  return it != matched_.end() && !it->second.empty();
}

bool Mailbox::has_server_message() {
  std::lock_guard<std::mutex> g(in_mu_);
  return !server_q_.empty();
}

bool Mailbox::next_server_message(Message* out, double timeout_s) {
  std::unique_lock<std::mutex> lk(in_mu_);
  auto ready = [&] { return !server_q_.empty() || stop_.load() || !error_.empty(); };
  if (timeout_s < 0) {
    in_cv_.wait(lk, ready);
  } else if (!in_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready)) {
    return false;
  }
  if (server_q_.empty()) {
    if (!error_.empty()) throw std::runtime_error("mailbox: " + error_);
    return false;
  }
  *out = std::move(server_q_.front());
  server_q_.pop_front();
  return true;
}

void Mailbox::flush() {
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    Peer& peer = *peers_[p];
    std::unique_lock<std::mutex> lk(peer.mu);
    peer.cv.wait(lk, [&] { return (peer.outq.empty() && !peer.writing) || stop_.load(); });
  }
}

void Mailbox::shutdown(bool success) {
  if (stop_.load()) return;
  // Tell every connected peer how this rank ends; senders drain their queues (this
  // frame included) before they exit below.
  if (listen_fd_ < 0) {
    auto f = frame(success ? GOODBYE : ABORT, CONTROL, std::string());
    for (int d = 0; d < world_; ++d) {
      if (d == rank_ || peers_[d]->fd < 0) continue;
      Peer& p = *peers_[d];
      {
        std::lock_guard<std::mutex> g(p.mu);
        p.outq.push_back(OutMsg{f, nullptr, 0});
      }
      p.cv.notify_all();
    }
  }
  if (stop_.exchange(true)) return;
  for (auto& p : peers_) {
    {
      std::lock_guard<std::mutex> g(p->mu);
    }
    p->cv.notify_all();
  }
  for (auto& p : peers_)
    if (p->sender.joinable()) p->sender.join();
  if (wake_pipe_[1] >= 0) {
    char c = 1;
    (void)!::write(wake_pipe_[1], &c, 1);
  }
  if (receiver_.joinable()) receiver_.join();
  for (auto& p : peers_) {
    if (p->fd >= 0) ::close(p->fd);
    p->fd = -1;
  }
  for (int i = 0; i < 2; ++i)
    if (wake_pipe_[i] >= 0) ::close(wake_pipe_[i]);
  if (listen_fd_ >= 0) ::close(listen_fd_);
  in_cv_.notify_all();
}

TransportStats Mailbox::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

}  // namespace smprt
