// Native self-test of the control-plane mailbox (reference native self-tests
// test/backend/d2d_test.py, p2p_rdma_test.py -- SURVEY §2.1 N1k, §4 "Backend / native").
//
// Runs a 4-rank full mesh inside one process (one thread per rank, loopback TCP) and
// checks: matched send/recv with transaction ids, FIFO order per (src, tid), server-
// channel routing, broadcast, stats, and the coordinated-shutdown protocol (an ABORT from
// one rank makes every other rank's blocked receive throw; GOODBYE shutdowns stay quiet).
// Built and run by tests/test_native_cpu.py under ThreadSanitizer and AddressSanitizer.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "mailbox.h"

using smprt::Mailbox;

#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::abort();                                                          \
    }                                                                        \
  } while (0)

static std::vector<std::unique_ptr<Mailbox>> make_mesh(int world) {
  std::vector<std::unique_ptr<Mailbox>> boxes;
  std::vector<std::string> hosts(world, "127.0.0.1");
  std::vector<int> ports(world);
  for (int r = 0; r < world; ++r) {
    boxes.emplace_back(new Mailbox(r, world));
    ports[r] = boxes[r]->listen("127.0.0.1");
  }
  std::vector<std::thread> ts;
  for (int r = 0; r < world; ++r) ts.emplace_back([&, r] { boxes[r]->connect(hosts, ports, 30.0); });
  for (auto& t : ts) t.join();
  return boxes;
}

static void test_messaging() {
  const int W = 4, N = 200;
  auto boxes = make_mesh(W);
  std::vector<std::thread> ts;
  for (int r = 0; r < W; ++r) {
    ts.emplace_back([&, r] {
      Mailbox& mb = *boxes[r];
      // every rank sends N ordered messages to every other rank on tid 7, plus one to itself
      for (int d = 0; d < W; ++d)
        for (int i = 0; i < N; ++i) mb.send(d, 7, smprt::USER, std::to_string(r) + ":" + std::to_string(i));
      for (int s = 0; s < W; ++s)
        for (int i = 0; i < N; ++i) {
          std::string got = mb.recv(s, 7, 30.0);
          CHECK(got == std::to_string(s) + ":" + std::to_string(i));
        }
      // broadcast on a distinct tid; large payload exercises partial socket writes
      std::string big(3 << 20, static_cast<char>('a' + r));
      std::vector<int> dsts;
      for (int d = 0; d < W; ++d) dsts.push_back(d);
      mb.broadcast(dsts, 11, smprt::USER, big);
      for (int s = 0; s < W; ++s) {
        std::string got = mb.recv(s, 11, 30.0);
        CHECK(got.size() == big.size() && got[0] == 'a' + s && got.back() == 'a' + s);
      }
      // server channel: unsolicited messages, FIFO per source
      int dst = (r + 1) % W;
      for (int i = 0; i < 5; ++i) mb.send(dst, 100 + i, smprt::SERVER, "srv" + std::to_string(i));
      int seen = 0;
      int last = -1;
      while (seen < 5) {
        smprt::Message m;
        CHECK(mb.next_server_message(&m, 30.0));
        CHECK(m.src == (r + W - 1) % W);
        CHECK(static_cast<int>(m.tid) == last + 101);
        last = static_cast<int>(m.tid) - 100;
        ++seen;
      }
      CHECK(!mb.poll((r + 1) % W, 12345));
      mb.flush();
    });
  }
  for (auto& t : ts) t.join();
  for (int r = 0; r < W; ++r) {
    auto st = boxes[r]->stats();
    CHECK(st.msgs_recv >= static_cast<uint64_t>(W * N + W + 5));
    CHECK(boxes[r]->error().empty());
  }
  // orderly shutdown: nobody records a failure
  for (int r = 0; r < W; ++r) boxes[r]->shutdown(true);
  for (int r = 0; r < W; ++r) CHECK(boxes[r]->error().empty());
  std::printf("messaging ok\n");
}

static void test_abort_propagates() {
  const int W = 4;
  auto boxes = make_mesh(W);
  std::atomic<int> raised{0};
  std::vector<std::thread> ts;
  for (int r = 0; r < W - 1; ++r) {
    ts.emplace_back([&, r] {
      try {
        boxes[r]->recv(W - 1, 42, -1.0);  // would wait forever without the ABORT
      } catch (const std::runtime_error& e) {
        std::string what = e.what();
        CHECK(what.find("aborted") != std::string::npos);
        raised++;
      }
      CHECK(boxes[r]->failed_rank() == W - 1);
      CHECK(!boxes[r]->wait_error(0.0).empty());
    });
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  boxes[W - 1]->shutdown(false);
  for (auto& t : ts) t.join();
  CHECK(raised.load() == W - 1);
  for (int r = 0; r < W - 1; ++r) boxes[r]->shutdown(false);
  std::printf("abort propagation ok\n");
}

static void test_wait_error_timeout() {
  auto boxes = make_mesh(2);
  CHECK(boxes[0]->wait_error(0.05).empty());
  bool threw = false;
  try {
    boxes[0]->recv(1, 5, 0.05);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
  for (auto& b : boxes) b->shutdown(true);
  std::printf("timeouts ok\n");
}

// Gated sends (the pipeline transport's "message leaves once the producer kernels are done"):
// a gated message and every later message to the SAME peer wait for the gate; other peers
// are not held up; FIFO order per peer is kept.
static std::atomic<int> g_gate{0};
static int test_gate(uintptr_t ctx) { return g_gate.load() >= static_cast<int>(ctx) ? 1 : 0; }

static void test_gated_send() {
  auto boxes = make_mesh(3);
  g_gate.store(0);
  boxes[0]->send_gated(1, 0, smprt::SERVER, "gated-a", &test_gate, 1);
  boxes[0]->send(1, 0, smprt::SERVER, "plain-after-a");  // queued behind the gate (FIFO)
  boxes[0]->send(2, 0, smprt::SERVER, "other-peer");     // a different peer is not held up
  smprt::Message m;
  CHECK(boxes[2]->next_server_message(&m, 10.0) && m.payload == "other-peer");
  CHECK(!boxes[1]->next_server_message(&m, 0.2));  // still gated
  g_gate.store(1);
  CHECK(boxes[1]->next_server_message(&m, 10.0) && m.payload == "gated-a");
  CHECK(boxes[1]->next_server_message(&m, 10.0) && m.payload == "plain-after-a");
  // a self-addressed gated message waits in place and is delivered
  g_gate.store(2);
  boxes[0]->send_gated(0, 0, smprt::SERVER, "self", &test_gate, 2);
  CHECK(boxes[0]->next_server_message(&m, 10.0) && m.payload == "self");
  auto st = boxes[0]->stats();
  CHECK(st.gated_sent == 1);
  for (auto& b : boxes) b->shutdown(true);
  std::printf("gated sends ok\n");
}

int main() {
  test_messaging();
  test_abort_propagates();
  test_wait_error_timeout();
  test_gated_send();
  std::printf("ALL OK\n");
  return 0;
}
