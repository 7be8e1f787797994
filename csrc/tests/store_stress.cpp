// Host-side stress driver for the native TCP store (csrc/store_core.h), built by
// tests/test_store_sanitize_cpu.py with AddressSanitizer + UndefinedBehaviorSanitizer and, separately, with
// ThreadSanitizer: the server's acceptor / per-connection threads, the condition-variable GET waits, ADD
// counters, barriers, timeouts and shutdown with blocked waiters all run concurrently from many client threads.
//   store_stress <clients> <rounds>      exit 0 on success, 1 on a wrong result
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../store_core.h"

using pdt_store::StoreClient;

int main(int argc, char** argv) {
  const int nclients = argc > 1 ? std::atoi(argv[1]) : 8;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 50;
  std::atomic<int> errors{0};
  auto fail = [&](const char* what) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    errors.fetch_add(1);
  };
  {
    auto server = std::make_unique<StoreClient>("127.0.0.1", 0, true, 30.0);
    const int port = server->port();
    std::vector<std::thread> ts;
    for (int r = 0; r < nclients; ++r) {
      ts.emplace_back([&, r] {
        try {
          StoreClient c("127.0.0.1", port, false, 30.0);
          for (int i = 0; i < rounds; ++i) {
            const std::string k = "k/" + std::to_string(r) + "/" + std::to_string(i);
            c.set(k, std::string(1 + (i * 37 + r) % 300, (char)('a' + r % 26)));
            // read a key another client produces (blocking GET until it exists)
            const int peer = (r + 1) % nclients;
            const std::string pk = "k/" + std::to_string(peer) + "/" + std::to_string(i);
            const std::string v = c.get(pk, -1.0);
            if (v.size() != (size_t)(1 + (i * 37 + peer) % 300) || v[0] != (char)('a' + peer % 26)) fail("get value");
            c.add("counter", 1);
            if (!c.check(k)) fail("check");
            c.barrier("round/" + std::to_string(i), nclients);
            if (c.add("counter", 0) < (int64_t)(i + 1) * nclients) fail("barrier before all adds");
          }
          c.del("k/" + std::to_string(r) + "/0");
          if (c.check("k/" + std::to_string(r) + "/0")) fail("del");
          bool timed_out = false;
          try {
            c.get("never-set/" + std::to_string(r), 0.05);
          } catch (const std::exception&) {
            timed_out = true;
          }
          if (!timed_out) fail("timeout");
        } catch (const std::exception& e) {
          std::fprintf(stderr, "client %d: %s\n", r, e.what());
          errors.fetch_add(1);
        }
      });
    }
    for (auto& t : ts) t.join();
    if (server->add("counter", 0) != (int64_t)nclients * rounds) fail("final counter");
    // shutdown with a client blocked in GET: the server must release it (error), never hang or crash
    std::thread blocked([&] {
      try {
        StoreClient c("127.0.0.1", port, false, 30.0);
        c.get("blocks-forever", 20.0);
      } catch (const std::exception&) {
      }
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    server.reset();  // server teardown releases the blocked waiter
    blocked.join();
  }
  std::printf("store_stress: %d clients x %d rounds, %d errors\n", nclients, rounds, errors.load());
  return errors.load() == 0 ? 0 : 1;
}
