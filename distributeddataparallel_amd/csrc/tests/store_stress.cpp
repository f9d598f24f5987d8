// Host-only stress test of the native stores, built with -fsanitize=address,undefined (and
// separately -fsanitize=thread) by tests/test_sanitizers_cpu.py (sanitizer
// builds of the C++ host code on CPU). Many client threads hammer one TCPStore server with
// set/get/add/compare_set/wait/append/delete, a FileStore is shared by two handles, and
// blocking waits race with late writers and timeouts.
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "store/tcp_store.h"

namespace xddp {
std::shared_ptr<Store> make_file_store(const std::string& path, int world_size);
}

using namespace xddp;

#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                    \
    }                                                                  \
  } while (0)

int main() {
  using namespace std::chrono;
  TCPStore server("127.0.0.1", 0, true, 1, milliseconds(20000), false);
  const int port = server.port();
  constexpr int kThreads = 8, kIters = 200;
  std::vector<std::thread> ts;
  std::atomic<int> errors{0};
  for (int t = 0; t < kThreads; ++t) {
    ts.emplace_back([&, t] {
      try {
        TCPStore c("127.0.0.1", port, false, 1, milliseconds(20000), false);
        for (int i = 0; i < kIters; ++i) {
          const std::string k = "k" + std::to_string(t) + "_" + std::to_string(i);
          c.set(k, std::string(static_cast<size_t>(i % 97), 'x'));
          CHECK(c.get(k).size() == static_cast<size_t>(i % 97));
          c.add("counter", 1);
          c.append("log" + std::to_string(t), "a");
          c.compare_set("cas", "", "init");
          if (i % 50 == 0) CHECK(c.delete_key(k));
        }
        c.set("done" + std::to_string(t), "1");
        // wait for everybody (server-side waiters)
        std::vector<std::string> keys;
        for (int u = 0; u < kThreads; ++u) keys.push_back("done" + std::to_string(u));
        c.wait(keys, milliseconds(20000));
      } catch (const std::exception& e) {
        std::fprintf(stderr, "thread %d: %s\n", t, e.what());
        errors++;
      }
    });
  }
  for (auto& th : ts) th.join();
  CHECK(errors == 0);
  CHECK(server.add("counter", 0) == kThreads * kIters);
  CHECK(server.get("log3").size() == static_cast<size_t>(kIters));
  // timeout path
  {
    TCPStore c("127.0.0.1", port, false, 1, milliseconds(200), false);
    bool timed_out = false;
    try {
      c.get("never");
    } catch (const StoreTimeout&) {
      timed_out = true;
    }
    CHECK(timed_out);
  }
  // late writer races a blocking get
  {
    TCPStore c("127.0.0.1", port, false, 1, milliseconds(5000), false);
    std::thread w([&] {
      std::this_thread::sleep_for(milliseconds(50));
      server.set("late", "v");
    });
    CHECK(c.get("late") == "v");
    w.join();
  }
  // file store shared by two handles with concurrent adders
  {
    char tmpl[] = "/tmp/xddp_fs_stressXXXXXX";
    int fd = mkstemp(tmpl);
    CHECK(fd >= 0);
    close(fd);
    unlink(tmpl);
    auto a = make_file_store(tmpl, 2);
    auto b = make_file_store(tmpl, 2);
    std::thread ta([&] { for (int i = 0; i < 200; ++i) a->add("n", 1); });
    std::thread tb([&] { for (int i = 0; i < 200; ++i) b->add("n", 1); });
    ta.join();
    tb.join();
    CHECK(a->add("n", 0) == 400);
    b->set("k", "v");
    CHECK(a->get("k") == "v");
  }
  std::printf("store_stress OK\n");
  return 0;
}
