// Core of the native TCP rendezvous store (csrc/store.cpp): wire protocol, server and a synchronous client,
// free of Python so the host-side sanitizer tests (tests/test_store_sanitize_cpu.py: ASan + UBSan, TSan) build
// it on its own.  See csrc/store.cpp for the protocol description.
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>


namespace pdt_store {

enum Op : uint8_t { kSet = 1, kGet = 2, kAdd = 3, kCheck = 4, kDel = 5 };
enum Status : uint8_t { kOk = 0, kTimeout = 1, kMissing = 2 };

static void send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      throw std::runtime_error("tcp store: connection lost while sending");
    }
    c += k;
    n -= (size_t)k;
  }
}

static bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

static void send_bytes(int fd, const std::string& s) {
  const uint64_t n = s.size();
  send_all(fd, &n, 8);
  if (n) send_all(fd, s.data(), n);
}

static bool recv_bytes(int fd, std::string& s) {
  uint64_t n = 0;
  if (!recv_all(fd, &n, 8)) return false;
  if (n > (1ull << 32)) return false;
  s.resize(n);
  return n == 0 || recv_all(fd, &s[0], n);
}

// ------------------------------------------------------------------------------------------------
class Server {
 public:
  explicit Server(int port) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ < 0) throw std::runtime_error("tcp store: socket() failed");
    int one = 1;
    ::setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = htons((uint16_t)port);
    if (::bind(fd_, (sockaddr*)&a, sizeof(a)) != 0) {
      ::close(fd_);
      throw std::runtime_error("tcp store: cannot bind port " + std::to_string(port) + ": " + std::strerror(errno));
    }
    if (::listen(fd_, 1024) != 0) {
      ::close(fd_);
      throw std::runtime_error("tcp store: listen() failed");
    }
    socklen_t len = sizeof(a);
    ::getsockname(fd_, (sockaddr*)&a, &len);
    port_ = ntohs(a.sin_port);
    acceptor_ = std::thread([this] { accept_loop(); });
  }
  ~Server() { stop(); }

  int port() const { return port_; }

  // Teardown lingers (bounded) until every client connection is gone: a client's last request -- e.g. the final
  // SET of a barrier, whose waiters (this process among them) may return and exit before that SET is acknowledged
  // -- must be answered before the sockets are shut down.
  void stop(int64_t linger_ms = 10000) {
    if (stopping_.load()) return;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(linger_ms),
                     [&] { return clients_.empty(); });
    }
    if (stopping_.exchange(true)) return;
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c : clients_) ::shutdown(c, SHUT_RDWR);
      cv_.notify_all();
    }
    if (acceptor_.joinable()) acceptor_.join();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
  }

 private:
  void accept_loop() {
    while (!stopping_) {
      pollfd p{fd_, POLLIN, 0};
      if (::poll(&p, 1, 200) <= 0) continue;
      const int c = ::accept(fd_, nullptr, nullptr);
      if (c < 0) continue;
      int one = 1;
      ::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> g(mu_);
      clients_.push_back(c);
      workers_.emplace_back([this, c] { serve(c); });
    }
  }

  void serve(int c) {
    for (;;) {
      uint8_t op = 0;
      if (!recv_all(c, &op, 1)) break;
      std::string key, val;
      if (!recv_bytes(c, key)) break;
      try {
        if (op == kSet) {
          if (!recv_bytes(c, val)) break;
          {
            std::lock_guard<std::mutex> g(mu_);
            kv_[key] = std::move(val);
          }
          const uint8_t st = kOk;  // acknowledge before waking the waiters (they may tear the server down)
          send_all(c, &st, 1);
          cv_.notify_all();
        } else if (op == kGet) {
          int64_t timeout_ms = 0;
          if (!recv_all(c, &timeout_ms, 8)) break;
          std::unique_lock<std::mutex> g(mu_);
          // wait_until on the system clock (pthread_cond_timedwait): the steady-clock wait_for compiles to
          // pthread_cond_clockwait, which this toolchain's ThreadSanitizer does not intercept (it then reports
          // a false "double lock" in the host sanitizer test)
          const bool ok = cv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms),
                                         [&] { return stopping_ || kv_.count(key) > 0; });
          if (ok && kv_.count(key)) {
            const std::string v = kv_[key];
            g.unlock();
            const uint8_t st = kOk;
            send_all(c, &st, 1);
            send_bytes(c, v);
          } else {
            g.unlock();
            const uint8_t st = kTimeout;
            send_all(c, &st, 1);
          }
        } else if (op == kAdd) {
          int64_t delta = 0;
          if (!recv_all(c, &delta, 8)) break;
          int64_t nv = 0;
          {
            std::lock_guard<std::mutex> g(mu_);
            std::string& s = kv_[key];
            int64_t cur = 0;
            if (s.size() == 8) std::memcpy(&cur, s.data(), 8);
            nv = cur + delta;
            s.assign(reinterpret_cast<const char*>(&nv), 8);
          }
          cv_.notify_all();
          const uint8_t st = kOk;
          send_all(c, &st, 1);
          send_all(c, &nv, 8);
        } else if (op == kCheck) {
          uint8_t st;
          {
            std::lock_guard<std::mutex> g(mu_);
            st = kv_.count(key) ? kOk : kMissing;
          }
          send_all(c, &st, 1);
        } else if (op == kDel) {
          {
            std::lock_guard<std::mutex> g(mu_);
            kv_.erase(key);
          }
          const uint8_t st = kOk;
          send_all(c, &st, 1);
        } else {
          break;
        }
      } catch (const std::exception&) {
        break;
      }
    }
    {  // forget the fd BEFORE closing it: stop() must never shut down a reused descriptor number
      std::lock_guard<std::mutex> g(mu_);
      for (auto it = clients_.begin(); it != clients_.end(); ++it)
        if (*it == c) {
          clients_.erase(it);
          break;
        }
    }
    cv_.notify_all();  // a lingering stop() waits for the last client to leave
    ::close(c);
  }

  int fd_ = -1, port_ = 0;
  std::atomic<bool> stopping_{false};
  std::thread acceptor_;
  std::vector<std::thread> workers_;
  std::vector<int> clients_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
};

// ------------------------------------------------------------------------------------------------
// Synchronous client (one socket, requests serialised by a mutex); ``is_server`` also runs the server here.
class StoreClient {
 public:
  StoreClient(const std::string& host, int port, bool is_server, double timeout_s)
      : timeout_ms_((int64_t)(timeout_s * 1000.0)) {
    if (is_server) {
      server_ = std::make_unique<Server>(port);
      port = server_->port();
    }
    port_ = port;
    connect_to(is_server ? std::string("127.0.0.1") : host, port);
  }
  ~StoreClient() {
    if (fd_ >= 0) ::close(fd_);
    if (server_) server_->stop();
  }
  StoreClient(const StoreClient&) = delete;
  StoreClient& operator=(const StoreClient&) = delete;

  int port() const { return port_; }

  void set(const std::string& key, const std::string& v) {
    std::lock_guard<std::mutex> g(mu_);
    request(kSet, key);
    send_bytes(fd_, v);
    expect_ok("set", key);
  }

  // timeout_s < 0: the client's default timeout
  std::string get(const std::string& key, double timeout_s) {
    std::string v;
    std::lock_guard<std::mutex> g(mu_);
    request(kGet, key);
    const int64_t t = timeout_s >= 0 ? (int64_t)(timeout_s * 1000.0) : timeout_ms_;
    send_all(fd_, &t, 8);
    uint8_t st = 0;
    if (!recv_all(fd_, &st, 1)) throw std::runtime_error("tcp store: server closed the connection");
    if (st != kOk) throw std::runtime_error("tcp store: timed out waiting for key '" + key + "'");
    if (!recv_bytes(fd_, v)) throw std::runtime_error("tcp store: server closed the connection");
    return v;
  }

  int64_t add(const std::string& key, int64_t delta) {
    std::lock_guard<std::mutex> g(mu_);
    request(kAdd, key);
    send_all(fd_, &delta, 8);
    expect_ok("add", key);
    int64_t nv = 0;
    if (!recv_all(fd_, &nv, 8)) throw std::runtime_error("tcp store: server closed the connection");
    return nv;
  }

  bool check(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    request(kCheck, key);
    uint8_t st = 0;
    if (!recv_all(fd_, &st, 1)) throw std::runtime_error("tcp store: server closed the connection");
    return st == kOk;
  }

  void del(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    request(kDel, key);
    expect_ok("del", key);
  }

  // all `world` participants arrive; the last one releases everybody
  void barrier(const std::string& tag, int world) {
    const int64_t n = add(tag + "/arrive", 1);
    if (n == world) {  // the last arriver releases everybody and is itself released
      set(tag + "/done", "1");
      return;
    }
    (void)get(tag + "/done", -1.0);
  }

 private:
  void connect_to(const std::string& host, int port) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
      throw std::runtime_error("tcp store: cannot resolve " + host);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    for (;;) {
      fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(fd_, res->ai_addr, res->ai_addrlen) == 0) break;
      ::close(fd_);
      fd_ = -1;
      if (std::chrono::steady_clock::now() > deadline) {
        ::freeaddrinfo(res);
        throw std::runtime_error("tcp store: cannot connect to " + host + ":" + std::to_string(port));
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));  // server not up yet (rendezvous race)
    }
    ::freeaddrinfo(res);
    int one = 1;
    ::setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  void request(Op op, const std::string& key) {
    const uint8_t o = op;
    send_all(fd_, &o, 1);
    send_bytes(fd_, key);
  }
  void expect_ok(const char* what, const std::string& key) {
    uint8_t st = 0;
    if (!recv_all(fd_, &st, 1) || st != kOk)
      throw std::runtime_error(std::string("tcp store: ") + what + " failed for key '" + key + "'");
  }

  int fd_ = -1, port_ = 0;
  int64_t timeout_ms_;
  std::mutex mu_;
  std::unique_ptr<Server> server_;
};

}  // namespace pdt_store
