// Native TCP KV store: one poll() server thread, length-prefixed binary protocol.
//
// Wire format (little-endian):
//   request  = u8 op | u32 nargs | nargs × (u32 len | bytes)
//   response = u8 status | u32 nparts | nparts × (u32 len | bytes)
// GET/WAIT that cannot be answered yet are parked server-side with a deadline and answered
// when a SET/ADD/CAS/APPEND makes all their keys present (or with status=TIMEOUT).
#include "store/tcp_store.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <deque>
#include <list>
#include <set>
#include <sstream>

namespace xddp {

namespace {

enum Op : uint8_t { SET = 1, GET, ADD, CAS, CHECK, WAIT, DEL, NUMKEYS, APPEND, PING };
enum Status : uint8_t { OK = 0, TIMEOUT = 1, ERR = 2 };

void put_u32(std::string& b, uint32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }

std::string encode(uint8_t head, const std::vector<std::string>& parts) {
  std::string b;
  b.push_back(static_cast<char>(head));
  put_u32(b, static_cast<uint32_t>(parts.size()));
  for (auto& p : parts) {
    put_u32(b, static_cast<uint32_t>(p.size()));
    b.append(p);
  }
  return b;
}

// Try to parse one message from buf; returns bytes consumed or 0 if incomplete.
size_t try_decode(const std::string& buf, uint8_t& head, std::vector<std::string>& parts) {
  if (buf.size() < 5) return 0;
  head = static_cast<uint8_t>(buf[0]);
  uint32_t n;
  std::memcpy(&n, buf.data() + 1, 4);
  size_t off = 5;
  parts.clear();
  for (uint32_t i = 0; i < n; ++i) {
    if (buf.size() < off + 4) return 0;
    uint32_t len;
    std::memcpy(&len, buf.data() + off, 4);
    off += 4;
    if (buf.size() < off + len) return 0;
    parts.emplace_back(buf.data() + off, len);
    off += len;
  }
  return off;
}

void write_all(int fd, const std::string& data) {
  size_t off = 0;
  while (off < data.size()) {
    ssize_t w = ::send(fd, data.data() + off, data.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd p{fd, POLLOUT, 0};
        ::poll(&p, 1, 1000);
        continue;
      }
      throw std::runtime_error(std::string("xddp store: send failed: ") + std::strerror(errno));
    }
    off += static_cast<size_t>(w);
  }
}

bool read_exact(int fd, char* dst, size_t n) {
  size_t off = 0;
  while (off < n) {
    ssize_t r = ::recv(fd, dst + off, n - off, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += static_cast<size_t>(r);
  }
  return true;
}

}  // namespace

// -------------------------------------------------------------------------------------
// Server
// -------------------------------------------------------------------------------------
class TCPStoreServer {
 public:
  explicit TCPStoreServer(int port) {
    listen_fd_ = ::socket(AF_INET6, SOCK_STREAM, 0);
    bool v6 = listen_fd_ >= 0;
    if (!v6) listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd_ < 0) throw std::runtime_error("xddp store: socket() failed");
    int one = 1;
    ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    int rc;
    if (v6) {
      int zero = 0;
      ::setsockopt(listen_fd_, IPPROTO_IPV6, IPV6_V6ONLY, &zero, sizeof(zero));
      sockaddr_in6 a{};
      a.sin6_family = AF_INET6;
      a.sin6_addr = in6addr_any;
      a.sin6_port = htons(static_cast<uint16_t>(port));
      rc = ::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a));
    } else {
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_addr.s_addr = htonl(INADDR_ANY);
      a.sin_port = htons(static_cast<uint16_t>(port));
      rc = ::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a));
    }
    if (rc != 0) {
      ::close(listen_fd_);
      throw std::runtime_error("xddp store: bind to port " + std::to_string(port) + " failed: " + std::strerror(errno));
    }
    if (::listen(listen_fd_, 1024) != 0) throw std::runtime_error("xddp store: listen failed");
    sockaddr_storage ss{};
    socklen_t sl = sizeof(ss);
    ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&ss), &sl);
    port_ = ss.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port)
                                     : ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    if (::pipe(wake_) != 0) throw std::runtime_error("xddp store: pipe failed");
    thread_ = std::thread([this] { loop(); });
  }
  ~TCPStoreServer() {
    stop_ = true;
    char c = 1;
    (void)!::write(wake_[1], &c, 1);
    if (thread_.joinable()) thread_.join();
    for (auto& kv : clients_) ::close(kv.first);
    ::close(listen_fd_);
    ::close(wake_[0]);
    ::close(wake_[1]);
  }
  int port() const { return port_; }

 private:
  struct Waiter {
    int fd;
    uint8_t op;
    std::vector<std::string> keys;
    std::chrono::steady_clock::time_point deadline;
  };

  void loop() {
    while (!stop_) {
      std::vector<pollfd> fds;
      fds.push_back({listen_fd_, POLLIN, 0});
      fds.push_back({wake_[0], POLLIN, 0});
      for (auto& kv : clients_) fds.push_back({kv.first, POLLIN, 0});
      int n = ::poll(fds.data(), fds.size(), 100);
      if (n < 0 && errno != EINTR) break;
      expire_waiters();
      if (n <= 0) continue;
      if (fds[0].revents & POLLIN) {
        int c = ::accept(listen_fd_, nullptr, nullptr);
        if (c >= 0) {
          int one = 1;
          ::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          clients_[c] = std::string();
        }
      }
      for (size_t i = 2; i < fds.size(); ++i) {
        if (!(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        int fd = fds[i].fd;
        char tmp[65536];
        ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
        if (r <= 0) {
          drop(fd);
          continue;
        }
        auto& buf = clients_[fd];
        buf.append(tmp, static_cast<size_t>(r));
        for (;;) {
          uint8_t op;
          std::vector<std::string> args;
          size_t used = try_decode(buf, op, args);
          if (!used) break;
          buf.erase(0, used);
          try {
            handle(fd, op, args);
          } catch (const std::exception& e) {
            reply(fd, ERR, {e.what()});
          }
        }
      }
    }
  }

  void drop(int fd) {
    ::close(fd);
    clients_.erase(fd);
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      if (it->fd == fd) it = waiters_.erase(it); else ++it;
    }
  }

  void reply(int fd, uint8_t st, const std::vector<std::string>& parts) {
    try {
      write_all(fd, encode(st, parts));
    } catch (...) {
    }
  }

  bool have_all(const std::vector<std::string>& keys) const {
    for (auto& k : keys)
      if (!kv_.count(k)) return false;
    return true;
  }

  void answer_waiter(const Waiter& w) {
    if (w.op == GET) reply(w.fd, OK, {kv_.at(w.keys[0])});
    else reply(w.fd, OK, {});
  }

  void on_change() {
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      if (have_all(it->keys)) {
        answer_waiter(*it);
        it = waiters_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void expire_waiters() {
    auto now = std::chrono::steady_clock::now();
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      if (now >= it->deadline) {
        reply(it->fd, TIMEOUT, {});
        it = waiters_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void handle(int fd, uint8_t op, const std::vector<std::string>& a) {
    switch (op) {
      case SET:
        kv_[a.at(0)] = a.at(1);
        reply(fd, OK, {});
        on_change();
        break;
      case GET:
      case WAIT: {
        // last arg = timeout ms
        int64_t tmo = std::stoll(a.back());
        std::vector<std::string> keys(a.begin(), a.end() - 1);
        if (have_all(keys)) {
          answer_waiter(Waiter{fd, op, keys, {}});
        } else {
          waiters_.push_back(Waiter{fd, op, keys, std::chrono::steady_clock::now() + std::chrono::milliseconds(tmo)});
        }
        break;
      }
      case ADD: {
        int64_t cur = 0;
        auto it = kv_.find(a.at(0));
        if (it != kv_.end() && !it->second.empty()) cur = std::stoll(it->second);
        cur += std::stoll(a.at(1));
        kv_[a.at(0)] = std::to_string(cur);
        reply(fd, OK, {std::to_string(cur)});
        on_change();
        break;
      }
      case CAS: {
        auto it = kv_.find(a.at(0));
        if (it == kv_.end()) {
          if (a.at(1).empty()) {
            kv_[a.at(0)] = a.at(2);
            reply(fd, OK, {a.at(2)});
            on_change();
          } else {
            reply(fd, OK, {a.at(1)});
          }
        } else if (it->second == a.at(1)) {
          it->second = a.at(2);
          reply(fd, OK, {a.at(2)});
          on_change();
        } else {
          reply(fd, OK, {it->second});
        }
        break;
      }
      case CHECK:
        reply(fd, OK, {have_all(a) ? "1" : "0"});
        break;
      case DEL:
        reply(fd, OK, {kv_.erase(a.at(0)) ? "1" : "0"});
        break;
      case NUMKEYS:
        reply(fd, OK, {std::to_string(kv_.size())});
        break;
      case APPEND:
        kv_[a.at(0)] += a.at(1);
        reply(fd, OK, {});
        on_change();
        break;
      case PING:
        reply(fd, OK, {"pong"});
        break;
      default:
        reply(fd, ERR, {"unknown op"});
    }
  }

  int listen_fd_ = -1;
  int port_ = 0;
  int wake_[2] = {-1, -1};
  std::atomic<bool> stop_{false};
  std::thread thread_;
  std::map<int, std::string> clients_;
  std::map<std::string, std::string> kv_;
  std::list<Waiter> waiters_;
};

// -------------------------------------------------------------------------------------
// Client
// -------------------------------------------------------------------------------------
static int connect_to(const std::string& host, int port, std::chrono::milliseconds timeout) {
  auto deadline = std::chrono::steady_clock::now() + timeout;
  std::string last_err = "unknown";
  while (std::chrono::steady_clock::now() < deadline) {
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    int g = ::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (g != 0) {
      last_err = gai_strerror(g);
    } else {
      for (addrinfo* r = res; r; r = r->ai_next) {
        int fd = ::socket(r->ai_family, r->ai_socktype, r->ai_protocol);
        if (fd < 0) continue;
        if (::connect(fd, r->ai_addr, r->ai_addrlen) == 0) {
          ::freeaddrinfo(res);
          int one = 1;
          ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          return fd;
        }
        last_err = std::strerror(errno);
        ::close(fd);
      }
      ::freeaddrinfo(res);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  throw StoreTimeout("xddp store: could not connect to " + host + ":" + std::to_string(port) + " (" + last_err + ")");
}

TCPStore::TCPStore(const std::string& host, int port, bool is_server, int world_size,
                   std::chrono::milliseconds tmo, bool wait_for_workers)
    : host_(host), port_(port) {
  timeout = tmo;
  if (is_server) {
    server_ = std::make_unique<TCPStoreServer>(port);
    port_ = server_->port();
  }
  fd_ = connect_to(is_server ? std::string("127.0.0.1") : host_, port_, tmo);
  if (world_size > 0) {
    add("__xddp_workers", 1);
    if (wait_for_workers && is_server) {
      auto deadline = std::chrono::steady_clock::now() + tmo;
      while (add("__xddp_workers", 0) < world_size) {
        if (std::chrono::steady_clock::now() > deadline) throw StoreTimeout("xddp store: timed out waiting for workers");
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
  }
}

TCPStore::~TCPStore() {
  if (fd_ >= 0) ::close(fd_);
  server_.reset();
}

std::vector<std::string> TCPStore::request(uint8_t op, const std::vector<std::string>& args) {
  std::lock_guard<std::mutex> g(mu_);
  write_all(fd_, encode(op, args));
  char head[5];
  if (!read_exact(fd_, head, 5)) throw std::runtime_error("xddp store: connection to server lost");
  uint8_t st = static_cast<uint8_t>(head[0]);
  uint32_t n;
  std::memcpy(&n, head + 1, 4);
  std::vector<std::string> parts;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t len;
    if (!read_exact(fd_, reinterpret_cast<char*>(&len), 4)) throw std::runtime_error("xddp store: connection lost");
    std::string s(len, '\0');
    if (len && !read_exact(fd_, &s[0], len)) throw std::runtime_error("xddp store: connection lost");
    parts.push_back(std::move(s));
  }
  if (st == TIMEOUT) {
    std::ostringstream os;
    os << "xddp store: timeout waiting for keys [";
    for (size_t i = 0; i + 1 < args.size(); ++i) os << (i ? ", " : "") << args[i];
    os << "]";
    throw StoreTimeout(os.str());
  }
  if (st == ERR) throw std::runtime_error("xddp store server error: " + (parts.empty() ? std::string() : parts[0]));
  return parts;
}

void TCPStore::set(const std::string& k, const std::string& v) { request(SET, {k, v}); }
std::string TCPStore::get(const std::string& k) {
  return request(GET, {k, std::to_string(timeout.count())}).at(0);
}
int64_t TCPStore::add(const std::string& k, int64_t d) { return std::stoll(request(ADD, {k, std::to_string(d)}).at(0)); }
std::string TCPStore::compare_set(const std::string& k, const std::string& e, const std::string& d) {
  return request(CAS, {k, e, d}).at(0);
}
bool TCPStore::check(const std::vector<std::string>& keys) { return request(CHECK, keys).at(0) == "1"; }
void TCPStore::wait(const std::vector<std::string>& keys, std::chrono::milliseconds t) {
  auto a = keys;
  a.push_back(std::to_string(t.count()));
  request(WAIT, a);
}
bool TCPStore::delete_key(const std::string& k) { return request(DEL, {k}).at(0) == "1"; }
int64_t TCPStore::num_keys() { return std::stoll(request(NUMKEYS, {}).at(0)); }
void TCPStore::append(const std::string& k, const std::string& v) { request(APPEND, {k, v}); }

// -------------------------------------------------------------------------------------
// HashStore
// -------------------------------------------------------------------------------------
void HashStore::set(const std::string& k, const std::string& v) {
  {
    std::lock_guard<std::mutex> g(mu_);
    kv_[k] = v;
  }
  cv_.notify_all();
}
std::string HashStore::get(const std::string& k) {
  std::unique_lock<std::mutex> g(mu_);
  if (!cv_.wait_for(g, timeout, [&] { return kv_.count(k) > 0; })) throw StoreTimeout("xddp HashStore: timeout on " + k);
  return kv_[k];
}
int64_t HashStore::add(const std::string& k, int64_t d) {
  int64_t v;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(k);
    v = (it == kv_.end() || it->second.empty() ? 0 : std::stoll(it->second)) + d;
    kv_[k] = std::to_string(v);
  }
  cv_.notify_all();
  return v;
}
std::string HashStore::compare_set(const std::string& k, const std::string& e, const std::string& d) {
  std::string r;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(k);
    if (it == kv_.end()) {
      if (e.empty()) { kv_[k] = d; r = d; } else { r = e; }
    } else if (it->second == e) {
      it->second = d;
      r = d;
    } else {
      r = it->second;
    }
  }
  cv_.notify_all();
  return r;
}
bool HashStore::check(const std::vector<std::string>& keys) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& k : keys)
    if (!kv_.count(k)) return false;
  return true;
}
void HashStore::wait(const std::vector<std::string>& keys, std::chrono::milliseconds t) {
  std::unique_lock<std::mutex> g(mu_);
  bool ok = cv_.wait_for(g, t, [&] {
    for (auto& k : keys)
      if (!kv_.count(k)) return false;
    return true;
  });
  if (!ok) throw StoreTimeout("xddp HashStore: wait timeout");
}
bool HashStore::delete_key(const std::string& k) {
  std::lock_guard<std::mutex> g(mu_);
  return kv_.erase(k) > 0;
}
int64_t HashStore::num_keys() {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int64_t>(kv_.size());
}
void HashStore::append(const std::string& k, const std::string& v) {
  {
    std::lock_guard<std::mutex> g(mu_);
    kv_[k] += v;
  }
  cv_.notify_all();
}

}  // namespace xddp
