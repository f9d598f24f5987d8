// File-backed key-value store for ``file://`` rendezvous on a shared filesystem (the reference
// stack's c10d::FileStore role).
//
// The file is an append-only log of records {u8 op, u32 klen, key, u32 vlen, value}; every
// process replays new records into a private map (incremental: it remembers the byte offset it
// has read up to). Mutations take an exclusive flock, replay, then append; blocking reads poll
// with a short sleep. The last process to detach (refcount key) unlinks the file.
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <map>
#include <thread>

#include "store/tcp_store.h"

namespace xddp {

namespace {

constexpr uint8_t kSet = 0, kDel = 1;
constexpr const char* kRefKey = "__xddp_filestore_refcount__";

class Flock {
 public:
  Flock(int fd, int how) : fd_(fd) {
    while (flock(fd_, how) != 0) {
      if (errno != EINTR) throw std::runtime_error(std::string("xddp FileStore: flock: ") + strerror(errno));
    }
  }
  ~Flock() { flock(fd_, LOCK_UN); }

 private:
  int fd_;
};

}  // namespace

class FileStore : public Store {
 public:
  FileStore(std::string path, int world_size) : path_(std::move(path)), world_size_(world_size) {
    fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT, 0644);
    if (fd_ < 0) throw std::runtime_error("xddp FileStore: cannot open " + path_ + ": " + strerror(errno));
    add(kRefKey, 1);
  }
  ~FileStore() override {
    try {
      if (add(kRefKey, -1) <= 0) ::unlink(path_.c_str());
    } catch (...) {
    }
    if (fd_ >= 0) ::close(fd_);
  }

  void set(const std::string& k, const std::string& v) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_EX);
    refresh();
    append_record(kSet, k, v);
  }
  std::string get(const std::string& k) override {
    wait({k}, timeout);
    std::lock_guard<std::mutex> g(mu_);
    return kv_.at(k);
  }
  int64_t add(const std::string& k, int64_t d) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_EX);
    refresh();
    auto it = kv_.find(k);
    const int64_t v = (it == kv_.end() || it->second.empty() ? 0 : std::stoll(it->second)) + d;
    append_record(kSet, k, std::to_string(v));
    return v;
  }
  std::string compare_set(const std::string& k, const std::string& e, const std::string& d) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_EX);
    refresh();
    auto it = kv_.find(k);
    if ((it == kv_.end() && e.empty()) || (it != kv_.end() && it->second == e)) {
      append_record(kSet, k, d);
      return d;
    }
    return it == kv_.end() ? e : it->second;
  }
  bool check(const std::vector<std::string>& keys) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_SH);
    refresh();
    for (auto& k : keys)
      if (!kv_.count(k)) return false;
    return true;
  }
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds t) override {
    const auto deadline = std::chrono::steady_clock::now() + t;
    auto sleep = std::chrono::milliseconds(1);
    while (!check(keys)) {
      if (std::chrono::steady_clock::now() >= deadline)
        throw StoreTimeout("xddp FileStore: timeout waiting for key " + (keys.empty() ? "" : keys[0]) + " in " +
                           path_);
      std::this_thread::sleep_for(sleep);
      sleep = std::min(sleep * 2, std::chrono::milliseconds(20));
    }
  }
  bool delete_key(const std::string& k) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_EX);
    refresh();
    if (!kv_.count(k)) return false;
    append_record(kDel, k, "");
    return true;
  }
  int64_t num_keys() override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_SH);
    refresh();
    return static_cast<int64_t>(kv_.size()) - (kv_.count(kRefKey) ? 1 : 0);
  }
  void append(const std::string& k, const std::string& v) override {
    std::lock_guard<std::mutex> g(mu_);
    Flock l(fd_, LOCK_EX);
    refresh();
    auto it = kv_.find(k);
    append_record(kSet, k, (it == kv_.end() ? std::string() : it->second) + v);
  }
  const std::string& path() const { return path_; }

 private:
  // Replays records appended since the last call (caller holds the flock).
  void refresh() {
    struct stat st;
    if (fstat(fd_, &st) != 0) throw std::runtime_error("xddp FileStore: fstat failed");
    if (st.st_size <= pos_) return;
    std::string buf(static_cast<size_t>(st.st_size - pos_), '\0');
    size_t got = 0;
    while (got < buf.size()) {
      ssize_t r = ::pread(fd_, &buf[got], buf.size() - got, pos_ + static_cast<off_t>(got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) throw std::runtime_error("xddp FileStore: short read of " + path_);
      got += static_cast<size_t>(r);
    }
    size_t i = 0;
    auto rd32 = [&](uint32_t& v) {
      std::memcpy(&v, buf.data() + i, 4);
      i += 4;
    };
    while (i + 9 <= buf.size()) {
      const size_t start = i;
      const uint8_t op = static_cast<uint8_t>(buf[i++]);
      uint32_t kl, vl;
      rd32(kl);
      if (i + kl + 4 > buf.size()) { i = start; break; }
      std::string k = buf.substr(i, kl);
      i += kl;
      rd32(vl);
      if (i + vl > buf.size()) { i = start; break; }
      if (op == kSet) kv_[k] = buf.substr(i, vl);
      else kv_.erase(k);
      i += vl;
    }
    pos_ += static_cast<off_t>(i);
  }
  void append_record(uint8_t op, const std::string& k, const std::string& v) {
    std::string rec;
    rec.push_back(static_cast<char>(op));
    const uint32_t kl = static_cast<uint32_t>(k.size()), vl = static_cast<uint32_t>(v.size());
    rec.append(reinterpret_cast<const char*>(&kl), 4);
    rec += k;
    rec.append(reinterpret_cast<const char*>(&vl), 4);
    rec += v;
    const off_t at = ::lseek(fd_, 0, SEEK_END);
    size_t put = 0;
    while (put < rec.size()) {
      ssize_t w = ::pwrite(fd_, rec.data() + put, rec.size() - put, at + static_cast<off_t>(put));
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) throw std::runtime_error("xddp FileStore: write failed on " + path_);
      put += static_cast<size_t>(w);
    }
    refresh();  // picks up our own record (and advances pos_)
  }

  std::string path_;
  int world_size_;
  int fd_ = -1;
  off_t pos_ = 0;
  std::mutex mu_;
  std::map<std::string, std::string> kv_;
};

std::shared_ptr<Store> make_file_store(const std::string& path, int world_size) {
  return std::make_shared<FileStore>(path, world_size);
}

}  // namespace xddp
