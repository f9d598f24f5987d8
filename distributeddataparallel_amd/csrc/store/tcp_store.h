// Native TCP key-value store used for rendezvous, RCCL unique-id exchange, barriers and
// error signalling (the reference stack's c10d::TCPStore, re-designed:
// one poll()-driven server thread, blocking clients, server-side waiters with deadlines).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <stdexcept>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace xddp {

class StoreTimeout : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Store {
 public:
  virtual ~Store() = default;
  virtual void set(const std::string& key, const std::string& value) = 0;
  // Blocks until key exists (or timeout).
  virtual std::string get(const std::string& key) = 0;
  virtual int64_t add(const std::string& key, int64_t delta) = 0;
  virtual std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired) = 0;
  virtual bool check(const std::vector<std::string>& keys) = 0;
  virtual void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) = 0;
  virtual bool delete_key(const std::string& key) = 0;
  virtual int64_t num_keys() = 0;
  virtual void append(const std::string& key, const std::string& value) = 0;
  std::chrono::milliseconds timeout{std::chrono::minutes(30)};
};

class TCPStoreServer;

// Client (and, on the master rank, owner of the server thread).
class TCPStore : public Store {
 public:
  // is_server: start a server bound on `port` (0 = ephemeral; see port()).
  TCPStore(const std::string& host, int port, bool is_server, int world_size, std::chrono::milliseconds timeout,
           bool wait_for_workers);
  ~TCPStore() override;

  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  int64_t add(const std::string& key, int64_t delta) override;
  std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired) override;
  bool check(const std::vector<std::string>& keys) override;
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override;
  bool delete_key(const std::string& key) override;
  int64_t num_keys() override;
  void append(const std::string& key, const std::string& value) override;

  int port() const { return port_; }
  const std::string& host() const { return host_; }

 private:
  std::vector<std::string> request(uint8_t op, const std::vector<std::string>& args);
  std::string host_;
  int port_;
  int fd_ = -1;
  std::mutex mu_;
  std::unique_ptr<TCPStoreServer> server_;
};

// Namespacing wrapper (c10d::PrefixStore analogue).
class PrefixStore : public Store {
 public:
  PrefixStore(std::string prefix, std::shared_ptr<Store> base) : prefix_(std::move(prefix)), base_(std::move(base)) {
    timeout = base_->timeout;
  }
  void set(const std::string& k, const std::string& v) override { base_->set(p(k), v); }
  std::string get(const std::string& k) override { return base_->get(p(k)); }
  int64_t add(const std::string& k, int64_t d) override { return base_->add(p(k), d); }
  std::string compare_set(const std::string& k, const std::string& e, const std::string& d) override {
    return base_->compare_set(p(k), e, d);
  }
  bool check(const std::vector<std::string>& keys) override { return base_->check(ps(keys)); }
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds t) override { base_->wait(ps(keys), t); }
  bool delete_key(const std::string& k) override { return base_->delete_key(p(k)); }
  int64_t num_keys() override { return base_->num_keys(); }
  void append(const std::string& k, const std::string& v) override { base_->append(p(k), v); }
  std::shared_ptr<Store> base() const { return base_; }

 private:
  std::string p(const std::string& k) const { return prefix_ + "/" + k; }
  std::vector<std::string> ps(const std::vector<std::string>& ks) const {
    std::vector<std::string> r;
    for (auto& k : ks) r.push_back(p(k));
    return r;
  }
  std::string prefix_;
  std::shared_ptr<Store> base_;
};

// In-process store (c10d::HashStore analogue) for single-process tests.
class HashStore : public Store {
 public:
  void set(const std::string& k, const std::string& v) override;
  std::string get(const std::string& k) override;
  int64_t add(const std::string& k, int64_t d) override;
  std::string compare_set(const std::string& k, const std::string& e, const std::string& d) override;
  bool check(const std::vector<std::string>& keys) override;
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds t) override;
  bool delete_key(const std::string& k) override;
  int64_t num_keys() override;
  void append(const std::string& k, const std::string& v) override;

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
};

}  // namespace xddp
