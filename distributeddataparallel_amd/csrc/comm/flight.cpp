// Flight-recorder serialization and dump-on-error (the reference stack's
// ProcessGroupNCCL dumps its per-collective trace buffer when the watchdog fires).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "comm/comm.h"

namespace xddp {

namespace {
std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    if (static_cast<unsigned char>(c) < 0x20) continue;
    o.push_back(c);
  }
  return o;
}
}  // namespace

std::string FlightRecorder::to_json(int rank, const std::string& backend, const std::string& reason) {
  auto entries = dump();
  std::ostringstream os;
  os << "{\"rank\": " << rank << ", \"backend\": \"" << esc(backend) << "\", \"reason\": \"" << esc(reason)
     << "\", \"dumped_at_ns\": " << now_ns() << ", \"num_collectives\": " << count() << ", \"entries\": [";
  for (size_t i = 0; i < entries.size(); ++i) {
    const auto& e = entries[i];
    os << (i ? ",\n  " : "\n  ") << "{\"seq\": " << e.seq << ", \"op\": \"" << esc(e.op) << "\", \"numel\": "
       << e.numel << ", \"dtype\": \"" << esc(e.dtype) << "\", \"t_enqueue_ns\": " << e.t_enqueue_ns
       << ", \"t_done_ns\": " << e.t_done_ns << ", \"state\": \"" << esc(e.state) << "\"}";
  }
  os << "]}\n";
  return os.str();
}

std::string Comm::dump_flight(const std::string& reason, bool force) {
  const char* on = std::getenv("XDDP_FLIGHT_DUMP_ON_ERROR");
  if (!force && on && std::string(on) == "0") return "";
  const char* pre = std::getenv("XDDP_FLIGHT_DUMP_PREFIX");
  const std::string path = std::string(pre && *pre ? pre : "/tmp/xddp_flight_rank_") + std::to_string(rank_) + ".json";
  std::ofstream f(path, std::ios::trunc);
  if (!f) return "";
  f << flight().to_json(rank_, backend(), reason);
  std::fprintf(stderr, "[xddp rank %d] flight record (%s) written to %s\n", rank_, reason.c_str(), path.c_str());
  return path;
}

}  // namespace xddp
