// Peer-memory collectives over IPC-mapped staging buffers on an MI355X node (SURVEY.md §5.8
// item 3). Every GPU has a direct xGMI link to each of the other seven, so a collective does not
// need a ring: ranks stage their input in their own IPC-exported buffer and read each other's
// staged copies straight over the links.
//
// Two lanes, each with its own staging buffer, flags and per-workgroup call counters:
//
//  * one-shot (latency-bound messages: the per-forward buffer broadcast, the find-unused bitmap,
//    the small first bucket): stage, one flag barrier, every rank reads ALL peers' copies and
//    reduces them in registers. One network hop, but each rank pulls (W-1)·S bytes.
//  * two-shot (bucket-sized messages): stage, barrier, rank r reduces slice r (1/W of the
//    message) by reading that slice from all W-1 peers at once, writes the result back into its
//    own staging slot, barrier, then every rank gathers the other W-1 reduced slices. Each rank
//    pulls 2(W-1)/W·S bytes and the reads of one launch are spread over all seven links — the
//    all-links bound of §5.8 (≈7 × 153 GB/s) instead of one ring's single link.
//
// Synchronisation, per lane and per workgroup b:
//   gen = gen_dev[b] + 1 is this workgroup's call number (a device-side counter, so a HIP-graph
//   replay of the same kernel still advances it). EVERY launch of a lane runs the lane's whole grid
//   — workgroups without data only take part in the barriers — so all workgroups of a lane agree on
//   gen and the double-buffer slot (gen & 1) is a property of the CALL, not of the workgroup: a
//   fast rank's call k+1 writes the other slot than the one its peers may still be reading for call
//   k, whatever the chunking of the two calls. A barrier raises flag [b][me] in every rank's buffer
//   (release, system scope) and spins until all flags [b][r] of my buffer reach the value (acquire;
//   a fast peer may already be further). One-shot calls use the value 2·gen, two-shot calls 2·gen-1
//   and 2·gen (flags only grow). Slot reuse is safe: a rank writes slot gen & 1 again at call
//   gen + 2, which needs every peer's first flag of call gen + 1, raised only after that peer's
//   call gen had finished (stream order).
// Every spin is bounded by the wall clock. A workgroup whose peer does not arrive in time sets the
// host-mapped status word (the communicator's watchdog and Work completion read it without a
// device sync and turn it into an error), still advances its counter and exits, so the grid always
// drains; the collective's output is then invalid and the communicator is torn down.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_fp16.h>
#include <torch/extension.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "comm/peer.h"
#include "common.h"

namespace xddp {

namespace {

constexpr int kThreads = 256;

struct PeerPtrs {
  uint8_t* data[kPeerMaxRanks];  // rank r's staging slots (slot s at s * slot_bytes)
  uint32_t* flags[kPeerMaxRanks];
};

__device__ __forceinline__ uint32_t ld_acquire_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_release_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Cross-rank barrier of workgroup b at value `val`. Returns false (and raises the status word)
// when a peer did not arrive within the timeout. Uses no LDS: wave 0 raises this rank's flags and
// EVERY wave polls the peers' flags itself. A spinning workgroup that held LDS (or many registers)
// would keep LDS-heavy compute kernels — the GEMMs and convolutions running concurrently on the
// compute stream — off its CU until the peers arrive; when the peers share the GPU (2 processes
// on one device) that is a deadlock broken only by the timeout.
// The verdict is workgroup-wide: a wave whose peer timed out writes the call number into the
// workgroup's own fail word (global memory, not LDS) before the block barrier, and every wave
// reads it after the barrier, so all waves take the same branch and reach the same later
// __syncthreads (per-wave verdicts could send some waves into a second barrier and others past it).
__device__ __forceinline__ bool flag_barrier(const PeerPtrs& pp, int b, int rank, int size, uint32_t val,
                                             int* status, uint64_t timeout_ticks, uint32_t* fail_word,
                                             uint32_t gen) {
  __threadfence_system();  // every thread's staging stores are visible system-wide before the flags go out
  __syncthreads();
  if (threadIdx.x < size) st_release_sys(pp.flags[threadIdx.x] + b * kPeerMaxRanks + rank, val);
  const int lane = threadIdx.x & 63;
  if (lane < size) {
    const uint32_t* f = pp.flags[rank] + b * kPeerMaxRanks + lane;
    const uint64_t t0 = wall_clock64();
    while (ld_acquire_sys(f) < val) {
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(fail_word, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();  // (workgroup-scope release/acquire: the fail word is visible to every wave)
  const bool ok = __hip_atomic_load(fail_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != gen;
  __threadfence_system();  // acquire side for the lanes that did not poll
  return ok;
}

// element <-> accumulator conversions (bf16 and fp16 reduce in fp32, integers in their own type)
template <typename T>
struct Acc {
  using type = T;
  __device__ static type get(T v) { return v; }
  __device__ static T put(type v) { return v; }
};
template <>
struct Acc<uint16_t> {  // bf16 storage
  using type = float;
  __device__ static float get(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
  __device__ static uint16_t put(float f) {
    const uint32_t u = __float_as_uint(f);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);  // RNE (finite inputs)
  }
};
template <>
struct Acc<__half> {
  using type = float;
  __device__ static float get(__half v) { return __half2float(v); }
  __device__ static __half put(float f) { return __float2half(f); }
};

template <typename T>
__device__ __forceinline__ void copy_range(T* __restrict__ dst, const T* __restrict__ src, int64_t lo, int64_t hi) {
  constexpr int V = 16 / sizeof(T);
  if (hi <= lo) return;
  const int64_t nv = (hi - lo) / V;  // lo is a multiple of V
  for (int64_t i = threadIdx.x; i < nv; i += kThreads)
    reinterpret_cast<uint4*>(dst + lo)[i] = reinterpret_cast<const uint4*>(src + lo)[i];
  for (int64_t i = lo + nv * V + threadIdx.x; i < hi; i += kThreads) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------- one-shot
// MODE 0: all-reduce in place (MAXOP: max instead of sum); 1: broadcast from root in place;
// 2: all-gather — io is this rank's input, out[r * n ...] receives rank r's.
template <typename T, int MODE, bool MAXOP = false>
__global__ __launch_bounds__(kThreads) void peer_kernel(T* __restrict__ io, int64_t n, PeerPtrs pp, int rank,
                                                        int size, int root, uint32_t* __restrict__ gen_dev,
                                                        uint32_t* __restrict__ fail_dev,
                                                        int* status, float scale, bool do_scale,
                                                        uint64_t timeout_ticks, int64_t slot_bytes, int64_t chunk,
                                                        T* __restrict__ out) {
  constexpr bool BCAST = MODE == 1;
  constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
  union Vec {
    uint4 u;
    T e[V];
  };
  const int b = blockIdx.x;
  const uint32_t gen = gen_dev[b] + 1u;  // every thread reads it (no LDS); thread 0 writes it back last
  const int64_t lo = min(n, (int64_t)b * chunk), hi = min(n, lo + chunk);  // chunk is a multiple of V
  const int64_t off = (int64_t)(gen & 1u) * slot_bytes;
  T* mine = reinterpret_cast<T*>(pp.data[rank] + off);

  // 1. stage this workgroup's chunk (empty for the workgroups past the end of the message)
  if (!BCAST || rank == root) copy_range(mine, io, lo, hi);
  // 2. cross-rank barrier on this workgroup's flags
  if (flag_barrier(pp, b, rank, size, 2u * gen, status, timeout_ticks, fail_dev + b, gen)) {
    // 3. reduce (or read the root's copy) straight from the peers' slots
    const int64_t nv = (hi - lo) / V;
    if (MODE == 2) {
      for (int r = 0; r < size; ++r)
        copy_range(out + (int64_t)r * n, reinterpret_cast<const T*>(pp.data[r] + off), lo, hi);
    } else if (BCAST) {
      if (rank != root) copy_range(io, reinterpret_cast<const T*>(pp.data[root] + off), lo, hi);
    } else {
      using A = typename Acc<T>::type;
      for (int64_t i = threadIdx.x; i < nv; i += kThreads) {
        A acc[V];
        for (int r = 0; r < size; ++r) {  // fixed rank order: every rank gets bitwise the same sum
          Vec v;
          v.u = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(pp.data[r] + off) + lo)[i];
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const A x = Acc<T>::get(v.e[e]);
            acc[e] = r == 0 ? x : (MAXOP ? (x > acc[e] ? x : acc[e]) : acc[e] + x);
          }
        }
        Vec o;
#pragma unroll
        for (int e = 0; e < V; ++e) o.e[e] = Acc<T>::put(do_scale ? A(acc[e] * scale) : acc[e]);
        reinterpret_cast<uint4*>(io + lo)[i] = o.u;
      }
      for (int64_t i = lo + nv * V + threadIdx.x; i < hi; i += kThreads) {
        A acc = A(0);
        for (int r = 0; r < size; ++r) {
          const A x = Acc<T>::get(reinterpret_cast<const T*>(pp.data[r] + off)[i]);
          acc = r == 0 ? x : (MAXOP ? (x > acc ? x : acc) : acc + x);
        }
        io[i] = Acc<T>::put(do_scale ? A(acc * scale) : acc);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) gen_dev[b] = gen;  // also after a timeout: the call is over for this workgroup
}

// ---------------------------------------------------------------------------------- two-shot
// Workgroup b owns chunk [b*chunk, (b+1)*chunk) of the message; slice s of the chunk is
// [lo + s*cs, lo + (s+1)*cs), cs = chunk / W (a multiple of the 16-B vector). Rank r reduces slice r.
template <typename T, int W>
__global__ __launch_bounds__(kThreads) void two_shot_kernel(T* __restrict__ io, int64_t n, PeerPtrs pp, int rank,
                                                            uint32_t* __restrict__ gen_dev, uint32_t* __restrict__ fail_dev,
                                                            int* status, float scale, bool do_scale, uint64_t timeout_ticks, int64_t slot_bytes,
                                                            int64_t chunk) {
  constexpr int V = 16 / sizeof(T);
  using A = typename Acc<T>::type;
  union Vec {
    uint4 u;
    T e[V];
  };
  const int b = blockIdx.x;
  const uint32_t gen = gen_dev[b] + 1u;
  const int64_t off = (int64_t)(gen & 1u) * slot_bytes;
  const int64_t cs = chunk / W;
  const int64_t lo = min(n, (int64_t)b * chunk), hi = min(n, lo + chunk);
  const int64_t my_lo = min(hi, lo + rank * cs), my_hi = min(hi, my_lo + cs);
  T* mine = reinterpret_cast<T*>(pp.data[rank] + off);

  // 1. stage the slices the peers will reduce (not my own: I reduce it from io directly)
  copy_range(mine, io, lo, my_lo);
  copy_range(mine, io, my_hi, hi);
  if (flag_barrier(pp, b, rank, W, 2u * gen - 1u, status, timeout_ticks, fail_dev + b, gen)) {
    // 2. reduce my slice from every rank, in rank order (every rank gets bitwise the same sum);
    // the result goes to io and to my staging slot, where the peers gather it from
    const T* src[W];
#pragma unroll
    for (int r = 0; r < W; ++r) src[r] = r == rank ? io : reinterpret_cast<const T*>(pp.data[r] + off);
    const int64_t nv = (my_hi - my_lo) / V;
    for (int64_t i = threadIdx.x; i < nv; i += kThreads) {
      Vec v[W];
#pragma unroll
      for (int r = 0; r < W; ++r) v[r].u = reinterpret_cast<const uint4*>(src[r] + my_lo)[i];  // W loads in flight
      Vec o;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        A acc = Acc<T>::get(v[0].e[e]);
#pragma unroll
        for (int r = 1; r < W; ++r) acc += Acc<T>::get(v[r].e[e]);
        o.e[e] = Acc<T>::put(do_scale ? A(acc * scale) : acc);
      }
      reinterpret_cast<uint4*>(io + my_lo)[i] = o.u;
      reinterpret_cast<uint4*>(mine + my_lo)[i] = o.u;
    }
    for (int64_t i = my_lo + nv * V + threadIdx.x; i < my_hi; i += kThreads) {
      A acc = Acc<T>::get(src[0][i]);
#pragma unroll
      for (int r = 1; r < W; ++r) acc += Acc<T>::get(src[r][i]);
      const T o = Acc<T>::put(do_scale ? A(acc * scale) : acc);
      io[i] = o;
      mine[i] = o;
    }
    // 3. gather the other ranks' reduced slices
    if (flag_barrier(pp, b, rank, W, 2u * gen, status, timeout_ticks, fail_dev + b, gen)) {
#pragma unroll
      for (int r = 0; r < W; ++r) {
        if (r == rank) continue;
        const int64_t s_lo = min(hi, lo + r * cs), s_hi = min(hi, s_lo + cs);
        copy_range(io, reinterpret_cast<const T*>(pp.data[r] + off), s_lo, s_hi);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) gen_dev[b] = gen;
}

}  // namespace

// One staging buffer (flags + two slots) per lane, IPC-mapped into every rank.
struct PeerLane {
  PeerPtrs pp{};
  uint8_t* own = nullptr;
  uint32_t* gen_dev = nullptr;
  int blocks = 0;
  int64_t slot_bytes = 0;

  // Every rank publishes its handle — or an error marker — before it looks at the others', so a
  // rank whose allocation or export failed never leaves its peers waiting on a key that will not
  // come; returns "" on success, else the first failure (this rank's or a peer's marker).
  std::string open(const std::shared_ptr<Store>& store, const std::string& tag, int rank, int size, int nblocks,
                   int64_t slot) {
    blocks = nblocks;
    slot_bytes = slot;
    const int64_t flag_bytes = ((int64_t)nblocks * kPeerMaxRanks * 4 + 4095) / 4096 * 4096;
    const size_t bytes = flag_bytes + 2 * (size_t)slot;
    std::string err, mine;
    try {
      // uncached: the flags and staged data are read by the peers over xGMI while this GPU writes them
      XDDP_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&own), bytes, hipDeviceMallocUncached));
      XDDP_HIP_CHECK(hipMemset(own, 0, bytes));
      // per workgroup: its call counter, then its fail word (the call number of a timed-out barrier)
      XDDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&gen_dev), 2 * nblocks * sizeof(uint32_t)));
      XDDP_HIP_CHECK(hipMemset(gen_dev, 0, 2 * nblocks * sizeof(uint32_t)));
      XDDP_HIP_CHECK(hipDeviceSynchronize());
      hipIpcMemHandle_t h;
      XDDP_HIP_CHECK(hipIpcGetMemHandle(&h, own));
      mine = std::string(reinterpret_cast<const char*>(&h), sizeof(h));
    } catch (const std::exception& e) {
      err = std::string("rank ") + std::to_string(rank) + ": " + e.what();
      mine = "ERR";
    }
    store->set("peer/h/" + tag + "/" + std::to_string(rank), mine);
    for (int r = 0; r < size; ++r) {
      uint8_t* base = own;
      if (r != rank) {
        std::string s = store->get("peer/h/" + tag + "/" + std::to_string(r));
        if (!err.empty()) continue;  // (still read every key: the exchange stays symmetric)
        if (s.size() != sizeof(hipIpcMemHandle_t)) {
          err = "rank " + std::to_string(r) + " could not export its staging buffer";
          continue;
        }
        hipIpcMemHandle_t ph;
        std::memcpy(&ph, s.data(), sizeof(ph));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          err = "rank " + std::to_string(rank) + ": hipIpcOpenMemHandle of rank " + std::to_string(r) + " failed (" +
                hipGetErrorString(e) + ")";
          continue;
        }
        base = static_cast<uint8_t*>(p);
      }
      if (err.empty()) {
        pp.flags[r] = reinterpret_cast<uint32_t*>(base);
        pp.data[r] = base + flag_bytes;
      }
    }
    return err;
  }

  void close(int rank, int size) {
    if (!own) return;
    for (int r = 0; r < size; ++r)
      if (r != rank && pp.flags[r]) (void)hipIpcCloseMemHandle(pp.flags[r]);
    (void)hipFree(own);
    (void)hipFree(gen_dev);
    own = nullptr;
  }
};

struct PeerAllReduce::Impl {
  PeerLane one, two;
  int* status_host = nullptr;  // host-mapped, coherent
  int* status_dev = nullptr;
  uint64_t timeout_ticks = 0;
  int khz = 100000;
};

PeerAllReduce::PeerAllReduce(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                             int64_t two_shot_capacity, std::chrono::milliseconds timeout)
    : rank_(rank), size_(size), device_(device), cap_(capacity), cap2_(two_shot_capacity), impl_(new Impl) {
  TORCH_CHECK(size >= 1 && size <= kPeerMaxRanks, "peer all-reduce: 1..", kPeerMaxRanks, " ranks");
  TORCH_CHECK(capacity > 0 && capacity % 4096 == 0, "peer all-reduce: capacity must be a positive multiple of 4 KiB");
  TORCH_CHECK(two_shot_capacity >= 0 && two_shot_capacity % 4096 == 0,
              "peer all-reduce: two-shot capacity must be a multiple of 4 KiB");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  XDDP_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&impl_->status_host), sizeof(int),
                               hipHostMallocMapped | hipHostMallocCoherent));
  *impl_->status_host = 0;
  XDDP_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&impl_->status_dev), impl_->status_host, 0));
  std::string err = impl_->one.open(store, "1", rank, size, kPeerMaxBlocks, capacity);
  if (two_shot_capacity > 0) {
    // XDDP_PEER_TWO_SHOT_BLOCKS: workgroups of the two-shot grid (8..256, default 64). Every
    // workgroup of a launch is resident while it waits for its peers, and a CU holding one cannot
    // take a whole-CU compute workgroup (all LDS, or 512 registers per SIMD): 64 keeps 3/4 of the
    // CUs for the backward that the all-reduce overlaps. With 256, two processes on one GPU whose
    // GEMMs run concurrently stalled every launch until the timeout (scripts/peer_stress.py).
    int nb = kPeerTwoShotDefaultBlocks;
    if (const char* e = std::getenv("XDDP_PEER_TWO_SHOT_BLOCKS")) nb = std::max(8, std::min(kPeerTwoShotBlocks, std::atoi(e)));
    const std::string e2 = impl_->two.open(store, "2", rank, size, nb, two_shot_capacity);
    if (err.empty()) err = e2;
  }
  int khz = 0;
  XDDP_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  const char* t = std::getenv("XDDP_PEER_TIMEOUT_MS");
  timeout_ms_ = t ? std::atof(t) : static_cast<double>(timeout.count());
  impl_->khz = khz > 0 ? khz : 100000;
  impl_->timeout_ticks = (uint64_t)(timeout_ms_ * impl_->khz);
  // every rank mapped every buffer before the first call raises a flag in it; a failure anywhere
  // fails the construction on EVERY rank (all of them read every rank's verdict)
  store->set("peer/ok/" + std::to_string(rank), err.empty() ? "1" : "0");
  std::string first_bad;
  for (int r = 0; r < size; ++r)
    if (store->get("peer/ok/" + std::to_string(r)) != "1" && first_bad.empty()) first_bad = std::to_string(r);
  if (!err.empty() || !first_bad.empty()) {
    close();
    TORCH_CHECK(false, "peer all-reduce: IPC setup failed (", err.empty() ? "rank " + first_bad + " failed" : err, ")");
  }
}

PeerAllReduce::~PeerAllReduce() {
  // Mappings and buffers live until process exit (the HIP runtime may be gone by the time a
  // static destructor runs); an explicit close() releases them.
}

void PeerAllReduce::close() {
  if (!impl_ || (!impl_->one.own && !impl_->two.own && !impl_->status_host)) return;
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  (void)hipDeviceSynchronize();  // best effort: close() also runs on error paths
  impl_->one.close(rank_, size_);
  impl_->two.close(rank_, size_);
  if (impl_->status_host) (void)hipHostFree(impl_->status_host);
  impl_->status_host = nullptr;
  impl_->status_dev = nullptr;
}

bool PeerAllReduce::supports(const at::Tensor& t, RedOp op, bool bcast) const {
  if (!impl_->one.own || !t.is_cuda() || !t.is_contiguous() || t.device().index() != device_) return false;
  if (t.nbytes() == 0 || (int64_t)t.nbytes() > cap_ || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) return false;
  if (bcast) return true;
  const auto st = t.scalar_type();
  const bool fl = st == at::kFloat || st == at::kBFloat16 || st == at::kHalf || st == at::kDouble;
  if (op == RedOp::SUM || op == RedOp::MAX) return fl || st == at::kInt || st == at::kLong;
  return op == RedOp::AVG && fl;
}

bool PeerAllReduce::supports_two_shot(const at::Tensor& t, RedOp op) const {
  if (!impl_->two.own || !t.is_cuda() || !t.is_contiguous() || t.device().index() != device_) return false;
  if (t.nbytes() == 0 || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) return false;
  const auto st = t.scalar_type();
  return (op == RedOp::SUM || op == RedOp::AVG) && (st == at::kFloat || st == at::kBFloat16 || st == at::kHalf);
}

void PeerAllReduce::run(at::Tensor t, RedOp op, int root, bool bcast, hipStream_t s) {
  TORCH_CHECK(supports(t, op, bcast), "peer all-reduce: unsupported tensor / op");
  launch(t, t, op, root, bcast ? 1 : 0, s);
}

void PeerAllReduce::allgather(at::Tensor out, at::Tensor in, hipStream_t s) {
  TORCH_CHECK(supports(in, RedOp::SUM, true) && out.is_cuda() && out.is_contiguous() &&
                  out.scalar_type() == in.scalar_type() && out.numel() == in.numel() * size_ &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "peer all-gather: unsupported tensors");
  launch(in, out, RedOp::SUM, 0, 2, s);
}

void PeerAllReduce::launch(at::Tensor t, at::Tensor out, RedOp op, int root, int mode, hipStream_t s) {
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  auto& L = impl_->one;
  // data movement modes move bytes: as 4-B words when the size allows (whole 16-B vectors per thread)
  const bool raw = mode != 0;
  const bool words = raw && t.nbytes() % 4 == 0 && (mode != 2 || out.nbytes() % 4 == 0);
  const int64_t esz = raw ? (words ? 4 : 1) : t.element_size();
  const int64_t n = (int64_t)t.nbytes() / esz, vec = 16 / esz;
  // >= 16 KiB per workgroup that has data; the grid is always the lane's full width
  const int64_t busy = std::min<int64_t>(L.blocks, std::max<int64_t>(1, (int64_t)t.nbytes() / 16384));
  int64_t chunk = (n + busy - 1) / busy;
  chunk = (chunk + vec - 1) / vec * vec;
  TORCH_CHECK(chunk * L.blocks >= n, "peer all-reduce: chunking");
  const float scale = 1.f / (float)size_;
  const bool do_scale = op == RedOp::AVG;
  auto go = [&](auto kern, auto* io, auto* o) {
    hipLaunchKernelGGL(kern, dim3((unsigned)L.blocks), dim3(kThreads), 0, s, io, n, L.pp, rank_, size_, root,
                       L.gen_dev, L.gen_dev + L.blocks, impl_->status_dev, scale, do_scale, impl_->timeout_ticks,
                       L.slot_bytes, chunk, o);
  };
  void* p = t.data_ptr();
  void* q = out.data_ptr();
  if (raw) {
    if (words) {
      if (mode == 1) go(peer_kernel<int32_t, 1>, static_cast<int32_t*>(p), static_cast<int32_t*>(q));
      else go(peer_kernel<int32_t, 2>, static_cast<int32_t*>(p), static_cast<int32_t*>(q));
    } else {
      if (mode == 1) go(peer_kernel<uint8_t, 1>, static_cast<uint8_t*>(p), static_cast<uint8_t*>(q));
      else go(peer_kernel<uint8_t, 2>, static_cast<uint8_t*>(p), static_cast<uint8_t*>(q));
    }
  } else {
    const bool mx = op == RedOp::MAX;
#define XDDP_PK(T_)                                                                               \
  if (mx) go(peer_kernel<T_, 0, true>, static_cast<T_*>(p), static_cast<T_*>(q));                 \
  else go(peer_kernel<T_, 0, false>, static_cast<T_*>(p), static_cast<T_*>(q))
    switch (t.scalar_type()) {
      case at::kFloat: XDDP_PK(float); break;
      case at::kDouble: XDDP_PK(double); break;
      case at::kBFloat16: XDDP_PK(uint16_t); break;
      case at::kHalf: XDDP_PK(__half); break;
      case at::kInt: XDDP_PK(int32_t); break;
      case at::kLong: XDDP_PK(int64_t); break;
      default: TORCH_CHECK(false, "peer all-reduce: dtype");
    }
#undef XDDP_PK
  }
  XDDP_HIP_CHECK(hipGetLastError());
}

namespace {

template <typename T, int W>
void launch_two_shot_w(T* io, int64_t n, PeerLane& L, int rank, int* status, float scale, bool do_scale,
                       uint64_t ticks, hipStream_t s) {
  constexpr int64_t V = 16 / sizeof(T);
  int64_t chunk = (n + L.blocks - 1) / L.blocks;
  chunk = (chunk + W * V - 1) / (W * V) * (W * V);  // every slice a whole number of vectors
  hipLaunchKernelGGL((two_shot_kernel<T, W>), dim3((unsigned)L.blocks), dim3(kThreads), 0, s, io, n, L.pp, rank,
                     L.gen_dev, L.gen_dev + L.blocks, status, scale, do_scale, ticks, L.slot_bytes, chunk);
}

template <typename T>
void launch_two_shot(T* io, int64_t n, PeerLane& L, int rank, int size, int* status, float scale, bool do_scale,
                     uint64_t ticks, hipStream_t s) {
  switch (size) {
    case 2: launch_two_shot_w<T, 2>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 3: launch_two_shot_w<T, 3>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 4: launch_two_shot_w<T, 4>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 5: launch_two_shot_w<T, 5>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 6: launch_two_shot_w<T, 6>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 7: launch_two_shot_w<T, 7>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    case 8: launch_two_shot_w<T, 8>(io, n, L, rank, status, scale, do_scale, ticks, s); break;
    default: TORCH_CHECK(false, "peer two-shot all-reduce: 2..8 ranks");
  }
}

}  // namespace

void PeerAllReduce::allreduce_two_shot(at::Tensor t, RedOp op, hipStream_t s) {
  TORCH_CHECK(supports_two_shot(t, op), "peer two-shot all-reduce: unsupported tensor / op");
  if (size_ == 1) {
    return;  // one rank: SUM and AVG are identities
  }
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  auto& L = impl_->two;
  const int64_t esz = t.element_size();
  const int64_t step = cap2_ / esz;  // capacity is a multiple of 4 KiB: whole vectors
  const int64_t n = t.numel();
  const float scale = 1.f / (float)size_;
  const bool do_scale = op == RedOp::AVG;
  for (int64_t off = 0; off < n; off += step) {  // one launch per staging-sized chunk
    const int64_t len = std::min(step, n - off);
    switch (t.scalar_type()) {
      case at::kFloat:
        launch_two_shot(t.data_ptr<float>() + off, len, L, rank_, size_, impl_->status_dev, scale, do_scale,
                        impl_->timeout_ticks, s);
        break;
      case at::kBFloat16:
        launch_two_shot(reinterpret_cast<uint16_t*>(t.data_ptr()) + off, len, L, rank_, size_, impl_->status_dev,
                        scale, do_scale, impl_->timeout_ticks, s);
        break;
      case at::kHalf:
        launch_two_shot(reinterpret_cast<__half*>(t.data_ptr()) + off, len, L, rank_, size_, impl_->status_dev,
                        scale, do_scale, impl_->timeout_ticks, s);
        break;
      default: TORCH_CHECK(false, "peer two-shot all-reduce: dtype");
    }
    XDDP_HIP_CHECK(hipGetLastError());
  }
}

void PeerAllReduce::set_timeout_ms(double ms) {
  timeout_ms_ = ms;
  impl_->timeout_ticks = (uint64_t)(ms * impl_->khz);
}

int PeerAllReduce::status() const {
  if (!impl_->status_host) return 0;
  return __atomic_load_n(impl_->status_host, __ATOMIC_ACQUIRE);
}

}  // namespace xddp
