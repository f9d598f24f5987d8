// One-shot all-reduce / broadcast over IPC-mapped peer buffers (xGMI), for latency-bound small
// messages: DDP's per-forward buffer broadcast, the 1 MiB first bucket,
// the find-unused bitmap, join/no_sync flags.
//
// On an MI355X node every GPU has a direct xGMI link to every other one, so a small message does
// not need a ring: each rank stages its input in its own (uncached, IPC-exported) buffer, raises
// a flag in every peer's buffer, waits for the peers' flags, then reads all peers' staged copies
// straight over xGMI and reduces them in registers — one kernel, one network hop, no RCCL
// protocol setup. Per workgroup the message chunk is independent (its own flags), so there is no
// grid-wide barrier.
//
// Synchronisation (per workgroup b, per call):
//   gen = gen_dev[b] + 1 (a device-side counter: the same kernel replayed from a HIP graph still
//   advances it); stage into slot gen & 1; fence (system scope); store gen into flag [b][me] of
//   every rank (release, system scope); spin until every flag [b][r] of my buffer is >= gen
//   (acquire; a fast peer may already have written gen + 1); read the peers' slot gen & 1.
//   Double-buffered slots are safe: a peer can only overwrite slot gen & 1 again at call gen + 2,
//   which needs my flag for gen + 1, raised only after my call gen finished (stream order).
// Every spin is bounded by the wall clock (XDDP_PEER_TIMEOUT_MS, default 10 s): a missing peer
// sets the status word and the workgroup exits, so the grid always drains.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_fp16.h>
#include <torch/extension.h>

#include <cstring>
#include <string>

#include "comm/peer.h"
#include "common.h"

namespace xddp {

namespace {

constexpr int kThreads = 256;
constexpr int kFlagBytes = kPeerMaxBlocks * kPeerMaxRanks * 4;

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

// MODE 0: all-reduce in place (MAXOP: max instead of sum); 1: broadcast from root in place;
// 2: all-gather — io is this rank's input, out[r * n ...] receives rank r's.
template <typename T, int MODE, bool MAXOP = false>
__global__ __launch_bounds__(kThreads) void peer_kernel(T* __restrict__ io, int64_t n, PeerPtrs pp, int rank,
                                                        int size, int root, uint32_t* __restrict__ gen_dev,
                                                        int* __restrict__ status, float scale, bool do_scale,
                                                        uint64_t timeout_ticks, int64_t slot_bytes, int64_t chunk,
                                                        T* __restrict__ out) {
  constexpr bool BCAST = MODE == 1;
  constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
  union Vec {
    uint4 u;
    T e[V];
  };
  const int b = blockIdx.x;
  __shared__ uint32_t s_gen;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    s_gen = gen_dev[b] + 1u;
    s_ok = 1;
  }
  __syncthreads();
  const uint32_t gen = s_gen;
  const int64_t lo = (int64_t)b * chunk, hi = min(n, lo + chunk);  // chunk is a multiple of V
  const int64_t off = (int64_t)(gen & 1u) * slot_bytes;
  T* mine = reinterpret_cast<T*>(pp.data[rank] + off);

  // 1. stage this workgroup's chunk
  if (!BCAST || rank == root) {
    const int64_t nv = (hi - lo) / V;
    for (int64_t i = threadIdx.x; i < nv; i += kThreads)
      reinterpret_cast<uint4*>(mine + lo)[i] = reinterpret_cast<const uint4*>(io + lo)[i];
    for (int64_t i = lo + nv * V + threadIdx.x; i < hi; i += kThreads) mine[i] = io[i];
  }
  // 2. cross-rank barrier on this workgroup's flags (every thread's staging stores are made
  // visible system-wide before the flags go out)
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < size) {
    st_release_sys(pp.flags[threadIdx.x] + b * kPeerMaxRanks + rank, gen);
    const uint32_t* f = pp.flags[rank] + b * kPeerMaxRanks + threadIdx.x;
    const uint64_t t0 = wall_clock64();
    while (ld_acquire_sys(f) < gen) {
      if (wall_clock64() - t0 > timeout_ticks) {
        s_ok = 0;
        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (!s_ok) return;  // a peer never arrived: leave io untouched, status says why
  __threadfence_system();  // acquire side for the threads that did not poll

  // 3. reduce (or read the root's copy) straight from the peers' slots
  const int64_t nv = (hi - lo) / V;
  if (MODE == 2) {
    for (int r = 0; r < size; ++r) {
      const T* src = reinterpret_cast<const T*>(pp.data[r] + off);
      T* dst = out + (int64_t)r * n;
      for (int64_t i = threadIdx.x; i < nv; i += kThreads)
        reinterpret_cast<uint4*>(dst + lo)[i] = reinterpret_cast<const uint4*>(src + lo)[i];
      for (int64_t i = lo + nv * V + threadIdx.x; i < hi; i += kThreads) dst[i] = src[i];
    }
  } else if (BCAST) {
    if (rank != root) {
      const T* src = reinterpret_cast<const T*>(pp.data[root] + off);
      for (int64_t i = threadIdx.x; i < nv; i += kThreads)
        reinterpret_cast<uint4*>(io + lo)[i] = reinterpret_cast<const uint4*>(src + lo)[i];
      for (int64_t i = lo + nv * V + threadIdx.x; i < hi; i += kThreads) io[i] = src[i];
    }
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
  __syncthreads();
  if (threadIdx.x == 0) gen_dev[b] = gen;
}

}  // namespace

struct PeerAllReduce::Impl {
  PeerPtrs pp{};
  uint8_t* own = nullptr;
  uint32_t* gen_dev = nullptr;
  int* status = nullptr;
  uint64_t timeout_ticks = 0;
};

PeerAllReduce::PeerAllReduce(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity)
    : rank_(rank), size_(size), device_(device), cap_(capacity), impl_(new Impl) {
  TORCH_CHECK(size >= 1 && size <= kPeerMaxRanks, "peer all-reduce: 1..", kPeerMaxRanks, " ranks");
  TORCH_CHECK(capacity > 0 && capacity % 4096 == 0, "peer all-reduce: capacity must be a positive multiple of 4 KiB");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  const size_t bytes = kFlagBytes + 2 * (size_t)capacity;
  // uncached: the flags and staged data are read by the peers over xGMI while this GPU writes them
  XDDP_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&impl_->own), bytes, hipDeviceMallocUncached));
  XDDP_HIP_CHECK(hipMemset(impl_->own, 0, bytes));
  XDDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&impl_->gen_dev), kPeerMaxBlocks * sizeof(uint32_t)));
  XDDP_HIP_CHECK(hipMemset(impl_->gen_dev, 0, kPeerMaxBlocks * sizeof(uint32_t)));
  XDDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&impl_->status), sizeof(int)));
  XDDP_HIP_CHECK(hipMemset(impl_->status, 0, sizeof(int)));
  XDDP_HIP_CHECK(hipDeviceSynchronize());
  hipIpcMemHandle_t h;
  XDDP_HIP_CHECK(hipIpcGetMemHandle(&h, impl_->own));
  store->set("peer/h/" + std::to_string(rank), std::string(reinterpret_cast<const char*>(&h), sizeof(h)));
  for (int r = 0; r < size; ++r) {
    uint8_t* base = impl_->own;
    if (r != rank) {
      std::string s = store->get("peer/h/" + std::to_string(r));
      TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "peer all-reduce: bad IPC handle from rank ", r);
      hipIpcMemHandle_t ph;
      std::memcpy(&ph, s.data(), sizeof(ph));
      void* p = nullptr;
      XDDP_HIP_CHECK(hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess));
      base = static_cast<uint8_t*>(p);
    }
    impl_->pp.flags[r] = reinterpret_cast<uint32_t*>(base);
    impl_->pp.data[r] = base + kFlagBytes;
  }
  int khz = 0;
  XDDP_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  const char* t = std::getenv("XDDP_PEER_TIMEOUT_MS");
  const double ms = t ? std::atof(t) : 10000.0;
  impl_->timeout_ticks = (uint64_t)(ms * (khz > 0 ? khz : 100000));
  // every rank mapped every buffer before the first call raises a flag in it
  store->set("peer/ok/" + std::to_string(rank), "1");
  for (int r = 0; r < size; ++r) store->get("peer/ok/" + std::to_string(r));
}

PeerAllReduce::~PeerAllReduce() {
  // Mappings and buffers live until process exit (the HIP runtime may be gone by the time a
  // static destructor runs); an explicit close() releases them.
}

void PeerAllReduce::close() {
  if (!impl_ || !impl_->own) return;
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  (void)hipDeviceSynchronize();  // best effort: close() also runs on error paths
  for (int r = 0; r < size_; ++r)
    if (r != rank_ && impl_->pp.flags[r]) (void)hipIpcCloseMemHandle(impl_->pp.flags[r]);
  (void)hipFree(impl_->own);
  (void)hipFree(impl_->gen_dev);
  (void)hipFree(impl_->status);
  impl_->own = nullptr;
}

bool PeerAllReduce::supports(const at::Tensor& t, RedOp op, bool bcast) const {
  if (!impl_->own || !t.is_cuda() || !t.is_contiguous() || t.device().index() != device_) return false;
  if (t.nbytes() == 0 || (int64_t)t.nbytes() > cap_ || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) return false;
  if (bcast) return true;
  const auto st = t.scalar_type();
  const bool fl = st == at::kFloat || st == at::kBFloat16 || st == at::kHalf || st == at::kDouble;
  if (op == RedOp::SUM || op == RedOp::MAX) return fl || st == at::kInt || st == at::kLong;
  return op == RedOp::AVG && fl;
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
  // data movement modes move bytes: as 4-B words when the size allows (whole 16-B vectors per thread)
  const bool raw = mode != 0;
  const bool words = raw && t.nbytes() % 4 == 0 && (mode != 2 || out.nbytes() % 4 == 0);
  const int64_t esz = raw ? (words ? 4 : 1) : t.element_size();
  const int64_t n = (int64_t)t.nbytes() / esz, vec = 16 / esz;
  // >= 16 KiB per workgroup, at most kPeerMaxBlocks workgroups; chunks are whole 16-B vectors
  int64_t blocks = std::min<int64_t>(kPeerMaxBlocks, std::max<int64_t>(1, (int64_t)t.nbytes() / 16384));
  int64_t chunk = (n + blocks - 1) / blocks;
  chunk = (chunk + vec - 1) / vec * vec;
  blocks = (n + chunk - 1) / chunk;
  const float scale = 1.f / (float)size_;
  const bool do_scale = op == RedOp::AVG;
  auto go = [&](auto kern, auto* io, auto* o) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), 0, s, io, n, impl_->pp, rank_, size_, root,
                       impl_->gen_dev, impl_->status, scale, do_scale, impl_->timeout_ticks, (int64_t)cap_, chunk, o);
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

int PeerAllReduce::status() {
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  int v = 0;
  XDDP_HIP_CHECK(hipMemcpy(&v, impl_->status, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

}  // namespace xddp
