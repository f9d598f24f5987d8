// Device-side helpers for CDNA4 (gfx950): 16-byte vector loads/stores with in-register
// dtype conversion (bf16 via v_cvt_pk_bf16_f32), 64-lane wave reductions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xddp {
namespace dev {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// Storage tags (bit-compatible with at::BFloat16 / at::Half).
struct bf16_t {
  uint16_t x;
};
struct f16_t {
  uint16_t x;
};

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  f32x2 v = {a, b};
  bf16x2 r = __builtin_convertvector(v, bf16x2);  // v_cvt_pk_bf16_f32 (RNE) on gfx950
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float a) { return (uint16_t)(pack_bf16x2(a, 0.f) & 0xffffu); }
__device__ __forceinline__ float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
  f32x2 v = {a, b};
  f16x2 r = __builtin_convertvector(v, f16x2);
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint16_t f32_to_f16(float a) { return __builtin_bit_cast(uint16_t, (_Float16)a); }

// ---- exact (erf-form) GELU at a few VALU ops ---------------------------------------
// erf(z) = 1 - t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) e^{-z^2}, t = 1 / (1 + p z), z >= 0
// (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7: below fp32 GELU rounding at the bf16 outputs
// these feed): one v_rcp_f32, one v_exp_f32 and ~10 FMAs, branch-free, instead of the library
// erff's two-range polynomial. For z = |x| / sqrt(2), e^{-z^2} = e^{-x^2/2} is also the Gaussian
// factor of gelu', so the gradient reuses it.
struct GeluTerms {
  float cdf;  // Phi(x) = (1 + erf(x / sqrt 2)) / 2
  float pdf;  // phi(x) = e^{-x^2/2} / sqrt(2 pi)
};
__device__ __forceinline__ GeluTerms gelu_terms(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  const float g = __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);  // e^{-z^2}
  const float e = fmaf(-poly, g, 1.f);                                    // erf(|x| / sqrt 2)
  return {0.5f + copysignf(0.5f * e, x), 0.39894228040143268f * g};
}
__device__ __forceinline__ float gelu(float x) { return x * gelu_terms(x).cdf; }
__device__ __forceinline__ float gelu_grad(float x) {
  const GeluTerms k = gelu_terms(x);
  return fmaf(x, k.pdf, k.cdf);
}

// ---- scalar access in compute type ------------------------------------------------
template <typename T, typename C>
struct Elem;
template <typename C>
struct Elem<float, C> {
  static __device__ __forceinline__ C ld(const float* p, int64_t i) { return (C)p[i]; }
  static __device__ __forceinline__ void st(float* p, int64_t i, C v) { p[i] = (float)v; }
};
template <typename C>
struct Elem<double, C> {
  static __device__ __forceinline__ C ld(const double* p, int64_t i) { return (C)p[i]; }
  static __device__ __forceinline__ void st(double* p, int64_t i, C v) { p[i] = (double)v; }
};
template <typename C>
struct Elem<bf16_t, C> {
  static __device__ __forceinline__ C ld(const bf16_t* p, int64_t i) { return (C)bf16_to_f32(p[i].x); }
  static __device__ __forceinline__ void st(bf16_t* p, int64_t i, C v) { p[i].x = f32_to_bf16((float)v); }
};
template <typename C>
struct Elem<f16_t, C> {
  static __device__ __forceinline__ C ld(const f16_t* p, int64_t i) { return (C)f16_to_f32(p[i].x); }
  static __device__ __forceinline__ void st(f16_t* p, int64_t i, C v) { p[i].x = f32_to_f16((float)v); }
};

// ---- 8-wide vector access (16 B per instruction where the dtype allows) ------------
template <typename T>
struct Vec8;
template <>
struct Vec8<float> {
  static constexpr int kAlign = 16;
  template <typename C>
  static __device__ __forceinline__ void ld(const float* p, C (&v)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  template <typename C>
  static __device__ __forceinline__ void st(float* p, const C (&v)[8]) {
    f32x4 a = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    f32x4 b = {(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
  // round values to storage precision in registers (identity for fp32)
  static __device__ __forceinline__ void rt(float (&)[8]) {}
};
template <>
struct Vec8<double> {
  static constexpr int kAlign = 16;
  template <typename C>
  static __device__ __forceinline__ void ld(const double* p, C (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f64x2 a = *reinterpret_cast<const f64x2*>(p + 2 * j);
      v[2 * j] = (C)a.x;
      v[2 * j + 1] = (C)a.y;
    }
  }
  template <typename C>
  static __device__ __forceinline__ void st(double* p, const C (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f64x2 a = {(double)v[2 * j], (double)v[2 * j + 1]};
      *reinterpret_cast<f64x2*>(p + 2 * j) = a;
    }
  }
  static __device__ __forceinline__ void rt(float (&)[8]) {}
};
template <>
struct Vec8<bf16_t> {
  static constexpr int kAlign = 16;
  template <typename C>
  static __device__ __forceinline__ void ld(const bf16_t* p, C (&v)[8]) {
    u32x4 a = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = (C)__uint_as_float(a[j] << 16);
      v[2 * j + 1] = (C)__uint_as_float(a[j] & 0xffff0000u);
    }
  }
  template <typename C>
  static __device__ __forceinline__ void st(bf16_t* p, const C (&v)[8]) {
    u32x4 a;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = pack_bf16x2((float)v[2 * j], (float)v[2 * j + 1]);
    *reinterpret_cast<u32x4*>(p) = a;
  }
  // streaming store: a write-once activation does not displace re-read data from L2 / MALL
  template <typename C>
  static __device__ __forceinline__ void st_nt(bf16_t* p, const C (&v)[8]) {
    u32x4 a;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = pack_bf16x2((float)v[2 * j], (float)v[2 * j + 1]);
    __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(p));
  }
  static __device__ __forceinline__ void rt(float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      v[2 * j] = __uint_as_float(u << 16);
      v[2 * j + 1] = __uint_as_float(u & 0xffff0000u);
    }
  }
};
template <>
struct Vec8<f16_t> {
  static constexpr int kAlign = 16;
  template <typename C>
  static __device__ __forceinline__ void ld(const f16_t* p, C (&v)[8]) {
    u32x4 a = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = (C)f16_to_f32((uint16_t)(a[j] & 0xffffu));
      v[2 * j + 1] = (C)f16_to_f32((uint16_t)(a[j] >> 16));
    }
  }
  template <typename C>
  static __device__ __forceinline__ void st(f16_t* p, const C (&v)[8]) {
    u32x4 a;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = pack_f16x2((float)v[2 * j], (float)v[2 * j + 1]);
    *reinterpret_cast<u32x4*>(p) = a;
  }
  static __device__ __forceinline__ void rt(float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u = pack_f16x2(v[2 * j], v[2 * j + 1]);
      v[2 * j] = f16_to_f32((uint16_t)(u & 0xffffu));
      v[2 * j + 1] = f16_to_f32((uint16_t)(u >> 16));
    }
  }
};

// Non-temporal store where the dtype has one (bf16: the activation dtype of the hot path).
template <typename T, typename C>
__device__ __forceinline__ void st8_stream(T* p, const C (&v)[8]) {
  if constexpr (__is_same(T, bf16_t)) Vec8<bf16_t>::st_nt(p, v);
  else Vec8<T>::st(p, v);
}

// ---- reductions over a 64-lane wavefront ------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `scratch` must hold blockDim.x/64 entries. Result valid in all threads.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

// ---- in-launch hand-off to the last arrivals (a finalize folded into its producer) ------------
// The producing blocks store their partials write-through (st_sc1: global_store … sc1), then
// arrive: every wave drains its stores (s_waitcnt vmcnt(0)), the workgroup barrier, one lane adds
// to the arrival counter (relaxed, agent scope). The last S arrivals become the reducers: one lane
// polls the counter with relaxed sc1 loads until every producer has arrived, the barrier releases
// the other waves, and every read of the partials is an sc1 load (ld_sc1). This is the
// write-through form of the guide's inter-workgroup hand-off (cdna_hip_programming.md §6 Guideline
// 16; MI355X_MICROARCH.md "Valid forms", row 1: atomic-add counter, sc1 poll, barrier, sc1 stores
// and loads), so neither a release nor an acquire fence is needed, and it holds for any placement
// of the blocks over CUs and XCDs. The reducers are arrivals, so every other block has finished
// its work: at most S - 1 blocks are still running, and spinning never starves them of a slot.
// Each reducer adds to the departure counter once its poll matched; the one whose add comes last
// zeroes both counters, so the next launch in stream order (and every graph replay) starts from
// zero with no memset. The spin is bounded: after ~1 s it sets *timeout and goes on.
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(
      __hip_atomic_load(const_cast<unsigned*>(reinterpret_cast<const unsigned*>(p)), __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_AGENT));
}

// Returns this block's reducer rank in [0, S), or -1 (no finalize work). Called by every thread;
// `word` is one int of LDS that no thread reads between this call's barriers.
__device__ __forceinline__ int tail_arrive(unsigned* ctr, int nblocks, int S, int* word, unsigned* timeout) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  const int tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int rank = (int)t - (nblocks - S);
    if (rank >= 0) {
      for (unsigned spins = 0;
           __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nblocks;) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {
          __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (__hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1)) {
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    *word = rank;
  }
  __syncthreads();
  const int rank = *word;
  __syncthreads();  // (the caller may reuse the word's LDS)
  return rank;
}

// XCD-aware remap (bijective for any grid): consecutive logical tiles land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace dev
}  // namespace xddp
