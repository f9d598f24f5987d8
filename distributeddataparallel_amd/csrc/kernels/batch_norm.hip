// BatchNorm for channels_last (NHWC) activations on gfx950, with fused epilogues.
//
// Reference hot path (SURVEY.md §2.6 K3–K6): per BN layer the eager stack runs
// native_batch_norm (MIOpen) + num_batches_tracked.add_ + relu_ (+ residual add) forward and
// batch_norm_backward + threshold_backward (+ add) backward: 4–6 full passes over the
// activation. Here:
//   forward : stats pass (read x) → tiny per-channel finalize (mean, invstd, running-stat EMA,
//             num_batches_tracked += 1, scale/shift) → apply pass (read x [+res], write y)
//             with BN·γ+β, + residual, ReLU fused;
//   backward: reduce pass (read dy, x, y) → finalize (dγ, dβ and the three dx coefficients)
//             → elementwise pass writing dx (and d(residual) when the add was fused).
// Layout: rows = N·H·W, each row has C contiguous channels. A lane owns 8 consecutive
// channels (16-byte bf16 loads); the block tiles TX lanes across channels × TY lanes down rows.
// Forward statistics are sums of (x - K_c) with one shared per-channel shift K_c = x[0, c],
// so partials add exactly like the backward's and large |mean|/std does not cancel.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <atomic>
#include <cstdlib>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

using dev::bf16_t;
using dev::f16_t;
using dev::Elem;
using dev::Vec8;

namespace {

constexpr int kBlock = 256;
#ifndef XDDP_BN_RED_ROWS
#define XDDP_BN_RED_ROWS 4  // rows per batch of the backward reduce (loads of a batch in flight together)
#endif
#ifndef XDDP_BN_NT
#define XDDP_BN_NT 1  // non-temporal (streaming) stores for the activation-sized outputs
#endif

struct Geo {
  int tx, ty;       // lanes across channel-vectors, lanes down rows
  int cblocks;      // grid.x
  int rblocks;      // grid.y
  int64_t rows_per; // rows per row-block
};

Geo make_geo(int64_t M, int C) {
  Geo g;
  const int cvec = C / 8;
  g.tx = std::min(cvec, 32);
  while (cvec % g.tx) g.tx--;  // tx divides the channel-vector count
  g.ty = kBlock / g.tx;
  g.cblocks = cvec / g.tx;
  // ~512 blocks total (2 per CU, 8 waves/CU) keeps HBM busy while the per-channel finalize
  // only has <= 512 row-block partials to merge
  int64_t want = std::max<int64_t>(1, 512 / g.cblocks);
  int64_t maxr = std::max<int64_t>(1, (M + g.ty - 1) / g.ty);
  g.rblocks = (int)std::min<int64_t>(std::min<int64_t>(want, maxr), 65535);
  g.rows_per = (M + g.rblocks - 1) / g.rblocks;
  g.rblocks = (int)((M + g.rows_per - 1) / g.rows_per);
  return g;
}

// ---------------------------------------------------------------- forward stats
// Common-shift sums: every lane subtracts K_c = x[row 0, c] (a sample of the same channel, so
// |mean - K| is O(std) and sum/sumsq of (x - K) do not cancel even when |mean| >> std — guide
// §5.4 rule 26; the large-offset case has its own test). Partials are then plain additive
// (sum, sumsq) pairs: LDS tree and finalize are adds, no per-merge divisions.
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, int64_t rows_per,
                                                          float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int c0 = (blockIdx.x * TX + tx) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = min(M, r0 + rows_per);
  float s[8] = {0}, ss[8] = {0}, k[8];
  Vec8<T>::ld(x + c0, k);
  int64_t r = r0 + ty;
  // 4 independent 16-B loads in flight per lane (memory-level parallelism), then the tail
  for (; r + 3 * TY < r1; r += 4 * TY) {
    float v0[8], v1[8], v2[8], v3[8];
    Vec8<T>::ld(x + r * C + c0, v0);
    Vec8<T>::ld(x + (r + TY) * C + c0, v1);
    Vec8<T>::ld(x + (r + 2 * TY) * C + c0, v2);
    Vec8<T>::ld(x + (r + 3 * TY) * C + c0, v3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d0 = v0[j] - k[j], d1 = v1[j] - k[j], d2 = v2[j] - k[j], d3 = v3[j] - k[j];
      s[j] += (d0 + d1) + (d2 + d3);
      ss[j] = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, ss[j]))));
    }
  }
  for (; r < r1; r += TY) {
    float v[8];
    Vec8<T>::ld(x + r * C + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - k[j];
      s[j] += d;
      ss[j] = fmaf(d, d, ss[j]);
    }
  }
  // LDS layout [ty][tx][16]: 8 sums then 8 sums of squares, 16-B vector stores
  float* my = lds + (ty * TX + tx) * 16;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    my[j] = s[j];
    my[8 + j] = ss[j];
  }
  __syncthreads();
  for (int stride = TY / 2; stride > 0; stride >>= 1) {
    if (ty < stride) {
      const float* o = lds + ((ty + stride) * TX + tx) * 16;
#pragma unroll
      for (int j = 0; j < 16; ++j) my[j] += o[j];
    }
    __syncthreads();
  }
  if (ty == 0) {
    float* dst = part + ((int64_t)blockIdx.y * C + c0) * 2;  // [rblock][c/8][16]
#pragma unroll
    for (int j = 0; j < 16; ++j) dst[j] = my[j];
  }
}

// One 64-lane wave per 8-channel vector: lanes stride over the row-block partials (4 loads in
// flight), then a 6-step xor-shuffle butterfly of plain adds — no LDS, no barriers.
// Lane j < 8 finalizes channel cv*8+j (mean, invstd, running-stat EMA, scale/shift).
// MOMENTS: write this rank's (count, mean, M2) to mean_out as [3, C] and stop (SyncBatchNorm merges
// the ranks' moments before any coefficient exists).
template <typename T, typename W, bool MOMENTS = false>
__global__ __launch_bounds__(64) void bn_stats_finalize_kernel(
    const float* __restrict__ part, int rblocks, int C, int64_t M, const T* __restrict__ x,
    const W* __restrict__ weight, const W* __restrict__ bias, W* running_mean, W* running_var,
    const int64_t* nbt, float momentum, bool cma, float eps, float* __restrict__ mean_out,
    float* __restrict__ invstd_out, float* __restrict__ scale, float* __restrict__ shift) {
  const int cv = blockIdx.x, lane = threadIdx.x;
  float a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = 0.f;
  const float* base = part + (int64_t)cv * 16;
  const int64_t rstride = (int64_t)C * 2;
  int b = lane;
  for (; b + 192 < rblocks; b += 256) {
    float4 q[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) q[u][v] = reinterpret_cast<const float4*>(base + (b + 64 * u) * rstride)[v];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        a[4 * v] += q[u][v].x; a[4 * v + 1] += q[u][v].y; a[4 * v + 2] += q[u][v].z; a[4 * v + 3] += q[u][v].w;
      }
  }
  for (; b < rblocks; b += 64) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 q = reinterpret_cast<const float4*>(base + b * rstride)[v];
      a[4 * v] += q.x; a[4 * v + 1] += q.y; a[4 * v + 2] += q.z; a[4 * v + 3] += q.w;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] += __shfl_xor(a[j], o, 64);
  if (lane >= 8) return;
  // lane j picks channel j out of its (identical) registers without dynamic indexing
  float S = a[0], SS = a[8];
#pragma unroll
  for (int j = 1; j < 8; ++j)
    if (lane == j) { S = a[j]; SS = a[8 + j]; }
  const int c = cv * 8 + lane;
  const float inv_m = 1.f / (float)M;
  const float dm = S * inv_m;
  const float var = fmaxf(SS * inv_m - dm * dm, 0.f);
  const float mean = Elem<T, float>::ld(x, c) + dm;
  if (MOMENTS) {
    mean_out[c] = (float)M;
    mean_out[C + c] = mean;
    mean_out[2 * C + c] = var * (float)M;
    return;
  }
  const float inv = rsqrtf(var + eps);
  mean_out[c] = mean;
  invstd_out[c] = inv;
  const float g = weight ? Elem<W, float>::ld(weight, c) : 1.f;
  const float bb = bias ? Elem<W, float>::ld(bias, c) : 0.f;
  scale[c] = g * inv;
  shift[c] = bb - mean * g * inv;
  if (running_mean) {
    float mom = momentum;
    if (cma && nbt) mom = 1.f / (float)(nbt[0] + 1);  // nbt is incremented later, by the apply kernel
    const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
    Elem<W, float>::st(running_mean, c, (1.f - mom) * Elem<W, float>::ld(running_mean, c) + mom * mean);
    Elem<W, float>::st(running_var, c, (1.f - mom) * Elem<W, float>::ld(running_var, c) + mom * unbiased);
  }
}

// eval mode: scale/shift from running stats
template <typename W>
__global__ void bn_eval_coef_kernel(int C, const W* weight, const W* bias, const W* rm, const W* rv, float eps,
                                    float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(Elem<W, float>::ld(rv, c) + eps);
  const float g = weight ? Elem<W, float>::ld(weight, c) : 1.f;
  const float b = bias ? Elem<W, float>::ld(bias, c) : 0.f;
  scale[c] = g * inv;
  shift[c] = b - Elem<W, float>::ld(rm, c) * g * inv;
}

// ---------------------------------------------------------------- apply
// mbits (optional, RELU only): one byte per 8-channel vector, bit j = (y_j > 0) — the backward
// reads 1/16 of a bf16 activation pass instead of y to rebuild the ReLU mask.
template <typename T, bool RES, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                          T* __restrict__ y, int64_t nvec, int C,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int64_t* nbt_inc,
                                                          uint8_t* __restrict__ mbits, const float* __restrict__ rss,
                                                          int64_t* nbt_inc2) {
  // rss: the residual is the raw output of another BatchNorm (the downsample's) whose apply is
  // folded in here: r -> r·rscale + rshift (rss = [2][C]); nbt_inc2 is that BN's counter
  if (nbt_inc && blockIdx.x == 0 && threadIdx.x == 0) nbt_inc[0] += 1;  // num_batches_tracked.add_(1), fused
  if (nbt_inc2 && blockIdx.x == 0 && threadIdx.x == 0) nbt_inc2[0] += 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // channel offset advanced incrementally: no 64-bit modulo in the loop
  const int cstep = (int)((stride * 8) % C);
  int c0 = (int)((v0 * 8) % C);
  for (int64_t v = v0; v < nvec; v += stride, c0 = (c0 + cstep >= C) ? c0 + cstep - C : c0 + cstep) {
    const int64_t e = v * 8;
    float a[8], r[8];
    Vec8<T>::ld(x + e, a);
    if (RES) {
      Vec8<T>::ld(res + e, r);
      if (rss) {  // (uniform per launch)
        float rs[8], rh[8];
        dev::Vec8<float>::ld(rss + c0, rs);
        dev::Vec8<float>::ld(rss + C + c0, rh);
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = fmaf(r[j], rs[j], rh[j]);
        Vec8<T>::rt(r);  // at storage precision, as the downsample's own apply pass would store it
      }
    }
    const dev::f32x4 s0 = *reinterpret_cast<const dev::f32x4*>(scale + c0);
    const dev::f32x4 s1 = *reinterpret_cast<const dev::f32x4*>(scale + c0 + 4);
    const dev::f32x4 h0 = *reinterpret_cast<const dev::f32x4*>(shift + c0);
    const dev::f32x4 h1 = *reinterpret_cast<const dev::f32x4*>(shift + c0 + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(a[j], sc[j], sh[j]);
      if (RES) o += r[j];
      if (RELU) {
        bits |= (o > 0.f ? 1u : 0u) << j;
        o = fmaxf(o, 0.f);
      }
      a[j] = o;
    }
    if (XDDP_BN_NT) dev::st8_stream(y + e, a); else Vec8<T>::st(y + e, a);
    if (RELU && mbits) mbits[v] = (uint8_t)bits;
  }
}

// Counters of the finalize folded into the reduce kernels (dev::tail_arrive): per launch slot and
// channel group an (arrival, departure) pair. Zero at code-object load, zeroed again by each
// launch's last reducer; a launch takes the next slot round-robin, so launches in flight on
// different streams do not share counters.
constexpr int kTailSlots = 64, kTailGroups = 64;
__device__ unsigned g_bn_tail_ctr[kTailSlots * kTailGroups * 2];
__device__ unsigned g_bn_tail_timeout;

struct BwdFin {
  int slot;       // folded form: this launch's counter slot in g_bn_tail_ctr (-1: separate kernel)
  int S;          // folded form: reducer blocks per channel group
  int wdt;
  int64_t M;
  const void* weight;
  const float* invstd;
  void* dweight;
  void* dbias;
  float* coef;
  const float* fold_mean;
  const float* ss_copy;
  int dbg = 0;  // (timing only, XDDP_BN_TAIL_DBG: 1 = stop after the partial stores, 3 = after the poll)
};

__device__ __forceinline__ float ld_w(const void* p, int wdt, int c) {
  return wdt == 1 ? Elem<bf16_t, float>::ld(static_cast<const bf16_t*>(p), c)
                  : (wdt == 2 ? Elem<f16_t, float>::ld(static_cast<const f16_t*>(p), c) : static_cast<const float*>(p)[c]);
}
__device__ __forceinline__ void st_w(void* p, int wdt, int c, float v) {
  if (wdt == 1) Elem<bf16_t, float>::st(static_cast<bf16_t*>(p), c, v);
  else if (wdt == 2) Elem<f16_t, float>::st(static_cast<f16_t*>(p), c, v);
  else static_cast<float*>(p)[c] = v;
}

// per channel: dgamma, dbeta; dx = k1*dy_eff + k2*(x-mean) + k3, for the 8-channel vector cv, by
// 256 threads. The vector's partials are 64 B per row block (16 floats); thread t reads float4 q =
// t & 3 of row blocks t >> 2, t >> 2 + 64, ..., so one wave load covers 16 whole 64-B segments
// (a row-per-lane layout would fetch every line 16 times over when the loads bypass L1). The 4
// sums per lane reduce over the lanes sharing q (4 xor steps), then over the 4 waves through LDS
// (red: 64 floats), in a fixed order. SC1: the partials were handed over inside this launch (the
// folded form) and every read of them is an sc1 load (16-B buffer loads); the additions are the
// same in the same order, so both forms give bitwise the same results.
template <bool SC1>
__device__ __forceinline__ void bwd_finalize_vec(const float* __restrict__ part, int rblocks, int C, int cv,
                                                 const BwdFin& f, float* red) {
  const int tid = threadIdx.x + blockDim.x * threadIdx.y, lane = tid & 63, wid = tid >> 6;
  const int q = tid & 3, rr = tid >> 2;
  // the per-channel parameters are loaded up front, under the partials' loads (not a second
  // dependent memory round trip after the reduction: the launch is latency-bound)
  const int c = cv * 8 + (tid & 7);
  float inv = 0.f, g = 1.f, fm = 0.f, ssc = 0.f, ssh = 0.f;
  if (tid < 8) {
    inv = f.invstd[c];
    if (f.weight) g = ld_w(f.weight, f.wdt, c);
    if (f.fold_mean) fm = f.fold_mean[c];
    if (f.ss_copy) {
      ssc = f.ss_copy[c];
      ssh = f.ss_copy[C + c];
    }
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t rstride = (int64_t)C * 2;           // floats per row block
  const int64_t off0 = (int64_t)cv * 16 + q * 4;     // this thread's float4 within a row block
  if (SC1) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(part), (short)0,
                                                        (int)(rblocks * rstride * 4), 0x00020000);
#pragma unroll 8
    for (int b = rr; b < rblocks; b += 64) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)((b * rstride + off0) * 4), 0, 16);  // sc1
      acc[0] += __uint_as_float(v[0]);
      acc[1] += __uint_as_float(v[1]);
      acc[2] += __uint_as_float(v[2]);
      acc[3] += __uint_as_float(v[3]);
    }
  } else {
#pragma unroll 8
    for (int b = rr; b < rblocks; b += 64) {
      const float4 v = *reinterpret_cast<const float4*>(part + b * rstride + off0);
      acc[0] += v.x;
      acc[1] += v.y;
      acc[2] += v.z;
      acc[3] += v.w;
    }
  }
#pragma unroll
  for (int o = 4; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wid * 16 + lane * 4 + k] = acc[k];
  }
  __syncthreads();
  if (tid < 8) {
    const float sd = (red[2 * tid] + red[16 + 2 * tid]) + (red[32 + 2 * tid] + red[48 + 2 * tid]);
    const float sdx = (red[2 * tid + 1] + red[16 + 2 * tid + 1]) + (red[32 + 2 * tid + 1] + red[48 + 2 * tid + 1]);
    if (f.dweight) st_w(f.dweight, f.wdt, c, sdx * inv);
    if (f.dbias) st_w(f.dbias, f.wdt, c, sd);
    const float invM = 1.f / (float)f.M;
    float* coef = f.coef;
    coef[c] = g * inv;                                   // k1
    coef[C + c] = -g * inv * inv * inv * sdx * invM;     // k2
    coef[2 * C + c] = -g * inv * sd * invM;              // k3
    // fold_mean: dx = k1·g + k2·x + (k3 - k2·mean), the form a consumer GEMM prologue applies
    if (f.fold_mean) coef[2 * C + c] -= coef[C + c] * fm;
    // ss_copy: rows 3-4 carry the forward scale / shift (the consumer recomputes the ReLU mask)
    if (f.ss_copy) {
      coef[3 * C + c] = ssc;
      coef[4 * C + c] = ssh;
    }
  }
}

// The separate finalize: one 256-thread block per 8-channel vector.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int rblocks, int C,
                                                              BwdFin f) {
  __shared__ float red[64];
  bwd_finalize_vec<false>(part, rblocks, C, blockIdx.x, f, red);
}

// ---------------------------------------------------------------- backward reduce
// part layout [rblocks][C][2] = (sum dy_eff, sum dy_eff*(x-mean))
// MASK: 0 = no ReLU, 1 = ReLU mask from the saved output y, 2 = ReLU mask recomputed from x
// (x*scale+shift > 0, exact for BN+ReLU without residual; saves reading y)
// 3 = ReLU mask from the forward's bit mask (1 byte per 8 channels).
// DUAL: the output had two consumers whose gradients arrive separately (dy + dy2 summed here,
// in registers, instead of by an autograd add kernel).
// WG: also store the effective gradient g = mask*(dy [+ dy2]) — it IS d(residual) — so the
// elementwise pass reads g and x only (residual BN backward: 10 -> ~7 activation passes).
template <typename T, int MASK, bool DUAL, bool WG>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                               const T* __restrict__ x, const T* __restrict__ y,
                                                               const uint8_t* __restrict__ mbits,
                                                               T* __restrict__ gout,
                                                               int64_t M, int C, int64_t rows_per,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ ss,
                                                               float* __restrict__ part, BwdFin fin) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int c0 = (blockIdx.x * TX + tx) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = min(M, r0 + rows_per);
  float mu[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j];
    if (MASK == 2) {
      sc[j] = ss[c0 + j];
      sh[j] = ss[C + c0 + j];
    }
  }
  float sd[8] = {0}, sdx[8] = {0};
  // one row: loads (dy [+ dy2], x, and the mask source) into g / a / o / b, then the mask, the
  // optional store and the sums; rows go in batches of RB with every batch's loads issued first
  // (the layer-2..4 shapes ran at 2.3-3.4 TB/s with two rows in flight per thread)
  auto ld_row = [&](int64_t r, float (&g)[8], float (&a)[8], float (&o)[8], uint32_t& b) {
    Vec8<T>::ld(dy + r * C + c0, g);
    if (DUAL) {
      float g2[8];
      Vec8<T>::ld(dy2 + r * C + c0, g2);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] += g2[j];
    }
    Vec8<T>::ld(x + r * C + c0, a);
    if (MASK == 1) Vec8<T>::ld(y + r * C + c0, o);
    if (MASK == 3) b = mbits[(r * C + c0) >> 3];
  };
  auto use_row = [&](int64_t r, float (&g)[8], const float (&a)[8], const float (&o)[8], uint32_t b) {
    if (MASK == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = o[j] > 0.f ? g[j] : 0.f;
    } else if (MASK == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(a[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    } else if (MASK == 3) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = ((b >> j) & 1u) ? g[j] : 0.f;
    }
    if (WG) {
      if (XDDP_BN_NT) dev::st8_stream(gout + r * C + c0, g); else Vec8<T>::st(gout + r * C + c0, g);
      Vec8<T>::rt(g);  // the elementwise pass sees g at storage precision: keep the sums consistent
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sd[j] += g[j];
      sdx[j] = fmaf(g[j], a[j] - mu[j], sdx[j]);
    }
  };
  constexpr int RB = XDDP_BN_RED_ROWS;
  int64_t r = r0 + ty;
  for (; r + (RB - 1) * TY < r1; r += RB * TY) {
    float g[RB][8], a[RB][8], o[RB][8];
    uint32_t b[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) ld_row(r + i * TY, g[i], a[i], o[i], b[i]);
#pragma unroll
    for (int i = 0; i < RB; ++i) use_row(r + i * TY, g[i], a[i], o[i], b[i]);
  }
  for (; r < r1; r += TY) {
    float g[8], a[8], o[8];
    uint32_t b = 0;
    ld_row(r, g, a, o, b);
    use_row(r, g, a, o, b);
  }
  float* my = lds + ((ty * TX + tx) * 8) * 2;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    my[j * 2] = sd[j];
    my[j * 2 + 1] = sdx[j];
  }
  __syncthreads();
  for (int stride = TY / 2; stride > 0; stride >>= 1) {
    if (ty < stride) {
      const float* o = lds + (((ty + stride) * TX + tx) * 8) * 2;
#pragma unroll
      for (int j = 0; j < 16; ++j) my[j] += o[j];
    }
    __syncthreads();
  }
  if (ty == 0) {
    float* dst = part + ((int64_t)blockIdx.y * C + c0) * 2;
    if (fin.slot >= 0) {
      float v[16];  // (all LDS reads first: an atomic store between them would serialize each)
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = my[j];
#pragma unroll
      for (int j = 0; j < 16; ++j) dev::st_sc1(dst + j, v[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) dst[j] = my[j];
    }
  }
  if (fin.slot < 0 || fin.dbg == 1) return;
  // the finalize, folded into the last arrivals of this channel group: fin.S reducer blocks, each
  // finalizing every fin.S-th of the group's TX channel vectors (dev::tail_arrive)
  const int rank = dev::tail_arrive(g_bn_tail_ctr + ((int64_t)fin.slot * kTailGroups + blockIdx.x) * 2, gridDim.y,
                                    fin.S, reinterpret_cast<int*>(lds), &g_bn_tail_timeout);
  if (rank < 0 || fin.dbg == 3) return;
  for (int v = rank; v < TX; v += fin.S) {
    bwd_finalize_vec<true>(part, gridDim.y, C, blockIdx.x * TX + v, fin, lds + 64);
    __syncthreads();  // (red is rewritten by the next vector)
  }
}

template <typename T, int MASK, bool DRES, bool DUAL>
__global__ __launch_bounds__(kBlock) void bn_bwd_elem_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                             const T* __restrict__ x,
                                                             const T* __restrict__ y,
                                                             const uint8_t* __restrict__ mbits, T* __restrict__ dx,
                                                             T* __restrict__ dres, int64_t nvec, int C,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ coef,
                                                             const float* __restrict__ ss) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cstep = (int)((stride * 8) % C);
  int c0 = (int)((v0 * 8) % C);
  for (int64_t v = v0; v < nvec; v += stride, c0 = (c0 + cstep >= C) ? c0 + cstep - C : c0 + cstep) {
    const int64_t e = v * 8;
    float g[8], a[8];
    Vec8<T>::ld(dy + e, g);
    if (DUAL) {
      float g2[8];
      Vec8<T>::ld(dy2 + e, g2);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] += g2[j];
    }
    Vec8<T>::ld(x + e, a);
    if (MASK == 1) {
      float o[8];
      Vec8<T>::ld(y + e, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = o[j] > 0.f ? g[j] : 0.f;
    } else if (MASK == 2) {
      float sc[8], sh[8];
      Vec8<float>::ld(ss + c0, sc);
      Vec8<float>::ld(ss + C + c0, sh);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(a[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    } else if (MASK == 3) {
      const uint32_t b = mbits[v];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = ((b >> j) & 1u) ? g[j] : 0.f;
    }
    if (DRES) { if (XDDP_BN_NT) dev::st8_stream(dres + e, g); else Vec8<T>::st(dres + e, g); }
    // per-channel coefficients as 16-B vector loads (L1/L2 resident; C*16 B per array)
    float k1[8], k2[8], k3[8], mu[8], out[8];
    Vec8<float>::ld(coef + c0, k1);
    Vec8<float>::ld(coef + C + c0, k2);
    Vec8<float>::ld(coef + 2 * C + c0, k3);
    Vec8<float>::ld(mean + c0, mu);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = fmaf(k1[j], g[j], fmaf(k2[j], a[j] - mu[j], k3[j]));
    if (XDDP_BN_NT) dev::st8_stream(dx + e, out); else Vec8<T>::st(dx + e, out);
  }
}

template <typename F>
void dispatch_act(at::ScalarType st, F&& f) {
  switch (st) {
    case at::kBFloat16: f(bf16_t{}); break;
    case at::kFloat: f(float{}); break;
    case at::kHalf: f(f16_t{}); break;
    default: TORCH_CHECK(false, "xddp batch_norm: unsupported activation dtype ", st);
  }
}

template <typename F>
void dispatch_w(at::ScalarType st, F&& f) {
  switch (st) {
    case at::kBFloat16: f(bf16_t{}); break;
    case at::kFloat: f(float{}); break;
    case at::kHalf: f(f16_t{}); break;
    default: TORCH_CHECK(false, "xddp batch_norm: unsupported weight dtype ", st);
  }
}

int elem_grid(int64_t nvec) { return (int)std::min<int64_t>((nvec + kBlock - 1) / kBlock, 256 * 16); }

void check_nhwc(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "xddp batch_norm expects a 4-D device tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "xddp batch_norm expects channels_last input");
  TORCH_CHECK(x.size(1) % 8 == 0, "xddp batch_norm needs C % 8 == 0");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, "xddp batch_norm needs 16-B aligned data");
}

template <typename W>
W* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<W*>(t->data_ptr()) : nullptr;
}

int wdt_code(at::ScalarType st) {
  TORCH_CHECK(st == at::kFloat || st == at::kBFloat16 || st == at::kHalf, "xddp batch_norm: unsupported weight dtype ", st);
  return st == at::kBFloat16 ? 1 : (st == at::kHalf ? 2 : 0);
}

// XDDP_BN_TAIL=1 runs the BN-backward finalize in the reduce kernel's last arrivals (BwdFin,
// dev::tail_arrive) instead of a separate launch. Opt-in: measured slower (profiles/
// r6_bn_finalize_fold.txt): the arrival fan-in and the reducers' poll cost 3.5-6 us per launch and
// the reduction after the last arrival 2-3 us, against 2.6-3.3 us for the whole separate finalize
// (one launch, coalesced 16-B partial reads); the headline step lost 1.1 %.
bool bn_tail_enabled() {
  const char* e = std::getenv("XDDP_BN_TAIL");  // (read per call: tests switch it in-process)
  return e && e[0] == '1';
}

int next_tail_slot() {
  static std::atomic<unsigned> n{0};
  return (int)(n.fetch_add(1, std::memory_order_relaxed) % kTailSlots);
}

}  // namespace

// Whether any folded finalize hit its spin bound (a producer never arrived) since the last call;
// clears the flag. Device-synchronizing: for tests and diagnostics.
bool bn_tail_timeouts(int64_t device) {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  unsigned v = 0, z = 0;
  XDDP_HIP_CHECK(hipDeviceSynchronize());
  XDDP_HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_bn_tail_timeout), sizeof(v), 0, hipMemcpyDeviceToHost));
  XDDP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_bn_tail_timeout), &z, sizeof(z), 0, hipMemcpyHostToDevice));
  return v != 0;
}

// returns (y, mean, invstd)
std::vector<at::Tensor> bn_forward(const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var,
                                   const c10::optional<at::Tensor>& num_batches_tracked, bool training,
                                   double momentum, bool cumulative, double eps,
                                   const c10::optional<at::Tensor>& residual, bool relu, bool save_mask) {
  check_nhwc(x);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), Wd = x.size(3);
  const int64_t M = N * H * Wd;
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  auto fopt = x.options().dtype(at::kFloat);
  auto y = at::empty_like(x, at::MemoryFormat::ChannelsLast);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ss = at::empty({2, C}, fopt);
  const bool has_res = residual.has_value() && residual->defined();
  at::Tensor mask_bits = (relu && save_mask) ? at::empty({N * H * Wd * C / 8}, x.options().dtype(at::kByte))
                                             : at::Tensor();
  if (has_res) {
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type() &&
                    residual->is_contiguous(at::MemoryFormat::ChannelsLast),
                "fused residual must match x (shape, dtype, channels_last)");
  }
  const auto wdt = weight.has_value() && weight->defined() ? weight->scalar_type()
                   : (running_mean.has_value() && running_mean->defined() ? running_mean->scalar_type() : at::kFloat);
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    dispatch_w(wdt, [&](auto tag_w) {
      using W = decltype(tag_w);
      const int fin_grid = (int)((C + kBlock - 1) / kBlock);
      if (training) {
        TORCH_CHECK(M > 0, "batch_norm on empty input");
        Geo g = make_geo(M, (int)C);
        auto part = at::empty({(int64_t)g.rblocks, C, 2}, fopt);
        const size_t lds = (size_t)kBlock * 16 * sizeof(float);
        hipLaunchKernelGGL((bn_stats_kernel<T>), dim3(g.cblocks, g.rblocks), dim3(g.tx, g.ty), lds, stream,
                           reinterpret_cast<const T*>(x.data_ptr()), M, (int)C, g.rows_per, part.data_ptr<float>());
        XDDP_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL((bn_stats_finalize_kernel<T, W>), dim3(C / 8), dim3(64), 0, stream,
                           part.data_ptr<float>(), g.rblocks, (int)C, M, reinterpret_cast<const T*>(x.data_ptr()),
                           opt_ptr<const W>(weight),
                           opt_ptr<const W>(bias), opt_ptr<W>(running_mean), opt_ptr<W>(running_var),
                           (num_batches_tracked.has_value() && num_batches_tracked->defined())
                               ? num_batches_tracked->data_ptr<int64_t>() : nullptr,
                           (float)momentum, cumulative, (float)eps, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                           ss.data_ptr<float>(), ss.data_ptr<float>() + C);
        XDDP_HIP_CHECK(hipGetLastError());
      } else {
        TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "eval batch_norm needs running stats");
        hipLaunchKernelGGL((bn_eval_coef_kernel<W>), dim3(fin_grid), dim3(kBlock), 0, stream, (int)C,
                           opt_ptr<const W>(weight), opt_ptr<const W>(bias), opt_ptr<const W>(running_mean),
                           opt_ptr<const W>(running_var), (float)eps, ss.data_ptr<float>(), ss.data_ptr<float>() + C);
        XDDP_HIP_CHECK(hipGetLastError());
      }
      const int64_t nvec = M * C / 8;
      const T* res = has_res ? reinterpret_cast<const T*>(residual->data_ptr()) : nullptr;
      int64_t* nbt_inc = (training && num_batches_tracked.has_value() && num_batches_tracked->defined())
                             ? num_batches_tracked->data_ptr<int64_t>() : nullptr;
      uint8_t* mb = mask_bits.defined() ? mask_bits.data_ptr<uint8_t>() : nullptr;
      auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(elem_grid(nvec)), dim3(kBlock), 0, stream,
                           reinterpret_cast<const T*>(x.data_ptr()), res, reinterpret_cast<T*>(y.data_ptr()), nvec,
                           (int)C, ss.data_ptr<float>(), ss.data_ptr<float>() + C, nbt_inc, mb, nullptr, nullptr);
      };
      if (has_res) { if (relu) launch(bn_apply_kernel<T, true, true>); else launch(bn_apply_kernel<T, true, false>); }
      else { if (relu) launch(bn_apply_kernel<T, false, true>); else launch(bn_apply_kernel<T, false, false>); }
      XDDP_HIP_CHECK(hipGetLastError());
    });
  });
  return {y, mean, invstd, ss, mask_bits};
}

// Per-channel (count, mean, M2) of an NHWC activation as float [3, C] — one rank's share of a
// SyncBatchNorm's statistics (merged across ranks by bn_stats_from_partials).
at::Tensor bn_moments(const at::Tensor& x) {
  check_nhwc(x);
  const int64_t C = x.size(1), M = x.size(0) * x.size(2) * x.size(3);
  TORCH_CHECK(M > 0, "bn_moments on empty input");
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  auto fopt = x.options().dtype(at::kFloat);
  auto out = at::empty({3, C}, fopt);
  Geo g = make_geo(M, (int)C);
  auto part = at::empty({(int64_t)g.rblocks, C, 2}, fopt);
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    const size_t lds = (size_t)kBlock * 16 * sizeof(float);
    hipLaunchKernelGGL((bn_stats_kernel<T>), dim3(g.cblocks, g.rblocks), dim3(g.tx, g.ty), lds, stream,
                       reinterpret_cast<const T*>(x.data_ptr()), M, (int)C, g.rows_per, part.data_ptr<float>());
    XDDP_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL((bn_stats_finalize_kernel<T, float, true>), dim3(C / 8), dim3(64), 0, stream,
                       part.data_ptr<float>(), g.rblocks, (int)C, M, reinterpret_cast<const T*>(x.data_ptr()), nullptr,
                       nullptr, nullptr, nullptr, nullptr, 0.f, false, 0.f, out.data_ptr<float>(), nullptr, nullptr,
                       nullptr);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return out;
}

// Per-row-block BN-backward partial sums (sum dy, sum dy·(x - mean)) as float [blocks, C, 2] (the
// layout bn_backward_from_partials reads): the local half of a SyncBatchNorm backward.
at::Tensor bn_grad_partials(const at::Tensor& dy_in, const at::Tensor& x, const at::Tensor& mean) {
  check_nhwc(x);
  auto dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  TORCH_CHECK(mean.is_cuda() && mean.scalar_type() == at::kFloat && mean.numel() == x.size(1), "mean: float [C]");
  const int64_t C = x.size(1), M = x.size(0) * x.size(2) * x.size(3);
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  Geo g = make_geo(M, (int)C);
  auto part = at::empty({(int64_t)g.rblocks, C, 2}, x.options().dtype(at::kFloat));
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    const size_t lds = (size_t)kBlock * 8 * 2 * sizeof(float);
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, 0, false, false>), dim3(g.cblocks, g.rblocks), dim3(g.tx, g.ty), lds,
                       stream, reinterpret_cast<const T*>(dy.data_ptr()), nullptr,
                       reinterpret_cast<const T*>(x.data_ptr()), nullptr, nullptr, nullptr, M, (int)C, g.rows_per,
                       mean.data_ptr<float>(), nullptr, part.data_ptr<float>(), BwdFin{-1});
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return part;
}

// Apply pass only, with coefficients computed elsewhere (e.g. from a conv epilogue's partial
// statistics): y = [relu](x*scale + shift [+ residual]); optional ReLU bit mask; optional
// num_batches_tracked += 1. Returns (y, mask_bits).
std::vector<at::Tensor> bn_apply(const at::Tensor& x, const at::Tensor& ss, const c10::optional<at::Tensor>& residual,
                                 bool relu, bool save_mask, const c10::optional<at::Tensor>& num_batches_tracked,
                                 const c10::optional<at::Tensor>& residual_ss,
                                 const c10::optional<at::Tensor>& residual_nbt, const c10::optional<at::Tensor>& out,
                                 const c10::optional<at::Tensor>& out_bits) {
  check_nhwc(x);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), Wd = x.size(3);
  TORCH_CHECK(ss.is_cuda() && ss.scalar_type() == at::kFloat && ss.numel() == 2 * C && ss.is_contiguous(),
              "bn_apply: scale/shift must be float [2, C]");
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res)
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type() &&
                    residual->is_contiguous(at::MemoryFormat::ChannelsLast),
                "fused residual must match x (shape, dtype, channels_last)");
  const bool has_rss = residual_ss.has_value() && residual_ss->defined();
  if (has_rss)
    TORCH_CHECK(has_res && residual_ss->is_cuda() && residual_ss->scalar_type() == at::kFloat &&
                    residual_ss->numel() == 2 * C && residual_ss->is_contiguous(),
                "bn_apply: residual scale/shift must be float [2, C] with a residual");
  // out / out_bits: write into given tensors (a deferred apply whose output tensor already exists)
  const bool has_out = out.has_value() && out->defined();
  if (has_out)
    TORCH_CHECK(out->sizes() == x.sizes() && out->scalar_type() == x.scalar_type() &&
                    out->is_contiguous(at::MemoryFormat::ChannelsLast),
                "bn_apply: out must match x (shape, dtype, channels_last)");
  auto y = has_out ? *out : at::empty_like(x, at::MemoryFormat::ChannelsLast);
  const bool has_obits = out_bits.has_value() && out_bits->defined();
  if (has_obits)
    TORCH_CHECK(relu && save_mask && out_bits->scalar_type() == at::kByte && out_bits->numel() * 8 == x.numel(),
                "bn_apply: out_bits must be uint8 with one byte per 8 elements (relu, save_mask)");
  at::Tensor mask_bits = has_obits ? *out_bits
                         : (relu && save_mask) ? at::empty({N * H * Wd * C / 8}, x.options().dtype(at::kByte))
                                               : at::Tensor();
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int64_t nvec = N * H * Wd * C / 8;
  int64_t* nbt_inc = (num_batches_tracked.has_value() && num_batches_tracked->defined())
                         ? num_batches_tracked->data_ptr<int64_t>() : nullptr;
  int64_t* nbt_inc2 = (residual_nbt.has_value() && residual_nbt->defined()) ? residual_nbt->data_ptr<int64_t>()
                                                                             : nullptr;
  const float* rss = has_rss ? residual_ss->data_ptr<float>() : nullptr;
  uint8_t* mb = mask_bits.defined() ? mask_bits.data_ptr<uint8_t>() : nullptr;
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    const T* res = has_res ? reinterpret_cast<const T*>(residual->data_ptr()) : nullptr;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(elem_grid(nvec)), dim3(kBlock), 0, stream,
                         reinterpret_cast<const T*>(x.data_ptr()), res, reinterpret_cast<T*>(y.data_ptr()), nvec,
                         (int)C, ss.data_ptr<float>(), ss.data_ptr<float>() + C, nbt_inc, mb, rss, nbt_inc2);
    };
    if (has_res) { if (relu) launch(bn_apply_kernel<T, true, true>); else launch(bn_apply_kernel<T, true, false>); }
    else { if (relu) launch(bn_apply_kernel<T, false, true>); else launch(bn_apply_kernel<T, false, false>); }
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return {y, mask_bits};
}

// returns (dx, dweight, dbias, dresidual)
std::vector<at::Tensor> bn_backward(const at::Tensor& dy_in, const at::Tensor& x, const c10::optional<at::Tensor>& y,
                                    const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                                    const at::Tensor& invstd, const c10::optional<at::Tensor>& ss, bool relu,
                                    bool need_dres, bool need_dweight, const c10::optional<at::Tensor>& dy2_in,
                                    const c10::optional<at::Tensor>& mask_bits, bool coef_only) {
  check_nhwc(x);
  auto dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const bool dual = dy2_in.has_value() && dy2_in->defined();
  at::Tensor dy2 = dual ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast) : at::Tensor();
  if (dual) TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == x.scalar_type(), "dy2 must match x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  const bool have_y = y.has_value() && y->defined();
  const bool have_ss = ss.has_value() && ss->defined();
  const bool have_bits = mask_bits.has_value() && mask_bits->defined();
  if (relu) TORCH_CHECK(have_bits || have_y || have_ss, "relu backward needs the mask bits, the output or scale/shift");
  const int mask = relu ? (have_bits ? 3 : (have_y ? 1 : 2)) : 0;
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), Wd = x.size(3);
  const int64_t M = N * H * Wd;
  if (mask == 3) TORCH_CHECK(mask_bits->numel() * 8 == M * C && mask_bits->scalar_type() == at::kByte,
                             "mask bits must be uint8[M*C/8]");
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  auto fopt = x.options().dtype(at::kFloat);
  // coef_only: skip the elementwise pass and return the per-channel (k1, k2, k3 - k2·mean) [3, C]
  // in dx's slot; the gradient k1·g + k2·x + k3' is formed by the consumer (conv GEMM prologue),
  // with g = dres (written here) or, without ReLU/second gradient, dy itself
  // with a ReLU whose mask is recomputed (scale/shift given, no residual gradient) the consumer
  // also needs (scale, shift): coef is then [5, C] = (k1, k2, k3', scale, shift)
  const bool coef_mask = coef_only && !need_dres && relu && !dual && !have_bits && !have_y && have_ss;
  if (coef_only) TORCH_CHECK(need_dres || (!relu && !dual) || coef_mask, "bn_backward: coef_only needs g materialized");
  auto dx = coef_only ? at::Tensor() : at::empty_like(x, at::MemoryFormat::ChannelsLast);
  at::Tensor dres = need_dres ? at::empty_like(x, at::MemoryFormat::ChannelsLast) : at::Tensor();
  const bool has_w = weight.has_value() && weight->defined();
  const auto wdt = has_w ? weight->scalar_type() : at::kFloat;
  at::Tensor dw = (has_w && need_dweight) ? at::empty({C}, weight->options()) : at::Tensor();
  at::Tensor db = (has_w && need_dweight) ? at::empty({C}, weight->options()) : at::Tensor();
  auto coef = at::empty({coef_mask ? 5 : 3, C}, fopt);
  Geo g = make_geo(M, (int)C);
  auto part = at::empty({(int64_t)g.rblocks, C, 2}, fopt);
  // need_dres: the reduce pass writes g = mask*(dy+dy2) into dres; the elementwise pass then
  // reads (g, x) with no mask and no second gradient
  const bool wg = need_dres;
  // the finalize runs in the reduce kernel's last arrivals when the grid allows it (the whole
  // grid resident: ~512 blocks; at most kTailGroups channel groups)
  const bool tail = bn_tail_enabled() && g.cblocks <= kTailGroups && (int64_t)g.cblocks * g.rblocks <= 1024;
  BwdFin fin{tail ? next_tail_slot() : -1, std::min(g.tx, g.rblocks), wdt_code(wdt), M,
             has_w ? weight->data_ptr() : nullptr, invstd.data_ptr<float>(), dw.defined() ? dw.data_ptr() : nullptr,
             db.defined() ? db.data_ptr() : nullptr, coef.data_ptr<float>(), coef_only ? mean.data_ptr<float>() : nullptr,
             coef_only && coef_mask ? ss->data_ptr<float>() : nullptr};
  if (const char* e = std::getenv("XDDP_BN_TAIL_DBG")) fin.dbg = std::atoi(e);
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    {
      const T* yp = mask == 1 ? reinterpret_cast<const T*>(y->data_ptr()) : nullptr;
      const float* ssp = mask == 2 ? ss->data_ptr<float>() : nullptr;
      const uint8_t* mbp = mask == 3 ? mask_bits->data_ptr<uint8_t>() : nullptr;
      const size_t lds = (size_t)kBlock * 8 * 2 * sizeof(float);
      const T* d2p = dual ? reinterpret_cast<const T*>(dy2.data_ptr()) : nullptr;
      T* gp = wg ? reinterpret_cast<T*>(dres.data_ptr()) : nullptr;
      auto launch_red = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(g.cblocks, g.rblocks), dim3(g.tx, g.ty), lds, stream,
                           reinterpret_cast<const T*>(dy.data_ptr()), d2p, reinterpret_cast<const T*>(x.data_ptr()),
                           yp, mbp, gp, M, (int)C, g.rows_per, mean.data_ptr<float>(), ssp, part.data_ptr<float>(),
                           fin);
      };
#define XDDP_BN_RED(MK)                                                                           \
  if (dual) { if (wg) launch_red(bn_bwd_reduce_kernel<T, MK, true, true>);                        \
              else launch_red(bn_bwd_reduce_kernel<T, MK, true, false>); }                        \
  else { if (wg) launch_red(bn_bwd_reduce_kernel<T, MK, false, true>);                            \
         else launch_red(bn_bwd_reduce_kernel<T, MK, false, false>); }
      if (mask == 1) { XDDP_BN_RED(1) }
      else if (mask == 2) { XDDP_BN_RED(2) }
      else if (mask == 3) { XDDP_BN_RED(3) }
      else { XDDP_BN_RED(0) }
#undef XDDP_BN_RED
      XDDP_HIP_CHECK(hipGetLastError());
      if (!tail) {
        hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C / 8), dim3(256), 0, stream, part.data_ptr<float>(),
                           g.rblocks, (int)C, fin);
        XDDP_HIP_CHECK(hipGetLastError());
      }
      const int64_t nvec = M * C / 8;
      if (coef_only) {  // nothing more: the consumer applies the coefficients
      } else if (wg) {
        hipLaunchKernelGGL((bn_bwd_elem_kernel<T, 0, false, false>), dim3(elem_grid(nvec)), dim3(kBlock), 0, stream,
                           reinterpret_cast<const T*>(dres.data_ptr()), nullptr,
                           reinterpret_cast<const T*>(x.data_ptr()), nullptr, nullptr,
                           reinterpret_cast<T*>(dx.data_ptr()), nullptr, nvec, (int)C, mean.data_ptr<float>(),
                           coef.data_ptr<float>(), nullptr);
      } else {
        auto launch = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(elem_grid(nvec)), dim3(kBlock), 0, stream,
                             reinterpret_cast<const T*>(dy.data_ptr()), d2p, reinterpret_cast<const T*>(x.data_ptr()),
                             yp, mbp, reinterpret_cast<T*>(dx.data_ptr()), nullptr, nvec, (int)C,
                             mean.data_ptr<float>(), coef.data_ptr<float>(), ssp);
        };
#define XDDP_BN_ELEM(MK) \
  if (dual) launch(bn_bwd_elem_kernel<T, MK, false, true>); else launch(bn_bwd_elem_kernel<T, MK, false, false>)
        if (mask == 1) { XDDP_BN_ELEM(1); }
        else if (mask == 2) { XDDP_BN_ELEM(2); }
        else if (mask == 3) { XDDP_BN_ELEM(3); }
        else { XDDP_BN_ELEM(0); }
#undef XDDP_BN_ELEM
      }
      XDDP_HIP_CHECK(hipGetLastError());
    }
  });
  return {coef_only ? coef : dx, dw, db, dres};
}

// BN backward coefficients from partials produced elsewhere (the EPI epilogue of conv_gemm.hip):
// part [groups, C, 2] = (sum g, sum g·(x - mean)) -> (coef [3, C] = (k1, k2, k3 - k2·mean), dw, db).
std::vector<at::Tensor> bn_backward_from_partials(const at::Tensor& part, int64_t M,
                                                  const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                                                  const at::Tensor& invstd, bool need_dweight, bool fold_mean) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(2) == 2 && part.scalar_type() == at::kFloat &&
                  part.is_contiguous(),
              "bn_backward_from_partials: partials must be float [groups, C, 2]");
  const int64_t C = part.size(1);
  TORCH_CHECK(C % 8 == 0 && mean.numel() == C && invstd.numel() == C, "bn_backward_from_partials: bad channel count");
  auto stream = c10::hip::getCurrentHIPStream(part.device().index()).stream();
  auto coef = at::empty({3, C}, part.options());
  const bool has_w = weight.has_value() && weight->defined();
  const auto wdt = has_w ? weight->scalar_type() : at::kFloat;
  at::Tensor dw = (has_w && need_dweight) ? at::empty({C}, weight->options()) : at::Tensor();
  at::Tensor db = (has_w && need_dweight) ? at::empty({C}, weight->options()) : at::Tensor();
  const BwdFin fin{-1, 0, wdt_code(wdt), M, has_w ? weight->data_ptr() : nullptr, invstd.data_ptr<float>(),
                   dw.defined() ? dw.data_ptr() : nullptr, db.defined() ? db.data_ptr() : nullptr, coef.data_ptr<float>(),
                   fold_mean ? mean.data_ptr<float>() : nullptr, nullptr};
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C / 8), dim3(256), 0, stream, part.data_ptr<float>(),
                     (int)part.size(0), (int)C, fin);
  XDDP_HIP_CHECK(hipGetLastError());
  return {coef, dw, db};
}

at::Tensor bn_backward_elem(const at::Tensor& g_in, const at::Tensor& x, const at::Tensor& mean, const at::Tensor& coef) {
  check_nhwc(x);
  auto g = g_in.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(g.sizes() == x.sizes() && g.scalar_type() == x.scalar_type(), "bn_backward_elem: g must match x");
  const int64_t C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.numel() >= 3 * C && coef.is_contiguous() &&
                  mean.scalar_type() == at::kFloat && mean.numel() == C,
              "bn_backward_elem: float coef [3, C] and mean [C] expected");
  auto dx = at::empty_like(x, at::MemoryFormat::ChannelsLast);
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int64_t nvec = M * C / 8;
  dispatch_act(x.scalar_type(), [&](auto tag_t) {
    using T = decltype(tag_t);
    hipLaunchKernelGGL((bn_bwd_elem_kernel<T, 0, false, false>), dim3(elem_grid(nvec)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const T*>(g.data_ptr()), nullptr, reinterpret_cast<const T*>(x.data_ptr()),
                       nullptr, nullptr, reinterpret_cast<T*>(dx.data_ptr()), nullptr, nvec, (int)C,
                       mean.data_ptr<float>(), coef.data_ptr<float>(), nullptr);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return dx;
}

}  // namespace kernels
}  // namespace xddp
