// NHWC max-pool (ResNet stem 3x3/s2/p1) on gfx950.
//
// Reference hot path: at::native max_pool forward/backward_nhwc keep an
// int64 index per output element and the backward took 634 us for [256,64,112,112] on
// MI355X (profiles/). Here the forward stores the argmax *within the window* as one byte
// (k*k <= 255) — 8x less index traffic — and the backward is a gather: each lane owns 8
// channels of one input pixel, visits the <= ceil(k/s)^2 windows covering it and sums the
// dy of windows whose argmax is this pixel. No atomics, no zero-fill pass, 16-B accesses.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

using dev::bf16_t;
using dev::f16_t;
using dev::Vec8;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                          int OH, int OW, int k, int s, int p) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * OH * OW * cv;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * 8;
    int64_t r = t / cv;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float m[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      am[j] = 0;
    }
    const int h0 = oh * s - p, w0 = ow * s - p;
    for (int kh = 0; kh < k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= W) continue;
        float v[8];
        Vec8<T>::ld(x + (((int64_t)n * H + h) * W + w) * C + c0, v);
        const int pos = kh * k + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v[j] > m[j] || isnan(v[j])) {  // first max wins; NaN propagates (torch semantics)
            m[j] = v[j];
            am[j] = pos;
          }
        }
      }
    }
    const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
    Vec8<T>::st(y + o, m);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (uint64_t)(am[j] & 0xff) << (8 * j);
    *reinterpret_cast<uint64_t*>(idx + o) = packed;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                          const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                          int OW, int k, int s, int p) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * 8;
    int64_t r = t / cv;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    // windows covering h: oh*s - p <= h <= oh*s - p + k - 1
    const int oh_lo = max(0, (h + p - k + s) / s), oh_hi = min(OH - 1, (h + p) / s);
    const int ow_lo = max(0, (w + p - k + s) / s), ow_hi = min(OW - 1, (w + p) / s);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = h - (oh * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = w - (ow * s - p);
        if (kw < 0 || kw >= k) continue;
        const int pos = kh * k + kw;
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        float g[8];
        Vec8<T>::ld(dy + o, g);
        if (dy2) {  // second consumer of the pooled output (dual-output ResNet stem)
          float g2[8];
          Vec8<T>::ld(dy2 + o, g2);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] += g2[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((int)((packed >> (8 * j)) & 0xff) == pos) acc[j] += g[j];
      }
    }
    Vec8<T>::st(dx + (((int64_t)n * H + h) * W + w) * C + c0, acc);
  }
}

// ResNet stem specialisation (k=3, s=2, p=1): one lane per 2x2 input quad (h = 2t, 2t+1;
// w = 2u, 2u+1) x 8 channels. The quad is covered by exactly the windows (t|t+1, u|u+1), so each
// window's dy/argmax is read once per quad instead of once per covered pixel (2.25x fewer gathered
// reads than the per-pixel gather above).
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2p1_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                                 const uint8_t* __restrict__ idx,
                                                                 T* __restrict__ dx, int N, int H, int W, int C,
                                                                 int OH, int OW) {
  const int cv = C / 8;
  const int QH = (H + 1) / 2, QW = (W + 1) / 2;
  const int64_t total = (int64_t)N * QH * QW * cv;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(q % cv) * 8;
    int64_t r = q / cv;
    const int u = (int)(r % QW);
    r /= QW;
    const int t = (int)(r % QH);
    const int n = (int)(r / QH);
    float acc[4][8];  // [h1*2 + w1][channel]
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int oh = t + dh, ow = u + dw;
        if (oh >= OH || ow >= OW) continue;
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        float g[8];
        Vec8<T>::ld(dy + o, g);
        if (dy2) {
          float g2[8];
          Vec8<T>::ld(dy2 + o, g2);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] += g2[j];
        }
        // input (2t + a, 2u + b) sits at window offset kh = 1 + a - 2*dh, kw = 1 + b - 2*dw
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int kh = 1 + a - 2 * dh, kw = 1 + b - 2 * dw;
            if (kh < 0 || kw < 0) continue;  // compile-time after unrolling
            const int pos = kh * 3 + kw;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if ((int)((packed >> (8 * j)) & 0xff) == pos) acc[a * 2 + b][j] += g[j];
          }
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * t + a, w = 2 * u + b;
        if (h < H && w < W) dev::st8_stream(dx + (((int64_t)n * H + h) * W + w) * C + c0, acc[a * 2 + b]);
      }
  }
}

// ------------------------------------------------------------------ stem: BN + ReLU + max-pool
// The ResNet stem's bn1 -> ReLU -> maxpool(3, 2, 1) without its 411 MB (bs256) normalized
// activation ever existing in HBM: the forward pools relu(y·scale + shift) straight from the conv
// output y (one read of y, pooled output + byte argmax written); the backward's two passes
// (BN-backward partial sums, then dX) rebuild the pooled gradient per 2x2 quad from (dy, argmax)
// and the ReLU mask from y, so neither the maxpool gradient nor the masked BN gradient is written.

template <typename T>
__device__ __forceinline__ float rnd(float v) {  // round to the storage precision of T
  if constexpr (__is_same(T, bf16_t)) return dev::bf16_to_f32(dev::f32_to_bf16(v));
  else if constexpr (__is_same(T, f16_t)) return dev::f16_to_f32(dev::f32_to_f16(v));
  else return v;
}

template <typename T>
__global__ __launch_bounds__(256) void stem_pool_fwd_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ y,
                                                            uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                            int OH, int OW) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * OH * OW * cv;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * 8;
    int64_t r = t / cv;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float sc[8], sh[8], m[8];
    int am[8];
    Vec8<float>::ld(scale + c0, sc);
    Vec8<float>::ld(shift + c0, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      am[j] = 0;
    }
    // branch-free window: the 9 loads are issued together (out-of-image taps read a clamped
    // in-image pixel and are masked out of the max). A strip walker that carries the shared
    // window row (6 loads per output instead of 9) measured slower: 178 vs 149 us at bs256.
    const int h0 = oh * 2 - 1, w0 = ow * 2 - 1;
    float v[9][8];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = min(max(h0 + kh, 0), H - 1), w = min(max(w0 + kw, 0), W - 1);
        Vec8<T>::ld(x + (((int64_t)n * H + h) * W + w) * C + c0, v[kh * 3 + kw]);
      }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const bool in = (unsigned)(h0 + kh) < (unsigned)H && (unsigned)(w0 + kw) < (unsigned)W;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // the value the unfused stack pools: BN + ReLU output rounded to storage precision
          const float a = rnd<T>(fmaxf(fmaf(v[kh * 3 + kw][j], sc[j], sh[j]), 0.f));
          if (in && (a > m[j] || isnan(a))) {  // first max wins; NaN propagates (torch semantics)
            m[j] = a;
            am[j] = kh * 3 + kw;
          }
        }
      }
    const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
    Vec8<T>::st(y + o, m);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (uint64_t)(am[j] & 0xff) << (8 * j);
    *reinterpret_cast<uint64_t*>(idx + o) = packed;
  }
}

// ELEM = false: per-block partials (sum g, sum g·(y - mean)) [blocks][C][2] of the masked BN
// gradient g = [y·scale + shift > 0] · maxpool_backward(dy + dy2); ELEM = true: the BN-backward
// input gradient dX = k1·g + k2·(y - mean) + k3 (coef [3, C], unfolded).
// A lane owns 8 channels of a vertical strip of 2x2 input quads (h = 2t, 2t+1; w = 2u, 2u+1) for
// t in [t0, t0 + kStrip): quad row t is covered by the pooling windows of rows t and t+1, so the
// lane walks down the strip carrying window row t+1 (argmax + dy) into the next quad row — each
// window is fetched twice (by the strips u and u-1, adjacent lanes) instead of four times by
// scattered quads, and the work of a block stays inside one XCD's L2. The lane's channel chunk
// is fixed (256 % (C / 8) == 0), so its BN sums stay in registers.
constexpr int kStrip = 14;

template <typename T>
struct Raw8 {  // 8 channel values as loaded: packed pairs for 16-bit dtypes, fp32 as is
  static constexpr bool kPacked = !__is_same(T, float);
  uint32_t w[kPacked ? 4 : 8];
  __device__ __forceinline__ void load(const T* p) {
    const dev::u32x4 a = *reinterpret_cast<const dev::u32x4*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = a[j];
    if constexpr (!kPacked) {
      const dev::u32x4 b = *reinterpret_cast<const dev::u32x4*>(p + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[4 + j] = b[j];
    }
  }
  __device__ __forceinline__ void set(const float (&v)[8]) {  // round to T
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (__is_same(T, bf16_t)) w[j] = dev::pack_bf16x2(v[2 * j], v[2 * j + 1]);
      else if constexpr (__is_same(T, f16_t)) w[j] = dev::pack_f16x2(v[2 * j], v[2 * j + 1]);
    }
    if constexpr (!kPacked) {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = __float_as_uint(v[j]);
    }
  }
  __device__ __forceinline__ float get(int j) const {
    if constexpr (__is_same(T, bf16_t)) return __uint_as_float((j & 1) ? (w[j >> 1] & 0xffff0000u) : (w[j >> 1] << 16));
    else if constexpr (__is_same(T, f16_t))
      return dev::f16_to_f32((uint16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xffffu)));
    else return __uint_as_float(w[j]);
  }
};

template <typename T>
struct PoolWin {  // two adjacent pooling windows (u, u+1) of one window row, dy + dy2 summed
  // the summed gradient is kept at storage precision (4 registers per window for 16-bit dtypes):
  // the unfused stack stores dy + dy2 in T too (autograd sums the two uses of the pool output)
  uint64_t packed[2];
  Raw8<T> g8[2];
  __device__ __forceinline__ void load(const T* dy, const T* dy2, const uint8_t* idx, int n, int oh, int u, int OH,
                                       int OW, int C, int c0) {
    const int ohc = min(oh, OH - 1);
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int64_t o = (((int64_t)n * OH + ohc) * OW + min(u + d, OW - 1)) * C + c0;
      packed[d] = *reinterpret_cast<const uint64_t*>(idx + o);
      if (dy2) {
        float g[8], g2[8];
        Vec8<T>::ld(dy + o, g);
        Vec8<T>::ld(dy2 + o, g2);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] += g2[j];
        g8[d].set(g);
      } else {
        g8[d].load(dy + o);
      }
      if (oh >= OH || u + d >= OW) packed[d] = ~0ull;  // no window: matches no position
    }
  }
  __device__ __forceinline__ float g(int d, int j) const { return g8[d].get(j); }
};

template <typename T, bool ELEM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ELEM && __is_same(T, bf16_t) ? 4 : 1)))
void stem_pool_bn_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ dy2, const uint8_t* __restrict__ idx, const T* __restrict__ y,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ coef, float* __restrict__ part, T* __restrict__ dx, int N, int H, int W, int C, int OH,
    int OW) {
  // Per-channel constants live in LDS, not in 40-48 registers per lane: the kernel streams (every
  // input read once, every output written once), so its speed is the number of waves in flight
  // (bf16 dX pass: 128 VGPRs, 4 waves per SIMD; it was 178, 2 waves). ELEM folds the mean into the
  // bias (dX = k1·g + k2·y + k3', k3' = k3 - k2·mean); each of the quad's four input pixels takes
  // its window contributions, masks and emits before the next one (one 8-wide accumulator).
  // cst rows: ELEM (scale, shift, k1, k3'), partials (scale, shift, mean); ck2 = k2 (ELEM only).
  __shared__ float cst[4][64 * 8];  // C <= 512
  __shared__ float ck2[ELEM ? 64 * 8 : 1];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    cst[0][c] = scale[c];
    cst[1][c] = shift[c];
    if (ELEM) {
      cst[2][c] = coef[c];
      cst[3][c] = fmaf(-coef[C + c], mean[c], coef[2 * C + c]);  // stem_conv_wgrad_fused: the same fma
      ck2[c] = coef[C + c];
    } else {
      cst[2][c] = mean[c];
    }
  }
  __syncthreads();
  const int cv = C / 8;
  const int QH = (H + 1) / 2, QW = (W + 1) / 2, NS = (QH + kStrip - 1) / kStrip;
  const int64_t total = (int64_t)N * NS * QW * cv;
  const int64_t q = (int64_t)dev::xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int c0 = (int)(threadIdx.x % cv) * 8;
  float s1[ELEM ? 1 : 8], s2[ELEM ? 1 : 8];
  if (!ELEM) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  }
  if (q < total) {
    int64_t r = q / cv;
    const int u = (int)(r % QW);
    r /= QW;
    const int strip = (int)(r % NS);
    const int n = (int)(r / NS);
    const int t0 = strip * kStrip, t1 = min(t0 + kStrip, QH);
    PoolWin<T> top, bot;
    top.load(dy, dy2, idx, n, t0, u, OH, OW, C, c0);
    for (int t = t0; t < t1; ++t) {
      // re-read the LDS constants each quad row (an LDS read is cheap; 40 hoisted registers are not)
      asm volatile("" ::: "memory");
      bot.load(dy, dy2, idx, n, t + 1, u, OH, OW, C, c0);
      // the quad's four y pixels are fetched together (clamped at the odd edge), outside the
      // per-pixel branches, so their latencies overlap; 16-bit values stay packed until used
      Raw8<T> yq[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int h = min(2 * t + (d >> 1), H - 1), w = min(2 * u + (d & 1), W - 1);
        yq[d].load(y + (((int64_t)n * H + h) * W + w) * C + c0);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          // input (2t + a, 2u + b) sits at offset (1 + a - 2dh, 1 + b - 2dw) of window (t + dh, u + dw)
          float acc[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
          for (int dh = 0; dh < 2; ++dh)
#pragma unroll
            for (int dw = 0; dw < 2; ++dw) {
              const int kh = 1 + a - 2 * dh, kw = 1 + b - 2 * dw;
              if (kh < 0 || kw < 0) continue;  // compile-time after unrolling
              const PoolWin<T>& win = dh ? bot : top;
              const int pos = kh * 3 + kw;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const uint32_t word = (uint32_t)(win.packed[dw] >> (32 * (j >> 2)));
                if (__builtin_amdgcn_ubfe(word, 8 * (j & 3), 8) == (uint32_t)pos) acc[j] += win.g(dw, j);
              }
            }
          const int h = 2 * t + a, w = 2 * u + b;
          if (h >= H || w >= W) continue;
          float yv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) yv[j] = yq[a * 2 + b].get(j);
          float out[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // constants are read four channels at a time (the barrier keeps the compiler from
            // issuing all 40 LDS reads at once, which set the kernel's register peak)
            if (j == 4) asm volatile("" ::: "memory");
            // g at the precision the unfused maxpool backward stores it, masked by the ReLU
            const float g = fmaf(yv[j], cst[0][c0 + j], cst[1][c0 + j]) > 0.f ? rnd<T>(acc[j]) : 0.f;
            if (ELEM) {
              out[j] = fmaf(cst[2][c0 + j], g, fmaf(ck2[c0 + j], yv[j], cst[3][c0 + j]));
            } else {
              s1[j] += g;
              s2[j] = fmaf(g, yv[j] - cst[2][c0 + j], s2[j]);
            }
          }
          if (ELEM) dev::st8_stream(dx + (((int64_t)n * H + h) * W + w) * C + c0, out);
        }
      top = bot;
    }
  }
  if (ELEM) return;
  // block reduce over the lanes sharing c0 (256 / cv of them), then [block][C][2] partials
  __shared__ float red[256][17];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x][j] = s1[j];
    red[threadIdx.x][8 + j] = s2[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * 2; i += blockDim.x) {  // i = channel * 2 + which
    const int c = i >> 1, which = i & 1, chunk = c / 8, j = c % 8;
    float v = 0.f;
    for (int l = chunk; l < (int)blockDim.x; l += cv) v += red[l][which * 8 + j];
    part[((int64_t)blockIdx.x * C + c) * 2 + which] = v;
  }
}

// Global average pool backward, channels_last: dX[b][h][w][c] = g[b][c] / (H·W). One lane per
// 8 channels of one pixel (a 16-B store), the lane's 8 g values loaded once per pixel run.
template <typename T, typename G>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const G* __restrict__ g, T* __restrict__ dx, int64_t nvec,
                                                       int C, int HW, float inv) {
  const int cv = C / 8;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 8;
    const int64_t b = pix / HW;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = dev::Elem<G, float>::ld(g, b * C + c0 + j) * inv;
    dev::st8_stream(dx + v * 8, o);
  }
}

template <typename F>
void dispatch_pool(at::ScalarType st, F&& f) {
  switch (st) {
    case at::kBFloat16: f(bf16_t{}); break;
    case at::kFloat: f(float{}); break;
    case at::kHalf: f(f16_t{}); break;
    default: TORCH_CHECK(false, "xddp maxpool: unsupported dtype ", st);
  }
}

void check(const at::Tensor& x, int64_t k) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "xddp maxpool expects a 4-D device tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "xddp maxpool expects channels_last");
  TORCH_CHECK(x.size(1) % 8 == 0, "xddp maxpool needs C % 8 == 0");
  TORCH_CHECK(k * k <= 255, "xddp maxpool kernel too large for a byte argmax");
}

int grid_for(int64_t total) { return (int)std::min<int64_t>((total + 255) / 256, 256 * 32); }

}  // namespace

std::vector<at::Tensor> maxpool_forward(const at::Tensor& x, int64_t k, int64_t stride, int64_t pad) {
  check(x, k);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (int)((H + 2 * pad - k) / stride + 1), OW = (int)((W + 2 * pad - k) / stride + 1);
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (total == 0) return {y, idx};
  dispatch_pool(x.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((maxpool_fwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(x.data_ptr()), reinterpret_cast<T*>(y.data_ptr()),
                       idx.data_ptr<uint8_t>(), N, H, W, C, OH, OW, (int)k, (int)stride, (int)pad);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return {y, idx};
}

at::Tensor maxpool_backward(const at::Tensor& dy_in, const at::Tensor& idx, const at::Tensor& x_like, int64_t k,
                            int64_t stride, int64_t pad, const c10::optional<at::Tensor>& dy2_in) {
  auto dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  at::Tensor dy2 = (dy2_in.has_value() && dy2_in->defined()) ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast)
                                                              : at::Tensor();
  const int N = (int)x_like.size(0), C = (int)x_like.size(1), H = (int)x_like.size(2), W = (int)x_like.size(3);
  const int OH = (int)dy.size(2), OW = (int)dy.size(3);
  TORCH_CHECK(idx.numel() == dy.numel(), "maxpool backward: index/dy size mismatch");
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (total == 0) return dx;
  dispatch_pool(dy.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    if (k == 3 && stride == 2 && pad == 1) {
      const int64_t quads = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
      hipLaunchKernelGGL((maxpool_bwd_k3s2p1_kernel<T>), dim3(grid_for(quads)), dim3(256), 0, stream,
                         reinterpret_cast<const T*>(dy.data_ptr()),
                         dy2.defined() ? reinterpret_cast<const T*>(dy2.data_ptr()) : nullptr,
                         idx.data_ptr<uint8_t>(), reinterpret_cast<T*>(dx.data_ptr()), N, H, W, C, OH, OW);
      XDDP_HIP_CHECK(hipGetLastError());
      return;
    }
    hipLaunchKernelGGL((maxpool_bwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(dy.data_ptr()),
                       dy2.defined() ? reinterpret_cast<const T*>(dy2.data_ptr()) : nullptr, idx.data_ptr<uint8_t>(),
                       reinterpret_cast<T*>(dx.data_ptr()), N, H, W, C, OH, OW, (int)k, (int)stride, (int)pad);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return dx;
}

// [B, C] gradient of a global average pool -> [B, C, H, W] channels_last (dtype of x_like)
at::Tensor global_avg_pool_backward(const at::Tensor& g, const at::Tensor& x_like) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && x_like.dim() == 4 && g.size(0) == x_like.size(0) &&
                  g.size(1) == x_like.size(1) && x_like.size(1) % 8 == 0,
              "global_avg_pool_backward: g [B, C] contiguous, C % 8 == 0");
  const int64_t B = x_like.size(0), C = x_like.size(1), H = x_like.size(2), W = x_like.size(3);
  auto dx = at::empty({B, C, H, W}, x_like.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t nvec = B * H * W * (C / 8);
  if (nvec == 0) return dx;
  auto stream = c10::hip::getCurrentHIPStream(g.device().index()).stream();
  dispatch_pool(x_like.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    auto go = [&](auto gtag) {
      using G = decltype(gtag);
      hipLaunchKernelGGL((gap_bwd_kernel<T, G>), dim3(grid_for(nvec)), dim3(256), 0, stream,
                         reinterpret_cast<const G*>(g.data_ptr()), reinterpret_cast<T*>(dx.data_ptr()), nvec, (int)C,
                         (int)(H * W), 1.f / (float)(H * W));
      XDDP_HIP_CHECK(hipGetLastError());
    };
    if (g.scalar_type() == at::kFloat) go(float{});
    else if (g.scalar_type() == at::kBFloat16) go(bf16_t{});
    else TORCH_CHECK(false, "global_avg_pool_backward: g must be float or bf16");
  });
  return dx;
}

// ResNet stem: maxpool(3, 2, 1) of relu(x·scale + shift) -> (pooled, byte argmax)
std::vector<at::Tensor> stem_pool_forward(const at::Tensor& x, const at::Tensor& ss) {
  check(x, 3);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(ss.is_cuda() && ss.scalar_type() == at::kFloat && ss.numel() == 2 * C && ss.is_contiguous(),
              "stem_pool_forward: scale/shift must be float [2, C]");
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (total == 0) return {y, idx};
  dispatch_pool(x.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((stem_pool_fwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(x.data_ptr()), ss.data_ptr<float>(), ss.data_ptr<float>() + C,
                       reinterpret_cast<T*>(y.data_ptr()), idx.data_ptr<uint8_t>(), N, H, W, C, OH, OW);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return {y, idx};
}

// Stem backward through maxpool(3, 2, 1) and the ReLU of bn(x): without coef, the BN-backward
// partial sums [blocks, C, 2] (for bn_backward_from_partials); with coef [3, C] (unfolded), dX.
at::Tensor stem_pool_bn_backward(const at::Tensor& dy_in, const c10::optional<at::Tensor>& dy2_in,
                                 const at::Tensor& idx, const at::Tensor& x, const at::Tensor& ss,
                                 const at::Tensor& mean, const c10::optional<at::Tensor>& coef) {
  check(x, 3);
  auto dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  at::Tensor dy2 = (dy2_in.has_value() && dy2_in->defined()) ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast)
                                                              : at::Tensor();
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == C && dy.size(2) == OH && dy.size(3) == OW &&
                  dy.scalar_type() == x.scalar_type() && idx.numel() == dy.numel(),
              "stem_pool_bn_backward: dy / argmax do not match x");
  if (dy2.defined()) TORCH_CHECK(dy2.sizes() == dy.sizes() && dy2.scalar_type() == dy.scalar_type(), "dy2 != dy");
  TORCH_CHECK(ss.numel() == 2 * C && mean.numel() == C && ss.scalar_type() == at::kFloat &&
                  mean.scalar_type() == at::kFloat, "stem_pool_bn_backward: ss [2, C], mean [C] float");
  const bool elem = coef.has_value() && coef->defined();
  if (elem) TORCH_CHECK(coef->numel() == 3 * C && coef->scalar_type() == at::kFloat, "coef must be float [3, C]");
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int64_t lanes = (int64_t)N * (((H + 1) / 2 + kStrip - 1) / kStrip) * ((W + 1) / 2) * (C / 8);
  TORCH_CHECK(lanes < ((int64_t)1 << 31) - 256, "stem_pool_bn_backward: input too large");
  const int grid = (int)((lanes + 255) / 256);
  TORCH_CHECK(256 % (C / 8) == 0 && C <= 512, "stem_pool_bn_backward: C / 8 must divide 256, C <= 512");
  at::Tensor out = elem ? at::empty_like(x, at::MemoryFormat::ChannelsLast)
                        : at::empty({grid, C, 2}, x.options().dtype(at::kFloat));
  dispatch_pool(x.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const T*>(dy.data_ptr()),
                         dy2.defined() ? reinterpret_cast<const T*>(dy2.data_ptr()) : nullptr, idx.data_ptr<uint8_t>(),
                         reinterpret_cast<const T*>(x.data_ptr()), ss.data_ptr<float>(), ss.data_ptr<float>() + C,
                         mean.data_ptr<float>(), elem ? coef->data_ptr<float>() : nullptr,
                         elem ? nullptr : out.data_ptr<float>(), elem ? reinterpret_cast<T*>(out.data_ptr()) : nullptr,
                         N, H, W, C, OH, OW);
      XDDP_HIP_CHECK(hipGetLastError());
    };
    if (elem) go(stem_pool_bn_bwd_kernel<T, true>);
    else go(stem_pool_bn_bwd_kernel<T, false>);
  });
  return out;
}

}  // namespace kernels
}  // namespace xddp
