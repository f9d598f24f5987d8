// LayerNorm / RMSNorm over the last dimension on gfx950 (ViT-L/16 and Llama-3 configs of
// BASELINE.json; SURVEY.md §2.6 "LayerNorm/RMSNorm are HIP (ours)").
//
// One 64-lane wavefront owns one row; the row lives in registers (D/512 16-byte vectors per
// lane, D <= 8192), so mean/variance are exact two-pass values with no LDS and no re-read.
// Four rows per 256-thread block. Backward computes dx per row the same way, and
// accumulates dγ/dβ column partials in registers across the rows a block visits
// (grid-stride), folded through LDS into one partial row per block and reduced by a second
// small kernel — no float atomics, bitwise reproducible.
#include <cstdlib>

#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

using dev::bf16_t;
using dev::Elem;
using dev::f16_t;
using dev::u32x4;
using dev::Vec8;

namespace {

constexpr int kRowsPerBlock = 4;
constexpr int kMaxVec = 16;  // 16 vectors × 8 × 64 lanes = D up to 8192

// addb / xb (optional): xb = x + addb, the residual stream with the NEXT linear's bias folded in
// (the transformer block then adds its projection onto xb with a beta = 1 GEMM: no add pass)
template <typename T, typename W, int NV, bool RMS>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const W* __restrict__ gamma,
                                                     const W* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int D, float eps, const W* __restrict__ addb,
                                                     T* __restrict__ xb) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * D;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < D) {
      Vec8<T>::ld(xr + c, v[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = dev::wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        q = fmaf(d, d, q);
      }
    }
  }
  const float rstd = rsqrtf(dev::wave_sum(q) / (float)D + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  T* yr = y + row * D;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < D) {
      float g[8], b[8], o[8];
      if (gamma) Vec8<W>::ld(gamma + c, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
      if (!RMS && beta) Vec8<W>::ld(beta + c, b); else for (int j = 0; j < 8; ++j) b[j] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf((v[k][j] - mean) * rstd, g[j], b[j]);
      Vec8<T>::st(yr + c, o);
      if (addb) {  // uniform per launch
        Vec8<W>::ld(addb + c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[k][j] + b[j];
        Vec8<T>::st(xb + row * D + c, o);
      }
    }
  }
}

// dx per row + register-resident dγ/dβ column partials; part = [gridDim.x][NP][D].
// RES: dx += res (the residual-stream gradient that bypasses this norm, so the caller's add pass
// disappears), and two more column partials: Σ res and Σ dx — the bias gradients of the linear
// layers whose outputs fed the residual sums after and before this norm. NP = RES ? 4 : 2.
// With RES the narrow-row loop prefetches res with the next row's x / dy (RPF).
// SUMS (LayerNorm's residual form): the Σ res / Σ dx column partials; RMSNorm's residual form
// (Llama's pre-norm blocks: the skip connection's gradient) only adds res to dx.
template <typename T, typename W, int NV, bool RMS, bool RES, bool RPF = RES, bool SUMS = RES>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ gamma, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                     float* __restrict__ part, int64_t rows, int D,
                                                     const T* __restrict__ res) {
  constexpr int NP = SUMS ? 4 : 2;
  constexpr bool DB = !RMS;  // RMSNorm has no beta: no Σdy partial (half the partial registers)
  __shared__ float red[kRowsPerBlock][64 * 8 * 2];  // one-vector-at-a-time fold buffer (two sums)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float dg[NV][8], db[NV][8], sr[SUMS ? NV : 1][8], so[SUMS ? NV : 1][8];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[k][j] = db[k][j] = 0.f;
  if (SUMS) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) sr[k][j] = so[k][j] = 0.f;
  }
  const float invD = 1.f / (float)D;
  if constexpr (NV <= 2) {
    float gm[NV][8];  // gamma: loaded once
  #pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (gamma && c < D) Vec8<W>::ld(gamma + c, gm[k]);
      else for (int j = 0; j < 8; ++j) gm[k][j] = 1.f;
    }
    // Software-pipelined over this wave's rows: the next row's x / dy / res (and mean, rstd) are
    // loaded while the current row is reduced and written, and each row is read once (both passes
    // run from registers) — the one-row-at-a-time version waited a full memory latency per pass,
    // and a res loaded in pass 2 one latency per row (ViT-L/16 rows, residual form: 117 -> 107 us).
    constexpr int NR = RPF ? NV : 1;
    const int64_t step = (int64_t)gridDim.x * kRowsPerBlock;
    auto load_row = [&](int64_t r, float (&a)[NV][8], float (&d)[NV][8], float (&rr)[NR][8], float& mu, float& rs) {
      mu = RMS ? 0.f : mean_in[r];
      rs = rstd_in[r];
  #pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < D) {
          Vec8<T>::ld(x + r * D + c, a[k]);
          Vec8<T>::ld(dy + r * D + c, d[k]);
          if (RPF) Vec8<T>::ld(res + r * D + c, rr[RPF ? k : 0]);
        }
      }
    };
    // both passes of one row from registers: dx (+ res), the column partials
    auto row_math = [&](int64_t row, const float (&a)[NV][8], const float (&d)[NV][8], const float (&rv)[NR][8],
                        float mean, float rstd) {
      // pass 1: row reductions
      float s1 = 0.f, s2 = 0.f;
  #pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < D) {
  #pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float gy = d[k][j] * gm[k][j];
            s1 += gy;
            s2 = fmaf(gy, (a[k][j] - mean) * rstd, s2);
          }
        }
      }
      const float m1 = RMS ? 0.f : dev::wave_sum(s1) * invD;
      const float m2 = dev::wave_sum(s2) * invD;
  #pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < D) {
          float o[8], r1[8];
          if (RES && !RPF) Vec8<T>::ld(res + row * D + c, r1);
  #pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xh = (a[k][j] - mean) * rstd;
            o[j] = rstd * (d[k][j] * gm[k][j] - m1 - xh * m2);
            dg[k][j] = fmaf(d[k][j], xh, dg[k][j]);
            if (DB) db[k][j] += d[k][j];
          }
          if (RES) {
  #pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float rj = RPF ? rv[RPF ? k : 0][j] : r1[j];
              o[j] += rj;
              if (SUMS) {
                sr[SUMS ? k : 0][j] += rj;
                so[SUMS ? k : 0][j] += o[j];
              }
            }
          }
          Vec8<T>::st(dx + row * D + c, o);
        }
      }
    };
    int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + w;
    if constexpr (__is_same(T, bf16_t) && RPF) {
      // bf16 residual form (ViT-L/16 rows): rows in flight as packed bf16, three slots rotating, so
      // two rows' loads (12 KB per wave) are outstanding while one is reduced and written — one
      // row of unpacked floats in flight left ~12 MB in flight chip-wide, short of the HBM latency
      // x bandwidth product. Row indices clamp to the last row (the look-ahead past the end re-reads
      // it), so the loads stay branch-free and the compiler's counted waits retire one slot at a time.
      struct Slot {
        u32x4 a[NV], d[NV], r[NV];
        float mu, rs;
      };
      auto ld_slot = [&](int64_t r, Slot& sl) {
        r = r < rows ? r : rows - 1;
        sl.mu = RMS ? 0.f : mean_in[r];
        sl.rs = rstd_in[r];
  #pragma unroll
        for (int k = 0; k < NV; ++k) {
          const int c = (k * 64 + lane) * 8;
          if (c < D) {
            sl.a[k] = *reinterpret_cast<const u32x4*>(x + r * D + c);
            sl.d[k] = *reinterpret_cast<const u32x4*>(dy + r * D + c);
            sl.r[k] = *reinterpret_cast<const u32x4*>(res + r * D + c);
          }
        }
      };
      auto run = [&](int64_t r, const Slot& sl) {
        float a[NV][8], d[NV][8], rv[NR][8];
  #pragma unroll
        for (int k = 0; k < NV; ++k)
  #pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[k][2 * j] = __uint_as_float(sl.a[k][j] << 16);
            a[k][2 * j + 1] = __uint_as_float(sl.a[k][j] & 0xffff0000u);
            d[k][2 * j] = __uint_as_float(sl.d[k][j] << 16);
            d[k][2 * j + 1] = __uint_as_float(sl.d[k][j] & 0xffff0000u);
            rv[RPF ? k : 0][2 * j] = __uint_as_float(sl.r[k][j] << 16);
            rv[RPF ? k : 0][2 * j + 1] = __uint_as_float(sl.r[k][j] & 0xffff0000u);
          }
        row_math(r, a, d, rv, sl.mu, sl.rs);
      };
      if (row < rows) {
        Slot s0, s1, s2;
        ld_slot(row, s0);
        ld_slot(row + step, s1);
        for (;;) {
          ld_slot(row + 2 * step, s2);
          run(row, s0);
          if ((row += step) >= rows) break;
          ld_slot(row + 2 * step, s0);
          run(row, s1);
          if ((row += step) >= rows) break;
          ld_slot(row + 2 * step, s1);
          run(row, s2);
          if ((row += step) >= rows) break;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      float a[NV][8], d[NV][8], rv[NR][8], mean = 0.f, rstd = 0.f;
      if (row < rows) load_row(row, a, d, rv, mean, rstd);
      for (; row < rows; row += step) {
        float na[NV][8], nd[NV][8], nr[NR][8], nmean = 0.f, nrstd = 0.f;
        if (row + step < rows) load_row(row + step, na, nd, nr, nmean, nrstd);
        row_math(row, a, d, rv, mean, rstd);
  #pragma unroll
        for (int k = 0; k < NV; ++k)
  #pragma unroll
          for (int j = 0; j < 8; ++j) {
            a[k][j] = na[k][j];
            d[k][j] = nd[k][j];
            if (RPF) rv[RPF ? k : 0][j] = nr[RPF ? k : 0][j];
          }
        mean = nmean;
        rstd = nrstd;
      }
    }
  } else {  // wide rows (D > 1024): the register-lean one-row-at-a-time loop (no spills)
    for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + w; row < rows; row += (int64_t)gridDim.x * kRowsPerBlock) {
      const float mean = RMS ? 0.f : mean_in[row];
      const float rstd = rstd_in[row];
      // pass 1: row reductions (x, dy re-read in pass 2 hit L1/L2; keeps VGPRs for the partials)
      float s1 = 0.f, s2 = 0.f;
  #pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < D) {
          float a[8], d[8], g[8];
          Vec8<T>::ld(x + row * D + c, a);
          Vec8<T>::ld(dy + row * D + c, d);
          if (gamma) Vec8<W>::ld(gamma + c, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
  #pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float gy = d[j] * g[j];
            s1 += gy;
            s2 = fmaf(gy, (a[j] - mean) * rstd, s2);
          }
        }
      }
      const float m1 = RMS ? 0.f : dev::wave_sum(s1) * invD;
      const float m2 = dev::wave_sum(s2) * invD;
  #pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < D) {
          float a[8], d[8], g[8], o[8];
          Vec8<T>::ld(x + row * D + c, a);
          Vec8<T>::ld(dy + row * D + c, d);
          if (gamma) Vec8<W>::ld(gamma + c, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
  #pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xh = (a[j] - mean) * rstd;
            o[j] = rstd * (d[j] * g[j] - m1 - xh * m2);
            dg[k][j] = fmaf(d[j], xh, dg[k][j]);
            if (DB) db[k][j] += d[j];
          }
          if (RES) {
            float r[8];
            Vec8<T>::ld(res + row * D + c, r);
  #pragma unroll
            for (int j = 0; j < 8; ++j) {
              o[j] += r[j];
              if (SUMS) {
                sr[SUMS ? k : 0][j] += r[j];
                so[SUMS ? k : 0][j] += o[j];
              }
            }
          }
          Vec8<T>::st(dx + row * D + c, o);
        }
      }
    }
  }
  if (!part) return;
  // fold the 4 waves' column partials, one vector slot (two sums) at a time
  auto fold = [&](float (&pa)[NV][8], float (&pb)[NV][8], int k, int p0, bool two) {
    const int c = (k * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[w][lane * 16 + j] = pa[k][j];
      red[w][lane * 16 + 8 + j] = pb[k][j];
    }
    __syncthreads();
    if (w == 0 && c < D) {
      float* pg = part + ((int64_t)blockIdx.x * NP + p0) * D;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int q = 0; q < kRowsPerBlock; ++q) {
          a += red[q][lane * 16 + j];
          b += red[q][lane * 16 + 8 + j];
        }
        pg[c + j] = a;
        if (two) pg[D + c + j] = b;
      }
    }
    __syncthreads();
  };
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    fold(dg, db, k, 0, DB);
    if constexpr (SUMS) fold(sr, so, k, 2, true);
  }
}

// Column sums of the [nblk][NP][D] partials: blockIdx.y = which of the NP sums (out.p[y], skipped
// when null). One 1024-thread block per 64 columns: 16 waves each sum nblk/16 partial rows (one
// coalesced 256-B row segment per load, 8 loads in flight per lane), then fold through LDS. A
// thread-per-column loop over all nblk rows was latency-bound (~255 us for ViT-L's D=1024, 1024
// partial rows); this is ~10 us.
template <typename W>
struct ColOuts {
  W* p[4];
};

template <typename W>
__global__ __launch_bounds__(1024) void ln_param_grad_kernel(const float* __restrict__ part, int nblk, int NP, int D,
                                                             ColOuts<W> out) {
  __shared__ float red[16][64];
  W* dst = out.p[blockIdx.y];
  if (!dst) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int64_t rs = (int64_t)NP * D;
  const float* src = part + (int64_t)blockIdx.y * D + c;
  float a = 0.f;
  if (c < D) {
    int i = w;
    for (; i + 16 * 7 < nblk; i += 16 * 8) {
      float ga[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) ga[u] = src[(int64_t)(i + 16 * u) * rs];
#pragma unroll
      for (int u = 0; u < 8; ++u) a += ga[u];
    }
    for (; i < nblk; i += 16) a += src[(int64_t)i * rs];
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && c < D) {
    float sa = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sa += red[q][lane];
    Elem<W, float>::st(dst, c, sa);
  }
}

template <typename F>
void dispatch_t(at::ScalarType st, F&& f) {
  switch (st) {
    case at::kBFloat16: f(bf16_t{}); break;
    case at::kFloat: f(float{}); break;
    case at::kHalf: f(f16_t{}); break;
    default: TORCH_CHECK(false, "xddp layer_norm: unsupported dtype ", st);
  }
}

template <int NV, typename F>
void nv_dispatch(int nv, F&& f) {
  if constexpr (NV > kMaxVec) {
    TORCH_CHECK(false, "xddp layer_norm: D too large (max 8192)");
  } else {
    if (nv <= NV) f(std::integral_constant<int, NV>{});
    else nv_dispatch<NV * 2>(nv, f);
  }
}

}  // namespace

// returns (y, mean (empty for RMS), rstd)
std::vector<at::Tensor> ln_forward(const at::Tensor& x_in, const c10::optional<at::Tensor>& gamma,
                                   const c10::optional<at::Tensor>& beta, double eps, bool rms,
                                   const c10::optional<at::Tensor>& add_bias) {
  auto x = x_in.contiguous();
  TORCH_CHECK(x.is_cuda(), "xddp layer_norm: device tensor expected");
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "xddp layer_norm needs D % 8 == 0 and D <= 8192");
  const int64_t rows = x.numel() / D;
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto rstd = at::empty({rows}, fopt);
  auto mean = rms ? at::Tensor() : at::empty({rows}, fopt);
  const bool hg = gamma.has_value() && gamma->defined(), hb = beta.has_value() && beta->defined();
  const auto wdt = hg ? gamma->scalar_type() : x.scalar_type();
  const bool ha = add_bias.has_value() && add_bias->defined();
  if (ha)
    TORCH_CHECK(add_bias->is_contiguous() && add_bias->numel() == D && add_bias->scalar_type() == wdt,
                "xddp layer_norm: add_bias must be [D] in the weight dtype");
  auto xb = ha ? at::empty_like(x) : at::Tensor();
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int nv = (D / 8 + 63) / 64;
  const int grid = (int)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  if (rows == 0) return {y, mean, rstd, xb};
  dispatch_t(x.scalar_type(), [&](auto tt) {
    using T = decltype(tt);
    dispatch_t(wdt, [&](auto tw) {
      using W = decltype(tw);
      nv_dispatch<1>(nv, [&](auto nvc) {
        constexpr int NV = decltype(nvc)::value;
        auto k = rms ? ln_fwd_kernel<T, W, NV, true> : ln_fwd_kernel<T, W, NV, false>;
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const T*>(x.data_ptr()),
                           hg ? reinterpret_cast<const W*>(gamma->data_ptr()) : nullptr,
                           hb ? reinterpret_cast<const W*>(beta->data_ptr()) : nullptr,
                           reinterpret_cast<T*>(y.data_ptr()), rms ? nullptr : mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), rows, D, (float)eps,
                           ha ? reinterpret_cast<const W*>(add_bias->data_ptr()) : nullptr,
                           ha ? reinterpret_cast<T*>(xb.data_ptr()) : nullptr);
        XDDP_HIP_CHECK(hipGetLastError());
      });
    });
  });
  return {y, mean, rstd, xb};
}

// returns (dx, dgamma, dbeta, Σ res, Σ dx); with res: dx = LN backward + res (the last two only then,
// LayerNorm only)
std::vector<at::Tensor> ln_backward(const at::Tensor& dy_in, const at::Tensor& x_in,
                                    const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& mean,
                                    const at::Tensor& rstd, bool rms, bool need_dgamma, bool need_dbeta,
                                    const c10::optional<at::Tensor>& res_in) {
  auto x = x_in.contiguous();
  auto dy = dy_in.contiguous();
  const int D = (int)x.size(-1);
  const int64_t rows = x.numel() / D;
  auto dx = at::empty_like(x);
  const bool hg = gamma.has_value() && gamma->defined();
  const bool hr = res_in.has_value() && res_in->defined();
  at::Tensor res;
  if (hr) {
    res = res_in->contiguous();
    TORCH_CHECK(res.sizes() == x.sizes() && res.scalar_type() == x.scalar_type(),
                "xddp layer_norm backward: res must match x");
  }
  const auto wdt = hg ? gamma->scalar_type() : x.scalar_type();
  auto wopt = hg ? gamma->options() : x.options();
  at::Tensor dgamma = (hg && need_dgamma) ? at::empty({D}, wopt) : at::Tensor();
  at::Tensor dbeta = (need_dbeta && !rms) ? at::empty({D}, wopt) : at::Tensor();
  const bool sums = hr && !rms;  // (RMSNorm's residual form: dx += res only)
  at::Tensor sres = sums ? at::empty({D}, wopt) : at::Tensor(), sout = sums ? at::empty({D}, wopt) : at::Tensor();
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int nv = (D / 8 + 63) / 64;
  const bool need_part = dgamma.defined() || dbeta.defined() || sums;
  const int NP = sums ? 4 : 2;
  // Block cap: the narrow-row (software-pipelined) loop runs at 2 waves per SIMD, so 512 blocks are
  // exactly one resident round on 256 CUs (ViT-L/16 rows: 107 -> 100 us with the residual form,
  // 96 -> 90 without, vs 1024 blocks; 2048 / 4096 were slower still: profiles/r3_ln_bwd_ab.txt).
  static const int cus = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  // (wide rows, Llama-3-8B's 4096: 512 blocks 33.5 us vs 1024 39.5 / 256 36.0 / 2048 39.2 us,
  // scripts/ln_bwd_time.py — fewer column-partial folds and a smaller partial buffer)
  const int grid_cap = 2 * cus;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + kRowsPerBlock - 1) / kRowsPerBlock, grid_cap));
  auto part = need_part ? at::empty({grid, NP, D}, x.options().dtype(at::kFloat)) : at::Tensor();
  if (rows == 0) return {dx, dgamma, dbeta, sres, sout};
  dispatch_t(x.scalar_type(), [&](auto tt) {
    using T = decltype(tt);
    dispatch_t(wdt, [&](auto tw) {
      using W = decltype(tw);
      nv_dispatch<1>(nv, [&](auto nvc) {
        constexpr int NV = decltype(nvc)::value;
        auto k = rms ? (hr ? ln_bwd_kernel<T, W, NV, true, true, true, false> : ln_bwd_kernel<T, W, NV, true, false>)
                     : (hr ? ln_bwd_kernel<T, W, NV, false, true> : ln_bwd_kernel<T, W, NV, false, false>);
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const T*>(dy.data_ptr()),
                           reinterpret_cast<const T*>(x.data_ptr()),
                           hg ? reinterpret_cast<const W*>(gamma->data_ptr()) : nullptr,
                           (!rms && mean.has_value()) ? mean->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),
                           reinterpret_cast<T*>(dx.data_ptr()), need_part ? part.data_ptr<float>() : nullptr, rows,
                           D, hr ? reinterpret_cast<const T*>(res.data_ptr()) : nullptr);
        XDDP_HIP_CHECK(hipGetLastError());
      });
      if (need_part) {
        auto ptr = [](at::Tensor& t) { return t.defined() ? reinterpret_cast<W*>(t.data_ptr()) : nullptr; };
        ColOuts<W> outs{{ptr(dgamma), ptr(dbeta), ptr(sres), ptr(sout)}};
        hipLaunchKernelGGL((ln_param_grad_kernel<W>), dim3((D + 63) / 64, NP), dim3(1024), 0, stream,
                           part.data_ptr<float>(), grid, NP, D, outs);
        XDDP_HIP_CHECK(hipGetLastError());
      }
    });
  });
  return {dx, dgamma, dbeta, sres, sout};
}

// Column sums of [P][N] fp32 partial rows into out [N] (dtype of out): the second stage of the
// bias-gradient reductions in transformer.hip.
void colsum_partials(const at::Tensor& part, at::Tensor& out) {
  TORCH_CHECK(part.is_contiguous() && part.scalar_type() == at::kFloat && part.dim() == 2 &&
                  out.numel() == part.size(1) && out.is_contiguous(),
              "colsum_partials: part [P, N] fp32, out [N]");
  const int P = (int)part.size(0), N = (int)part.size(1);
  auto stream = c10::hip::getCurrentHIPStream(part.device().index()).stream();
  dispatch_t(out.scalar_type(), [&](auto tw) {
    using W = decltype(tw);
    ColOuts<W> outs{{reinterpret_cast<W*>(out.data_ptr()), nullptr, nullptr, nullptr}};
    hipLaunchKernelGGL((ln_param_grad_kernel<W>), dim3((N + 63) / 64, 1), dim3(1024), 0, stream,
                       part.data_ptr<float>(), P, 1, N, outs);
    XDDP_HIP_CHECK(hipGetLastError());
  });
}

}  // namespace kernels
}  // namespace xddp
