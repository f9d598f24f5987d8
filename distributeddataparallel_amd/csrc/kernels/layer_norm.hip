// LayerNorm / RMSNorm over the last dimension on gfx950 (ViT-L/16 and Llama-3 configs of
// BASELINE.json; SURVEY.md §2.6 "LayerNorm/RMSNorm are HIP (ours)").
//
// One 64-lane wavefront owns one row; the row lives in registers (D/512 16-byte vectors per
// lane, D <= 8192), so mean/variance are exact two-pass values with no LDS and no re-read.
// Four rows per 256-thread block. Backward computes dx per row the same way, and
// accumulates dγ/dβ column partials in registers across the rows a block visits
// (grid-stride), folded through LDS into one partial row per block and reduced by a second
// small kernel — no float atomics, bitwise reproducible.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

using dev::bf16_t;
using dev::Elem;
using dev::f16_t;
using dev::Vec8;

namespace {

constexpr int kRowsPerBlock = 4;
constexpr int kMaxVec = 16;  // 16 vectors × 8 × 64 lanes = D up to 8192

template <typename T, typename W, int NV, bool RMS>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const W* __restrict__ gamma,
                                                     const W* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int D, float eps) {
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
    }
  }
}

// dx per row + register-resident dγ/dβ column partials; part = [gridDim.x][2][D]
template <typename T, typename W, int NV, bool RMS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ gamma, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                     float* __restrict__ part, int64_t rows, int D) {
  __shared__ float red[kRowsPerBlock][64 * 8 * 2];  // one-vector-at-a-time fold buffer
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[k][j] = db[k][j] = 0.f;
  const float invD = 1.f / (float)D;
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
          db[k][j] += d[j];
        }
        Vec8<T>::st(dx + row * D + c, o);
      }
    }
  }
  if (!part) return;
  // fold the 4 waves' column partials, one vector slot at a time
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[w][lane * 16 + j] = dg[k][j];
      red[w][lane * 16 + 8 + j] = db[k][j];
    }
    __syncthreads();
    if (w == 0 && c < D) {
      float* pg = part + (int64_t)blockIdx.x * 2 * D;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int q = 0; q < kRowsPerBlock; ++q) {
          a += red[q][lane * 16 + j];
          b += red[q][lane * 16 + 8 + j];
        }
        pg[c + j] = a;
        pg[D + c + j] = b;
      }
    }
    __syncthreads();
  }
}

// dγ/dβ = column sums of the [nblk][2][D] partials. One 1024-thread block per 64 columns: 16
// waves each sum nblk/16 partial rows (one coalesced 256-B row segment per load, 8 loads in
// flight per lane), then fold through LDS. A thread-per-column loop over all nblk rows was
// latency-bound (~255 us for ViT-L's D=1024, 1024 partial rows); this is ~10 us.
template <typename W>
__global__ __launch_bounds__(1024) void ln_param_grad_kernel(const float* __restrict__ part, int nblk, int D,
                                                             W* __restrict__ dgamma, W* __restrict__ dbeta) {
  __shared__ float red[2][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a = 0.f, b = 0.f;
  if (c < D) {
    int i = w;
    for (; i + 16 * 7 < nblk; i += 16 * 8) {
      float ga[8], gb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        ga[u] = part[(int64_t)(i + 16 * u) * 2 * D + c];
        gb[u] = part[(int64_t)(i + 16 * u) * 2 * D + D + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += ga[u];
        b += gb[u];
      }
    }
    for (; i < nblk; i += 16) {
      a += part[(int64_t)i * 2 * D + c];
      b += part[(int64_t)i * 2 * D + D + c];
    }
  }
  red[0][w][lane] = a;
  red[1][w][lane] = b;
  __syncthreads();
  if (w == 0 && c < D) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      sa += red[0][q][lane];
      sb += red[1][q][lane];
    }
    if (dgamma) Elem<W, float>::st(dgamma, c, sa);
    if (dbeta) Elem<W, float>::st(dbeta, c, sb);
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
                                   const c10::optional<at::Tensor>& beta, double eps, bool rms) {
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
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int nv = (D / 8 + 63) / 64;
  const int grid = (int)((rows + kRowsPerBlock - 1) / kRowsPerBlock);
  if (rows == 0) return {y, mean, rstd};
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
                           rstd.data_ptr<float>(), rows, D, (float)eps);
        XDDP_HIP_CHECK(hipGetLastError());
      });
    });
  });
  return {y, mean, rstd};
}

// returns (dx, dgamma, dbeta)
std::vector<at::Tensor> ln_backward(const at::Tensor& dy_in, const at::Tensor& x_in,
                                    const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& mean,
                                    const at::Tensor& rstd, bool rms, bool need_dgamma, bool need_dbeta) {
  auto x = x_in.contiguous();
  auto dy = dy_in.contiguous();
  const int D = (int)x.size(-1);
  const int64_t rows = x.numel() / D;
  auto dx = at::empty_like(x);
  const bool hg = gamma.has_value() && gamma->defined();
  const auto wdt = hg ? gamma->scalar_type() : x.scalar_type();
  at::Tensor dgamma = (hg && need_dgamma) ? at::empty({D}, gamma->options()) : at::Tensor();
  at::Tensor dbeta = (need_dbeta && !rms) ? at::empty({D}, hg ? gamma->options() : x.options()) : at::Tensor();
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const int nv = (D / 8 + 63) / 64;
  const bool need_part = dgamma.defined() || dbeta.defined();
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + kRowsPerBlock - 1) / kRowsPerBlock, 1024));
  auto part = need_part ? at::empty({grid, 2, D}, x.options().dtype(at::kFloat)) : at::Tensor();
  if (rows == 0) return {dx, dgamma, dbeta};
  dispatch_t(x.scalar_type(), [&](auto tt) {
    using T = decltype(tt);
    dispatch_t(wdt, [&](auto tw) {
      using W = decltype(tw);
      nv_dispatch<1>(nv, [&](auto nvc) {
        constexpr int NV = decltype(nvc)::value;
        auto k = rms ? ln_bwd_kernel<T, W, NV, true> : ln_bwd_kernel<T, W, NV, false>;
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, stream, reinterpret_cast<const T*>(dy.data_ptr()),
                           reinterpret_cast<const T*>(x.data_ptr()),
                           hg ? reinterpret_cast<const W*>(gamma->data_ptr()) : nullptr,
                           (!rms && mean.has_value()) ? mean->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),
                           reinterpret_cast<T*>(dx.data_ptr()), need_part ? part.data_ptr<float>() : nullptr, rows,
                           D);
        XDDP_HIP_CHECK(hipGetLastError());
      });
      if (need_part) {
        hipLaunchKernelGGL((ln_param_grad_kernel<W>), dim3((D + 63) / 64), dim3(1024), 0, stream,
                           part.data_ptr<float>(), grid, D,
                           dgamma.defined() ? reinterpret_cast<W*>(dgamma.data_ptr()) : nullptr,
                           dbeta.defined() ? reinterpret_cast<W*>(dbeta.data_ptr()) : nullptr);
        XDDP_HIP_CHECK(hipGetLastError());
      }
    });
  });
  return {dx, dgamma, dbeta};
}

}  // namespace kernels
}  // namespace xddp
