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

}  // namespace kernels
}  // namespace xddp
