// Fused elementwise kernels of the transformer configs (Llama-3-8B, BASELINE.json config 5) on
// gfx950: rotary position embedding and the SwiGLU gate, forward and backward.
//
// Reference path (models/llama.py before these kernels): RoPE was ~10 PyTorch ops per tensor
// (two strided fp32 slices, four products, stack, flatten, cast) and SwiGLU three (silu, mul,
// and their autograd partners), each a full pass over a [tokens, heads x 128] or
// [tokens, 14336] activation. Here each is one read and one write: a lane owns 8 consecutive
// elements (one 16-B bf16 vector = 4 rotary pairs), cos/sin come from a [S, Dh/2] fp32 table
// (L2-resident), and the SwiGLU backward recomputes sigmoid(a) instead of saving it.
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

constexpr int kBlock = 256;

// x, y: [rows = B*S*H, Dh] contiguous (token-major: row r has position s = (r / H) % S).
// Pair (2i, 2i+1) of a row rotates by angle (s, i): y0 = x0 c - x1 s, y1 = x0 s + x1 c.
// BWD applies the transpose rotation: dx0 = dy0 c + dy1 s, dx1 = -dy0 s + dy1 c.
template <typename T, bool BWD>
__global__ __launch_bounds__(kBlock) void rope_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                      const float* __restrict__ cosv, const float* __restrict__ sinv,
                                                      int64_t nvec, int H, int S, int Dh) {
  const int vpr = Dh / 8;  // 16-B vectors per row
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = v / vpr;
    const int i0 = (int)(v - row * vpr) * 4;  // first rotary pair of this vector
    const int s = (int)((row / H) % S);
    float a[8], c[4], sn[4];
    Vec8<T>::ld(x + v * 8, a);
    const dev::f32x4 cc = *reinterpret_cast<const dev::f32x4*>(cosv + (int64_t)s * (Dh / 2) + i0);
    const dev::f32x4 ss = *reinterpret_cast<const dev::f32x4*>(sinv + (int64_t)s * (Dh / 2) + i0);
    c[0] = cc.x; c[1] = cc.y; c[2] = cc.z; c[3] = cc.w;
    sn[0] = ss.x; sn[1] = ss.y; sn[2] = ss.z; sn[3] = ss.w;
    float o[8];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float x0 = a[2 * p], x1 = a[2 * p + 1];
      if (BWD) {
        o[2 * p] = fmaf(x0, c[p], x1 * sn[p]);
        o[2 * p + 1] = fmaf(x1, c[p], -x0 * sn[p]);
      } else {
        o[2 * p] = fmaf(x0, c[p], -x1 * sn[p]);
        o[2 * p + 1] = fmaf(x0, sn[p], x1 * c[p]);
      }
    }
    Vec8<T>::st(y + v * 8, o);
  }
}

// SwiGLU gate: h = silu(a) * b. Backward: with s = sigmoid(a),
//   da = g * b * s * (1 + a * (1 - s)),   db = g * a * s.
template <typename T>
__global__ __launch_bounds__(kBlock) void swiglu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                            T* __restrict__ h, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    float x[8], z[8], o[8];
    Vec8<T>::ld(a + v * 8, x);
    Vec8<T>::ld(b + v * 8, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = x[j] / (1.f + __expf(-x[j])) * z[j];
    Vec8<T>::st(h + v * 8, o);
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void swiglu_bwd_kernel(const T* __restrict__ g, const T* __restrict__ a,
                                                            const T* __restrict__ b, T* __restrict__ da,
                                                            T* __restrict__ db, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    float gg[8], x[8], z[8], oa[8], ob[8];
    Vec8<T>::ld(g + v * 8, gg);
    Vec8<T>::ld(a + v * 8, x);
    Vec8<T>::ld(b + v * 8, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = 1.f / (1.f + __expf(-x[j]));
      ob[j] = gg[j] * x[j] * s;
      oa[j] = gg[j] * z[j] * s * fmaf(x[j], 1.f - s, 1.f);
    }
    Vec8<T>::st(da + v * 8, oa);
    Vec8<T>::st(db + v * 8, ob);
  }
}

template <typename F>
void dispatch16(at::ScalarType st, F&& f) {
  switch (st) {
    case at::kBFloat16: f(bf16_t{}); break;
    case at::kHalf: f(f16_t{}); break;
    case at::kFloat: f(float{}); break;
    default: TORCH_CHECK(false, "xddp transformer kernels: unsupported dtype ", st);
  }
}

int grid_for(int64_t nvec) { return (int)std::min<int64_t>((nvec + kBlock - 1) / kBlock, 256 * 16); }

void check_vec(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, ": expects a contiguous GPU tensor");
  TORCH_CHECK(t.numel() % 8 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what,
              ": numel % 8 == 0 and 16-B alignment required");
}

}  // namespace

// x: [B, S, H, Dh] contiguous; cos/sin: [>= S, Dh/2] fp32 contiguous. Returns the rotated tensor
// (backward = the inverse rotation, applied to the incoming gradient).
at::Tensor rope(const at::Tensor& x, const at::Tensor& cosv, const at::Tensor& sinv, bool backward) {
  check_vec(x, "rope");
  TORCH_CHECK(x.dim() == 4, "rope: x must be [B, S, H, Dh]");
  const int S = (int)x.size(1), H = (int)x.size(2), Dh = (int)x.size(3);
  TORCH_CHECK(Dh % 8 == 0, "rope: head dim must be a multiple of 8");
  TORCH_CHECK(cosv.scalar_type() == at::kFloat && sinv.scalar_type() == at::kFloat && cosv.is_contiguous() &&
                  sinv.is_contiguous() && cosv.dim() == 2 && cosv.size(0) >= S && cosv.size(1) == Dh / 2 &&
                  sinv.sizes() == cosv.sizes() && cosv.is_cuda(),
              "rope: cos/sin must be fp32 [>= S, Dh/2] on the GPU");
  auto y = at::empty_like(x);
  const int64_t nvec = x.numel() / 8;
  if (nvec == 0) return y;
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  dispatch16(x.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    auto k = backward ? rope_kernel<T, true> : rope_kernel<T, false>;
    hipLaunchKernelGGL(k, dim3(grid_for(nvec)), dim3(kBlock), 0, stream, reinterpret_cast<const T*>(x.data_ptr()),
                       reinterpret_cast<T*>(y.data_ptr()), cosv.data_ptr<float>(), sinv.data_ptr<float>(), nvec, H, S,
                       Dh);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return y;
}

at::Tensor swiglu_forward(const at::Tensor& a, const at::Tensor& b) {
  check_vec(a, "swiglu");
  check_vec(b, "swiglu");
  TORCH_CHECK(a.sizes() == b.sizes() && a.scalar_type() == b.scalar_type(), "swiglu: a and b must match");
  auto h = at::empty_like(a);
  const int64_t nvec = a.numel() / 8;
  if (nvec == 0) return h;
  auto stream = c10::hip::getCurrentHIPStream(a.device().index()).stream();
  dispatch16(a.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((swiglu_fwd_kernel<T>), dim3(grid_for(nvec)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const T*>(a.data_ptr()), reinterpret_cast<const T*>(b.data_ptr()),
                       reinterpret_cast<T*>(h.data_ptr()), nvec);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return h;
}

std::vector<at::Tensor> swiglu_backward(const at::Tensor& g, const at::Tensor& a, const at::Tensor& b) {
  check_vec(g, "swiglu_backward");
  check_vec(a, "swiglu_backward");
  check_vec(b, "swiglu_backward");
  TORCH_CHECK(g.sizes() == a.sizes() && a.sizes() == b.sizes() && g.scalar_type() == a.scalar_type(),
              "swiglu_backward: shapes/dtypes must match");
  auto da = at::empty_like(a), db = at::empty_like(b);
  const int64_t nvec = a.numel() / 8;
  if (nvec == 0) return {da, db};
  auto stream = c10::hip::getCurrentHIPStream(a.device().index()).stream();
  dispatch16(a.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((swiglu_bwd_kernel<T>), dim3(grid_for(nvec)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const T*>(g.data_ptr()), reinterpret_cast<const T*>(a.data_ptr()),
                       reinterpret_cast<const T*>(b.data_ptr()), reinterpret_cast<T*>(da.data_ptr()),
                       reinterpret_cast<T*>(db.data_ptr()), nvec);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return {da, db};
}

}  // namespace kernels
}  // namespace xddp
