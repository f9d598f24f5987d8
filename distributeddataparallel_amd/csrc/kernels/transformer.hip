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
#include "kernels/norm.h"

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

// GELU (exact, erf form): gelu(x) = x Φ(x), Φ(x) = (1 + erf(x / √2)) / 2;
// gelu'(x) = Φ(x) + x φ(x), φ(x) = exp(-x² / 2) / √(2π).
// (dev::gelu / dev::gelu_grad: the branch-free erf of dev_utils.h, shared with the GEMM epilogues)
__device__ __forceinline__ float gelu_f(float x) { return dev::gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return dev::gelu_grad(x); }

template <typename T>
__global__ __launch_bounds__(kBlock) void gelu_fwd_kernel(const T* __restrict__ h, T* __restrict__ a, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    float x[8];
    Vec8<T>::ld(h + v * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = gelu_f(x[j]);
    Vec8<T>::st(a + v * 8, x);
  }
}

// Bias gradient of a linear layer = column sums of its output gradient g [rows, N]; with GELU the
// layer feeds a GELU and g is the gradient after it: dh = g · gelu'(h) is written and summed in
// the same pass. Each thread owns one 8-column chunk (fixed, so its 8 sums stay in registers) and
// every rgroups-th row; part [rgroups][N] fp32 is summed by colsum_partials (layer_norm.hip).
template <typename T, bool GELU>
__global__ __launch_bounds__(kBlock) void bias_grad_kernel(const T* __restrict__ g, const T* __restrict__ h,
                                                           T* __restrict__ dh, float* __restrict__ part, int64_t rows,
                                                           int N, int rgroups) {
  const int cpr = N / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)rgroups * cpr) return;
  const int c = (int)(t % cpr) * 8, r0 = (int)(t / cpr);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
#pragma unroll 4
  for (int64_t r = r0; r < rows; r += rgroups) {
    float d[8];
    Vec8<T>::ld(g + r * N + c, d);
    if (GELU) {
      float x[8];
      Vec8<T>::ld(h + r * N + c, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] *= gelu_grad(x[j]);
      Vec8<T>::st(dh + r * N + c, d);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += d[j];
  }
  float* p = part + (int64_t)r0 * N + c;
  *reinterpret_cast<dev::f32x4*>(p) = dev::f32x4{s[0], s[1], s[2], s[3]};
  *reinterpret_cast<dev::f32x4*>(p + 4) = dev::f32x4{s[4], s[5], s[6], s[7]};
}

// 16-bit 2-D transpose [R][C] -> [C][R] through 64x64 LDS tiles (padded rows: conflict-free column
// reads): the K-major copy of a weight a GEMM wants as [N][K] rows (e.g. ViT fc2's Wᵀ for the fused
// dGELU input-gradient GEMM), at HBM speed instead of torch's strided-copy kernel.
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                          int R, int C) {
  __shared__ uint16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  // full interior tiles (R, C multiples of 8 there) move 16 B per lane each way; edges go by element
  const bool vec = r0 + 64 <= R && c0 + 64 <= C && (C & 7) == 0 && (R & 7) == 0;
  if (vec) {
#pragma unroll
    for (int i = threadIdx.x; i < 64 * 8; i += 256) {  // 64 rows x 8 chunks of 8 columns
      const int r = i >> 3, c = (i & 7) * 8;
      const dev::u32x4 v = *reinterpret_cast<const dev::u32x4*>(in + (int64_t)(r0 + r) * C + c0 + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tile[r][c + 2 * e] = (uint16_t)(v[e] & 0xffffu);
        tile[r][c + 2 * e + 1] = (uint16_t)(v[e] >> 16);
      }
    }
  } else {
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int r = i >> 6, c = i & 63;
      if (r0 + r < R && c0 + c < C) tile[r][c] = in[(int64_t)(r0 + r) * C + c0 + c];
    }
  }
  __syncthreads();
  if (vec) {
#pragma unroll
    for (int i = threadIdx.x; i < 64 * 8; i += 256) {  // 64 output rows (tile columns) x 8 chunks
      const int c = i >> 3, r = (i & 7) * 8;
      dev::u32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (uint32_t)tile[r + 2 * e][c] | ((uint32_t)tile[r + 2 * e + 1][c] << 16);
      *reinterpret_cast<dev::u32x4*>(out + (int64_t)(c0 + c) * R + r0 + r) = v;
    }
  } else {
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int c = i >> 6, r = i & 63;
      if (c0 + c < C && r0 + r < R) out[(int64_t)(c0 + c) * R + r0 + r] = tile[r][c];
    }
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

// [R, C] 16-bit contiguous -> its transpose [C, R] contiguous
at::Tensor transpose16(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.is_contiguous() && x.element_size() == 2,
              "transpose16: a contiguous 2-D 16-bit CUDA tensor expected");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(R < (int64_t(1) << 31) / 64 && C < (int64_t(1) << 31) / 64, "transpose16: too large");
  auto out = at::empty({C, R}, x.options());
  if (R == 0 || C == 0) return out;
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64)), dim3(256), 0,
                     stream, reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()),
                     (int)R, (int)C);
  XDDP_HIP_CHECK(hipGetLastError());
  return out;
}

at::Tensor gelu_forward(const at::Tensor& h) {
  check_vec(h, "gelu_forward");
  auto a = at::empty_like(h);
  const int64_t nvec = h.numel() / 8;
  if (nvec == 0) return a;
  auto stream = c10::hip::getCurrentHIPStream(h.device().index()).stream();
  dispatch16(h.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((gelu_fwd_kernel<T>), dim3(grid_for(nvec)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const T*>(h.data_ptr()), reinterpret_cast<T*>(a.data_ptr()), nvec);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  return a;
}

// g: [..., N] output gradient of a linear layer; gelu_input (optional): the pre-activation h of a
// GELU applied to that output, g then being the gradient after the GELU. Returns (bias gradient
// [N] in bias_like's dtype, dh = g · gelu'(h) or an undefined tensor).
std::vector<at::Tensor> bias_grad(const at::Tensor& g, const c10::optional<at::Tensor>& gelu_input,
                                  const at::Tensor& bias_like) {
  check_vec(g, "bias_grad");
  const int64_t N = g.size(-1), rows = g.numel() / N;
  TORCH_CHECK(N % 8 == 0 && bias_like.numel() == N, "bias_grad: N % 8 == 0 and a bias of N elements required");
  const bool gelu = gelu_input.has_value() && gelu_input->defined();
  if (gelu) {
    check_vec(*gelu_input, "bias_grad");
    TORCH_CHECK(gelu_input->sizes() == g.sizes() && gelu_input->scalar_type() == g.scalar_type(),
                "bias_grad: gelu_input must match grad");
  }
  auto dh = gelu ? at::empty_like(g) : at::Tensor();
  auto db = at::empty({N}, bias_like.options().memory_format(at::MemoryFormat::Contiguous));
  const int cpr = (int)(N / 8);
  // each thread sums rows / rgroups rows of its column chunk, one dependent 16-B load after
  // another: at 128K threads (8 waves per CU) the pass is latency-limited (GELU: 283 us, 4.4 TB/s
  // on ViT-L/16's [50432, 4096]; plain: 70 us, 1.5 TB/s on [50432, 1024]); 512K threads fill the CUs
  const int64_t target = 524288;
  const int rgroups = (int)std::max<int64_t>(1, std::min<int64_t>(rows, (target + cpr - 1) / cpr));
  auto part = at::empty({rgroups, N}, g.options().dtype(at::kFloat));
  if (rows == 0) {
    db.zero_();
    return {db, dh};
  }
  auto stream = c10::hip::getCurrentHIPStream(g.device().index()).stream();
  const int64_t threads = (int64_t)rgroups * cpr;
  dispatch16(g.scalar_type(), [&](auto tag) {
    using T = decltype(tag);
    auto k = gelu ? bias_grad_kernel<T, true> : bias_grad_kernel<T, false>;
    hipLaunchKernelGGL(k, dim3((unsigned)((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const T*>(g.data_ptr()),
                       gelu ? reinterpret_cast<const T*>(gelu_input->data_ptr()) : nullptr,
                       gelu ? reinterpret_cast<T*>(dh.data_ptr()) : nullptr, part.data_ptr<float>(), rows, (int)N,
                       rgroups);
    XDDP_HIP_CHECK(hipGetLastError());
  });
  colsum_partials(part, db);
  return {db, dh};
}

}  // namespace kernels
}  // namespace xddp
