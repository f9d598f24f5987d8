// ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels, NHWC bf16) for gfx950, with
// the batch statistics of the BatchNorm that follows it reduced in the epilogue.
//
// MIOpen runs this layer as a generic implicit GEMM (igemm_fwd_gtcx35, 360 us at ResNet-50 bs256
// on MI355X, profiles/). Its shape is awkward for a GEMM: K = 7·7·3 = 147 and 3-channel pixels
// (6 B, no vector alignment). Here:
// * an output tile of 16 x 16 pixels needs a 37 x 38 input halo; it is staged once into LDS with
//   the channels padded to 4 (8 B per pixel) and read as the MFMA B operand directly: for kernel
//   row kh the 32-wide k-step is (kw 0..7) x (ci 0..3), so a lane's 8 k values are two
//   horizontally adjacent halo pixels — one 16-B ds_read_b128, conflict-free (16 output columns
//   at a 16-B stride, duplicate addresses broadcast). K = 7 x 32 = 224 (147 real);
// * swapped product Y^T = W·X^T on mfma_f32_16x16x32_bf16: A = weights from LDS in a
//   chunk-major [k/8][co][8] image (the 16 lanes of a b128 lane group read 16 distinct co: no
//   conflicts), B = the halo; each lane ends up with 4 consecutive channels of one pixel, stored
//   as one 8-B write;
// * persistent workgroups (2 per CU, 4 waves, each wave 4 output rows x 16 columns x 64
//   channels); the next tile's halo is loaded into registers during the current tile's MFMAs;
// * the BN statistics: shifted sums (shift = the workgroup's first output pixel, a sample of the
//   same channel) of the bf16-rounded outputs per lane, added over lanes and waves at the end, as
//   (count, mean, M2) partials per workgroup for bn_stats_from_partials — no separate stats pass
//   over the 411 MB output.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
using dev::f32x4;

constexpr int kT = 16;                 // output tile is kT x kT pixels
constexpr int kHR = 2 * kT + 5;        // halo rows (kh 0..6)
constexpr int kHC = 2 * kT + 6;        // halo cols (kw 0..7; kw = 7 has zero weight)
constexpr int kHalo = kHR * kHC * 8;   // bytes, 4 bf16 per pixel
constexpr int kSlots = (kHR * kHC + 255) / 256;
constexpr int kWBytes = 28 * 64 * 16;  // [28 k-chunks][64 co][8 bf16]

struct WStrides {
  int64_t co, ci, kh, kw;
};

__device__ __forceinline__ float bf16r(float v) { return __uint_as_float((uint32_t)dev::f32_to_bf16(v) << 16); }

__global__ __launch_bounds__(256, 2) void stem_conv_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w, WStrides ws,
                                                               uint16_t* __restrict__ y, float* __restrict__ part,
                                                               int N, int H, int W, int OH, int OW, int tiles_h,
                                                               int tiles_w) {
  __shared__ __attribute__((aligned(16))) uint8_t Wl[kWBytes];
  __shared__ __attribute__((aligned(16))) uint8_t Hl[kHalo];
  __shared__ __attribute__((aligned(16))) uint8_t Ol[4 * 64 * 128];  // per-wave output staging
  __shared__ __attribute__((aligned(16))) float Kl[64];
  __shared__ float red[4][64][2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l15 = lane & 15, l4 = lane >> 4;

  // weights -> LDS, chunk c = kh * 4 + q holds k = (kw = 2q + (e >> 2), ci = e & 3), e = 0..7
  for (int i = tid; i < 28 * 64; i += 256) {
    const int c = i >> 6, co = i & 63, kh = c >> 2, q = c & 3;
    uint32_t pk[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      uint32_t two = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * e2 + h, kw = 2 * q + (e >> 2), ci = e & 3;
        const uint16_t v = (kw < 7 && ci < 3) ? w[co * ws.co + ci * ws.ci + kh * ws.kh + kw * ws.kw] : (uint16_t)0;
        two |= (uint32_t)v << (16 * h);
      }
      pk[e2] = two;
    }
    *reinterpret_cast<uint4*>(Wl + (c * 64 + co) * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }

  const int ntiles = N * tiles_h * tiles_w;
  uint2 stage[kSlots];
  auto load_halo = [&](int tile) {
    const int tw = tile % tiles_w, th = (tile / tiles_w) % tiles_h, n = tile / (tiles_w * tiles_h);
    const int ih0 = th * 2 * kT - 3, iw0 = tw * 2 * kT - 3;
    const uint16_t* xn = x + (int64_t)n * H * W * 3;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int p = tid + 256 * s, hr = p / kHC, hc = p % kHC;
      const int ih = ih0 + hr, iw = iw0 + hc;
      const bool ok = p < kHR * kHC && hc < kHC - 1 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      uint32_t c01 = 0, c2 = 0;
      if (ok) {
        const uint16_t* px = xn + ((int64_t)ih * W + iw) * 3;
        c01 = (uint32_t)px[0] | ((uint32_t)px[1] << 16);
        c2 = px[2];
      }
      stage[s] = make_uint2(c01, c2);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int p = tid + 256 * s;
      if (p < kHR * kHC) *reinterpret_cast<uint2*>(Hl + p * 8) = stage[s];
    }
  };

  // statistics of channels 8u..8u+7 (u = lane & 7: the chunk this lane stores) over its pixels
  float st_s[8], st_ss[8], st_n = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) st_s[i] = st_ss[i] = 0.f;

  int tile = blockIdx.x;
  if (tile < ntiles) load_halo(tile);
  bool first = true;
  for (; tile < ntiles; tile += gridDim.x) {
    const int tw = tile % tiles_w, th = (tile / tiles_w) % tiles_h, n = tile / (tiles_w * tiles_h);
    __syncthreads();  // previous tile's halo reads are done (and, first time, the weights are in LDS)
    store_halo();
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);  // in flight during the MFMAs

    f32x4 acc[4][4];
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) acc[cf][pf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
        a[cf] = *reinterpret_cast<const bf16x8*>(Wl + ((kh * 4 + l4) * 64 + cf * 16 + l15) * 16);
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) {
        const int hr = 2 * (4 * wv + pf) + kh, hc = 2 * l15 + 2 * l4;
        b[pf] = *reinterpret_cast<const bf16x8*>(Hl + (hr * kHC + hc) * 8);
      }
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int pf = 0; pf < 4; ++pf) acc[cf][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cf], b[pf], acc[cf][pf], 0, 0, 0);
    }

    // epilogue: lane holds channels cf*16 + 4*l4 + (0..3) of pixel (row 4*wv + pf, col l15)
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
      for (int pf = 0; pf < 4; ++pf)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[cf][pf][i] = bf16r(acc[cf][pf][i]);
    if (first) {  // the statistics shift: this workgroup's first output pixel (always in the image)
      // (rounded acc: the bf16 values the statistics see)
      if (wv == 0 && l15 == 0) {
#pragma unroll
        for (int cf = 0; cf < 4; ++cf)
#pragma unroll
          for (int i = 0; i < 4; ++i) Kl[cf * 16 + 4 * l4 + i] = acc[cf][0][i];
      }
      __syncthreads();
      first = false;
    }
    const int ow = tw * kT + l15;
    // bf16 tile through this wave's LDS slice (8 KB, 16-B chunks XOR-swizzled by pixel bits 1..3
    // so both the 8-B writes and the 16-B reads are conflict-free), then full 128-B pixel rows out
    uint8_t* Os = Ol + wv * (64 * 128);
#pragma unroll
    for (int pf = 0; pf < 4; ++pf) {
      const int px = pf * 16 + l15;
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        uint2 pk;
        pk.x = dev::pack_bf16x2(acc[cf][pf][0], acc[cf][pf][1]);
        pk.y = dev::pack_bf16x2(acc[cf][pf][2], acc[cf][pf][3]);
        const int chunk = 2 * cf + (l4 >> 1);
        *reinterpret_cast<uint2*>(Os + px * 128 + ((chunk ^ ((px >> 1) & 7)) * 16) + (l4 & 1) * 8) = pk;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's slice is written (wave-local)
    const int u = lane & 7;
    float kv[8];
    dev::Vec8<float>::ld(Kl + 8 * u, kv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int px = i * 8 + (lane >> 3);
      const int oh = th * kT + 4 * wv + (px >> 4), owp = tw * kT + (px & 15);
      const dev::u32x4 v = *reinterpret_cast<const dev::u32x4*>(Os + px * 128 + ((u ^ ((px >> 1) & 7)) * 16));
      if (oh < OH && owp < OW) {
        __builtin_nontemporal_store(v, reinterpret_cast<dev::u32x4*>(y + (((int64_t)n * OH + oh) * OW + owp) * 64 + u * 8));
        st_n += 1.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = __uint_as_float(e & 1 ? (v[e >> 1] & 0xffff0000u) : (v[e >> 1] << 16)) - kv[e];
          st_s[e] += d;
          st_ss[e] = fmaf(d, d, st_ss[e]);
        }
      }
    }
  }
  if ((int)blockIdx.x >= ntiles) return;  // (no tile: nothing to report; grid <= ntiles by construction)

  // lanes sharing u = lane & 7 hold the same 8 channels: add over lane bits 3..5, then over the
  // waves through LDS (st_n: pixels this lane stored, the same count for its 8 channels)
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    st_n += __shfl_xor(st_n, o, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      st_s[e] += __shfl_xor(st_s[e], o, 64);
      st_ss[e] += __shfl_xor(st_ss[e], o, 64);
    }
  }
  __shared__ float cnt[4];
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wv][8 * lane + e][0] = st_s[e];
      red[wv][8 * lane + e][1] = st_ss[e];
    }
    if (lane == 0) cnt[wv] = st_n;
  }
  __syncthreads();
  if (tid < 64) {
    const float nn = cnt[0] + cnt[1] + cnt[2] + cnt[3];
    float S = 0.f, SS = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      S += red[v][tid][0];
      SS += red[v][tid][1];
    }
    const float mean_d = S / nn;
    part[((int64_t)blockIdx.x * 3 + 0) * 64 + tid] = nn;
    part[((int64_t)blockIdx.x * 3 + 1) * 64 + tid] = Kl[tid] + mean_d;
    part[((int64_t)blockIdx.x * 3 + 2) * 64 + tid] = fmaxf(SS - S * mean_d, 0.f);
  }
}

// ------------------------------------------------------------------------------------ wgrad
// dW[co][k] = sum over output pixels p of dY[p][co] · Xcol[p][k], k = kh·32 + kw·4 + ci, on
// mfma_f32_16x16x32_bf16 with the PIXELS as the reduction dimension:
// * A = dY^T (16 co x 32 pixels) by transposing ds_read_b64_tr_b16 from the dY tile, staged
//   global -> LDS by LDS-DMA as [pixel][64 co] rows with the 32-B blocks XOR-swizzled by two row
//   bits (the 8 rows of a half-wave transposed read hit distinct banks);
// * B = Xcol (32 pixels x 16 k): for kernel row kh and kw in 0..3 (or 4..7) the 16 k of output
//   pixel (oh, ow) are the 4 channels of the 4 adjacent halo pixels (2·oh + kh, 2·ow + kw), a
//   contiguous 32 B of the halo image — so the same transposed read builds Xcol straight from the
//   halo, no im2col;
// * a workgroup (persistent) walks 8 x 16-pixel output tiles, double-buffered (next tile's dY by
//   DMA and halo by registers while this tile's MFMAs run, one barrier per tile); wave w owns
//   co-fragments 2(w&1), 2(w&1)+1 and k-fragments 7(w>>1)..+6 of the 4 x 14 output fragments and
//   writes its fp32 partial dW once; stem_wgrad_reduce sums the workgroups.
constexpr int kWT = 8;                     // wgrad tile: kWT output rows x 16 cols
constexpr int kWHR = 2 * kWT + 5;          // halo rows
constexpr int kWHalo = kWHR * kHC * 8;     // bytes
constexpr int kWSlots = (kWHR * kHC + 255) / 256;
constexpr int kDBytes = kWT * 16 * 128;    // dY tile: 128 pixels x 64 co bf16

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ v4s lds_tr16(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}
// 32-B block swizzle of a dY tile row (4 blocks of 16 co): rows r, r+2, r+8, r+10 (the even rows of
// one half-wave transposed read) land in distinct blocks
__device__ __forceinline__ int dswz(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }

__device__ __forceinline__ float bfx(uint32_t w, int hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); }

__global__ __launch_bounds__(256, 2) void stem_conv_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                                 const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ zeros,
                                                                 float* __restrict__ ws, int N, int H, int W, int OH,
                                                                 int OW, int tiles_h, int tiles_w) {
  __shared__ __attribute__((aligned(16))) uint8_t Dl[2][kDBytes];
  __shared__ __attribute__((aligned(16))) uint8_t Hl[2][kWHalo];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l15 = lane & 15, l4 = lane >> 4;
  const int cp = wv & 1, nh = wv >> 1;
  const int ntiles = N * tiles_h * tiles_w;

  auto tile_pos = [&](int tile, int& n, int& oh0, int& ow0) {
    const int tw = tile % tiles_w, th = (tile / tiles_w) % tiles_h;
    n = tile / (tiles_w * tiles_h);
    oh0 = th * kWT;
    ow0 = tw * 16;
  };
  // dY tile -> LDS by DMA: 16 x 1-KB pieces (8 pixel rows each), 4 per wave; lane i of a piece
  // fills 16 B of row 8q + i/8 at physical 16-B unit i%8 (the source co is pre-swizzled)
  auto issue_dy = [&](int tile, int buf) {
    int n, oh0, ow0;
    tile_pos(tile, n, oh0, ow0);
#pragma unroll
    for (int i = 0; i < kDBytes / 1024 / 4; ++i) {
      const int q = wv * (kDBytes / 1024 / 4) + i, row = 8 * q + (lane >> 3), u = lane & 7;
      const int co = (((u >> 1) ^ dswz(row)) * 2 + (u & 1)) * 8;
      const int oh = oh0 + row / 16, ow = ow0 + row % 16;
      const uint16_t* src = (oh < OH && ow < OW) ? dy + (((int64_t)n * OH + oh) * OW + ow) * 64 + co : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(Dl[buf] + q * 1024), 16, 0, 0);
    }
  };
  uint2 stage[kWSlots];
  auto load_halo = [&](int tile) {
    int n, oh0, ow0;
    tile_pos(tile, n, oh0, ow0);
    const int ih0 = oh0 * 2 - 3, iw0 = ow0 * 2 - 3;
    const uint16_t* xn = x + (int64_t)n * H * W * 3;
#pragma unroll
    for (int s = 0; s < kWSlots; ++s) {
      const int p = tid + 256 * s, hr = p / kHC, hc = p % kHC;
      const int ih = ih0 + hr, iw = iw0 + hc;
      const bool ok = p < kWHR * kHC && hc < kHC - 1 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      uint32_t c01 = 0, c2 = 0;
      if (ok) {
        const uint16_t* px = xn + ((int64_t)ih * W + iw) * 3;
        c01 = (uint32_t)px[0] | ((uint32_t)px[1] << 16);
        c2 = px[2];
      }
      stage[s] = make_uint2(c01, c2);
    }
  };

  f32x4 acc[2][7];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[c][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int k = 0;
  if ((int)blockIdx.x < ntiles) {
    issue_dy(blockIdx.x, 0);
    load_halo(blockIdx.x);
  }
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++k) {
    const int buf = k & 1;
#pragma unroll
    for (int s = 0; s < kWSlots; ++s) {
      const int p = tid + 256 * s;
      if (p < kWHR * kHC) *reinterpret_cast<uint2*>(Hl[buf] + p * 8) = stage[s];
    }
    // this tile's DMA landed and every wave is done with the tile before (whose buffers the next
    // issue overwrites)
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int next = tile + gridDim.x;
    if (next < ntiles) {
      issue_dy(next, buf ^ 1);
      load_halo(next);
    }
    const uint8_t* D = Dl[buf];
    const uint8_t* X = Hl[buf];
#pragma unroll
    for (int ks = 0; ks < kWT * 16 / 32; ++ks) {
      // pixel rows of this lane's transposed reads: r0 and r0 + 4
      const int r0 = ks * 32 + 8 * l4 + (l15 >> 2);
      bf16x8 a[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int cf = 2 * cp + c;
        const v4s lo = lds_tr16(D + r0 * 128 + ((cf ^ dswz(r0)) * 32) + 8 * (lane & 3));
        const v4s hi = lds_tr16(D + (r0 + 4) * 128 + ((cf ^ dswz(r0 + 4)) * 32) + 8 * (lane & 3));
        const v4s v8[2] = {lo, hi};
        a[c] = __builtin_bit_cast(bf16x8, v8);
      }
      const int oh_a = r0 >> 4, ow_a = r0 & 15, oh_b = (r0 + 4) >> 4, ow_b = (r0 + 4) & 15;
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) {
        const int j = 7 * nh + jj, kh = j >> 1, nf = j & 1;
        const v4s lo = lds_tr16(X + ((2 * oh_a + kh) * kHC + 2 * ow_a + 4 * nf) * 8 + 8 * (lane & 3));
        const v4s hi = lds_tr16(X + ((2 * oh_b + kh) * kHC + 2 * ow_b + 4 * nf) * 8 + 8 * (lane & 3));
        const v4s v8[2] = {lo, hi};
        const bf16x8 b = __builtin_bit_cast(bf16x8, v8);
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[c][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b, acc[c][jj], 0, 0, 0);
      }
    }
  }
  // partial dW of this workgroup: lane holds co = cf*16 + 4*l4 + i, k = j*16 + l15
  float* out = ws + (int64_t)blockIdx.x * 64 * 224;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int jj = 0; jj < 7; ++jj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = (2 * cp + c) * 16 + 4 * l4 + i, kk = (7 * nh + jj) * 16 + l15;
        out[co * 224 + kk] = acc[c][jj][i];
      }
}

// Sum of the workgroups' partial dW in two steps (enough blocks to stream the partials at full
// bandwidth): stage 1 sums G/kRedSplit partials per (split, co) block into ws2[split][co][k];
// stage 2 adds the splits and writes dW[co][ci][kh][kw] in the weight's strides and dtype.
constexpr int kRedSplit = 16;

__global__ __launch_bounds__(256) void stem_wgrad_reduce1_kernel(const float* __restrict__ ws, int G,
                                                                 float* __restrict__ ws2) {
  const int co = blockIdx.x, split = blockIdx.y, k = threadIdx.x;
  if (k >= 224) return;
  const int per = (G + kRedSplit - 1) / kRedSplit, g0 = split * per, g1 = min(G, g0 + per);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int g = g0;
  for (; g + 3 < g1; g += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += ws[((int64_t)(g + u) * 64 + co) * 224 + k];
  }
  for (; g < g1; ++g) s[0] += ws[((int64_t)g * 64 + co) * 224 + k];
  ws2[((int64_t)split * 64 + co) * 224 + k] = (s[0] + s[1]) + (s[2] + s[3]);
}

template <typename T>
__global__ __launch_bounds__(256) void stem_wgrad_reduce2_kernel(const float* __restrict__ ws2, T* __restrict__ dw,
                                                                 WStrides st) {
  const int co = blockIdx.x, k = threadIdx.x;
  if (k >= 224) return;
  float v = 0.f;
#pragma unroll
  for (int sp = 0; sp < kRedSplit; ++sp) v += ws2[((int64_t)sp * 64 + co) * 224 + k];
  const int kh = k >> 5, kw = (k >> 2) & 7, ci = k & 3;
  if (kw < 7 && ci < 3) dev::Elem<T, float>::st(dw, co * st.co + ci * st.ci + kh * st.kh + kw * st.kw, v);
}

}  // namespace

// x [N, 3, H, W] channels_last bf16, w [64, 3, 7, 7] bf16 (any strides) -> (y [N, 64, OH, OW]
// channels_last, partials [groups, 3, 64] = (count, mean, M2) of y per workgroup)
std::vector<at::Tensor> stem_conv_forward(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) == 3 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_conv_forward: x must be a channels_last bf16 [N, 3, H, W] GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 &&
                  w.size(2) == 7 && w.size(3) == 7,
              "stem_conv_forward: w must be bf16 [64, 3, 7, 7]");
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int tiles_h = (OH + kT - 1) / kT, tiles_w = (OW + kT - 1) / kT;
  const int64_t ntiles = (int64_t)N * tiles_h * tiles_w;
  TORCH_CHECK(ntiles > 0 && ntiles < (1 << 30), "stem_conv_forward: bad size");
  auto y = at::empty({N, 64, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  int dev_id = x.device().index(), cus = 0;
  XDDP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id));
  const int grid = (int)std::min<int64_t>(ntiles, 2 * (int64_t)cus);
  auto part = at::empty({grid, 3, 64}, x.options().dtype(at::kFloat));
  auto stream = c10::hip::getCurrentHIPStream(dev_id).stream();
  WStrides ws{w.stride(0), w.stride(1), w.stride(2), w.stride(3)};
  hipLaunchKernelGGL(stem_conv_fwd_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                     ws, reinterpret_cast<uint16_t*>(y.data_ptr()), part.data_ptr<float>(), N, H, W, OH, OW, tiles_h,
                     tiles_w);
  XDDP_HIP_CHECK(hipGetLastError());
  return {y, part};
}

}  // namespace kernels
}  // namespace xddp

namespace xddp {
namespace kernels {

namespace {
at::Tensor stem_wgrad_reduce(const at::Tensor& ws, int grid, const at::Tensor& w_like, hipStream_t stream);
}

// dY [N, 64, OH, OW] channels_last bf16, x [N, 3, H, W] channels_last bf16 -> dW like w_like
at::Tensor stem_conv_wgrad(const at::Tensor& dy_in, const at::Tensor& x, const at::Tensor& w_like) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) == 3 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_conv_wgrad: x must be a channels_last bf16 [N, 3, H, W] GPU tensor");
  auto dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.size(0) == N && dy.size(1) == 64 && dy.size(2) == OH &&
                  dy.size(3) == OW,
              "stem_conv_wgrad: dy must be bf16 [N, 64, OH, OW]");
  TORCH_CHECK(w_like.dim() == 4 && w_like.size(0) == 64 && w_like.size(1) == 3 && w_like.size(2) == 7 &&
                  w_like.size(3) == 7,
              "stem_conv_wgrad: w must be [64, 3, 7, 7]");
  const int tiles_h = (OH + kWT - 1) / kWT, tiles_w = (OW + 15) / 16;
  const int64_t ntiles = (int64_t)N * tiles_h * tiles_w;
  TORCH_CHECK(ntiles > 0 && ntiles < (1 << 30), "stem_conv_wgrad: bad size");
  int dev_id = x.device().index(), cus = 0;
  XDDP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id));
  const int grid = (int)std::min<int64_t>(ntiles, 2 * (int64_t)cus);
  auto ws = at::empty({grid, 64, 224}, x.options().dtype(at::kFloat));
  auto zeros = at::zeros({64}, x.options());
  auto stream = c10::hip::getCurrentHIPStream(dev_id).stream();
  hipLaunchKernelGGL(stem_conv_wgrad_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                     reinterpret_cast<const uint16_t*>(zeros.data_ptr()), ws.data_ptr<float>(), N, H, W, OH, OW,
                     tiles_h, tiles_w);
  XDDP_HIP_CHECK(hipGetLastError());
  return stem_wgrad_reduce(ws, grid, w_like, stream);
}

namespace {
at::Tensor stem_wgrad_reduce(const at::Tensor& ws, int grid, const at::Tensor& w_like, hipStream_t stream) {
  auto dw = at::empty_like(w_like);
  WStrides st{dw.stride(0), dw.stride(1), dw.stride(2), dw.stride(3)};
  auto ws2 = at::empty({kRedSplit, 64, 224}, ws.options());
  hipLaunchKernelGGL(stem_wgrad_reduce1_kernel, dim3(64, kRedSplit), dim3(256), 0, stream, ws.data_ptr<float>(), grid,
                     ws2.data_ptr<float>());
  XDDP_HIP_CHECK(hipGetLastError());
  auto go = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((stem_wgrad_reduce2_kernel<T>), dim3(64), dim3(256), 0, stream, ws2.data_ptr<float>(),
                       reinterpret_cast<T*>(dw.data_ptr()), st);
    XDDP_HIP_CHECK(hipGetLastError());
  };
  switch (dw.scalar_type()) {
    case at::kBFloat16: go(dev::bf16_t{}); break;
    case at::kFloat: go(float{}); break;
    default: TORCH_CHECK(false, "stem_conv_wgrad: weight dtype must be bf16 or fp32");
  }
  return dw;
}
}  // namespace

}  // namespace kernels
}  // namespace xddp
