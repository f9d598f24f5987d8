// 3x3 convolution (NHWC, bf16, pad 1, stride 1 or 2) as an implicit MFMA GEMM for gfx950, with
// the following BatchNorm's batch statistics optionally produced by its epilogue.
//
//   Y[M, N] = sum over taps (r, s) and channels c of X[pix(m) + (r-1, s-1), c] · W[n, r, s, c]
//   M = batch·OH·OW output pixels, N = Cout, reduction K = 9·Cin walked as 9 taps x Cin/64 steps.
//
// The same kernel computes the stride-1 input gradient: dX = conv(dY, W') with W'[c, r, s, n] =
// W[n, 2-r, 2-s, c] (a 180-degree rotation and an in/out channel swap of the small weight).
//
// Why a different structure from the 1x1 GEMM (conv_gemm.hip): the ResNet-50 3x3 convs are
// compute-bound (K = 576..4608), where register staging costs VGPRs and LDS-store issue slots
// the MFMAs need. Here both operands go global -> LDS directly with global_load_lds_dwordx4
// (LDS-DMA, no VGPR round trip): each wave-instruction fills 8 full 128-B rows, the per-lane
// SOURCE address is pre-swizzled so the LDS image has the XOR-swizzled chunk order the
// ds_read_b128 fragment reads want (the DMA destination itself is lane-linear). Padding taps
// and rows past M point their lanes at a zero line instead of branching. Three LDS stages: at
// step k the loads of steps k+1 and k+2 are in flight; a counted `s_waitcnt vmcnt(LPS)` +
// raw s_barrier (never vmcnt(0) inside the loop) retires step k's stage for every wave.
// One block per CU (64x64 output per wave = 16 accumulators, 2 waves per SIMD), block ids
// remapped XCD-contiguously so the N-tiles of one M-panel and neighbouring panels (which share
// input rows through the 3x3 halo) sit in one L2. Since r5 it runs the shapes the row-band kernel
// (conv3x3_band.hip) and the dense-GEMM path do not: stride 2 at N < 256, W > 56 or odd channel
// counts, and the stride-2 input gradient's generic (odd-size) case.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"
#include "kernels/norm.h"

namespace xddp {
namespace kernels {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
using dev::f32x4;
using dev::u32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kStages = 3;

__device__ __forceinline__ int swz3(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }
__device__ __forceinline__ float round_bf16(float v) { return __uint_as_float(dev::pack_bf16x2(v, 0.f) << 16); }

struct Geo3 {
  int IH, IW, OH, OW, stride;
};

// DG2 (stride-2 input gradient, pad 1): dX pixel (2p + a, 2q + b) only receives the taps whose
// forward window put it under dY pixel (p + di, q + dj): a = 0 -> tap row 1 (di = 0); a = 1 -> tap
// rows 0 (di = 1) and 2 (di = 0); columns alike. So dX splits into four phase grids, each an
// implicit GEMM over dY with 1, 2, 2 or 4 taps of the rotated weights (4 of 9 MACs a pixel, no zero
// insertion), its rows scattered to the strided output pixels. All four phases share one launch,
// heaviest first: block tiles [start[k], start[k+1]) belong to phase k = (a, b) in order
// (1,1), (1,0), (0,1), (0,0).
struct Dg2Geo {
  int B, H, W;       // dX batch and spatial size (geo.IH / IW are dY's)
  int start[4];      // first block tile of each phase
};

// TAPS = 9: the 3x3 conv (pad 1). (TAPS = 1, a 1x1 conv on this pipeline, lost its r2 A/B to the
// register-staged 1x1 GEMM and the deep-K LDS-DMA GEMM; its entry point was removed in r5.) Earlier
// rationale: the K loop of the register-staged 1x1 GEMM (conv_gemm.hip) waits a
// full memory latency per 64-deep step, which dominates the deep-K / few-tile layers (ResNet-50
// layer3/4: K = 1024..2048 with 400-800 output tiles).
template <int BM, int BN, int WM, int WN, bool STATS, int TAPS = 9, bool DG2 = false>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv3x3_fwd_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y,
    const uint16_t* __restrict__ zeros, int M, int N, int C, Geo3 geo, float* __restrict__ part, int ntiles,
    Dg2Geo dg) {
  static_assert(!DG2 || (TAPS == 9 && !STATS), "the stride-2 input gradient is a 3x3 tap walk without stats");
  constexpr int NT = 64 * WM * WN, NW = NT / 64;
  constexpr int AI = BM / 8 / NW, BI = BN / 8 / NW;  // DMA wave-instructions per stage (8 rows each)
  static_assert(AI * NW * 8 == BM && BI * NW * 8 == BN, "tile rows must split evenly over the waves");
  constexpr int LPS = AI + BI;                        // vmcnt units per stage per thread
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE = (BM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  int wg = dev::xcd_remap(blockIdx.x, gridDim.x);
  int pa = 0, pb = 0, PH = geo.OH, PW = geo.OW, Mk = M;  // DG2: this block's phase and its grid
  if (DG2) {
    const int k = (wg >= dg.start[1]) + (wg >= dg.start[2]) + (wg >= dg.start[3]);
    wg -= dg.start[k];
    pa = k < 2;
    pb = !(k & 1);
    PH = (dg.H - pa + 1) >> 1;
    PW = (dg.W - pb + 1) >> 1;
    Mk = dg.B * PH * PW;
  }
  const int nt = wg % ntiles, mt = wg / ntiles;
  const int n0 = nt * BN, m0 = mt * BM;
  constexpr int PAD = TAPS == 9 && !DG2 ? 1 : 0;
  const int ntaps = DG2 ? (1 + pa) * (1 + pb) : TAPS;
  const int cb_n = C >> 6, nk = ntaps * cb_n;
  const int pos = lane & 7;  // 16-B slot this lane fills in its 128-B LDS row

  // A rows: output pixel -> top-left input pixel of its 3x3 window (may be outside the image)
  int ih0[AI], iw0[AI];
  int64_t aoff[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wid * AI + i) * 8 + (lane >> 3);
    const int m = m0 + row;
    const int hw = PH * PW;
    const int b = m / hw, rem = m - b * hw, oh = rem / PW, ow = rem - oh * PW;
    const int st = DG2 ? 1 : geo.stride;  // DG2: phase pixel (p, q) reads dY from (p, q) on
    ih0[i] = m < Mk ? oh * st - PAD : -4;  // rows past M: every tap out of bounds -> zeros
    iw0[i] = ow * st - PAD;
    aoff[i] = (((int64_t)b * geo.IH + ih0[i]) * geo.IW + iw0[i]) * C + 8 * (pos ^ ((row >> 1) & 7));
  }
  int64_t boff[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int row = (wid * BI + j) * 8 + (lane >> 3);
    boff[j] = (int64_t)(n0 + row) * TAPS * C + 8 * (pos ^ ((row >> 1) & 7));
  }

  auto issue = [&](int kt, int buf) {
    int t = TAPS == 1 ? 0 : kt / cb_n;
    const int cb = kt - t * cb_n;
    int r = t / 3, s = t - 3 * r;  // A-operand offset of the tap (rows, columns)
    if (DG2) {  // t-th tap of the phase: forward tap (fr, fs), rotated-weight index 8 - (3 fr + fs)
      const int rr = pb ? t >> 1 : t, sr = pb ? t & 1 : 0;
      const int fr = pa ? 2 * rr : 1, fs = pb ? 2 * sr : 1;  // a = 1: rows 0 and 2; a = 0: row 1
      r = fr == 0;
      s = fs == 0;
      t = 8 - (3 * fr + fs);
    }
    uint8_t* A = smem + buf * STAGE;
    const int64_t tap = ((int64_t)r * geo.IW + s) * C + cb * 64;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = (unsigned)(ih0[i] + r) < (unsigned)geo.IH && (unsigned)(iw0[i] + s) < (unsigned)geo.IW;
      const uint16_t* src = ok ? X + aoff[i] + tap : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(A + (wid * AI + i) * 1024), 16, 0, 0);
    }
    uint8_t* B = A + BM * 128;
    const int64_t wk = (int64_t)t * C + cb * 64;
#pragma unroll
    for (int j = 0; j < BI; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(Wt + boff[j] + wk), (lds_ptr_t)(B + (wid * BI + j) * 1024), 16,
                                       0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    // retire step kt's stage (step kt+1's may stay in flight), then make every wave's DMA
    // visible: after this barrier no wave still reads the stage that step kt+2 overwrites
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % kStages);
    const uint8_t* A = smem + (kt % kStages) * STAGE;
    const uint8_t* B = A + BM * 128;
    // all fragments of the 64-deep step first: the second half's LDS reads overlap the first
    // half's MFMAs (the compiler counts lgkmcnt down per use)
    bf16x8 a[2][TM], b[2][TN];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[h][i] = *reinterpret_cast<const bf16x8*>(A + swz3(wm * WTM + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j) b[h][j] = *reinterpret_cast<const bf16x8*>(B + swz3(wn * WTN + j * 16 + (lane & 15), ch));
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[h][j], a[h][i], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: bf16 C tile through LDS (rows padded 16 B), 16-B row stores ----
  // (the MFMA above computes the transposed tile: a lane's 4 accumulators are 4 consecutive
  // output channels of one pixel, stored as one 8-B LDS write)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done reading the stages
  constexpr int CST = BN * 2 + 16;
  static_assert(BM * CST <= kStages * STAGE, "C tile must fit in the stage buffers");
  uint8_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wm * WTM + i * 16 + (lane & 15);
      const int col = wn * WTN + j * 16 + (lane >> 4) * 4;
      uint2 pk;
      pk.x = dev::pack_bf16x2(acc[i][j][0], acc[i][j][1]);
      pk.y = dev::pack_bf16x2(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(Cs + row * CST + col * 2) = pk;
    }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "readout mapping needs a fixed chunk column per thread");
  const int cc = tid % CPR;
  const int rows_valid = min(BM, Mk - m0);
  float st_n = 0.f, st_s[8], st_ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) st_s[e] = st_ss[e] = 0.f;
  const u32x4 st_k = *reinterpret_cast<const u32x4*>(Cs + cc * 16);  // row 0 (always valid): the shift
  // rows tid / CPR + (NT / CPR)·i; each batch's LDS reads issued before its stores (rows past M read
  // row rows_valid - 1 and are not stored): a read-then-use per row inside `if (row < rows_valid)`
  // compiled to one ds_read + s_waitcnt lgkmcnt(0) round trip per row
  constexpr int NIT = BM * CPR / NT, RSTR = NT / CPR, EB = NIT < 4 ? NIT : 4;
  static_assert(BM * CPR % NT == 0, "readout rows must divide evenly over the threads");
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += EB) {
    u32x4 vv[EB];
#pragma unroll
    for (int j = 0; j < EB; ++j)
      if (i0 + j < NIT)
        vv[j] = *reinterpret_cast<const u32x4*>(Cs + min(tid / CPR + RSTR * (i0 + j), rows_valid - 1) * CST + cc * 16);
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int row = tid / CPR + RSTR * (i0 + j);
      if (i0 + j < NIT && row < rows_valid) {
        const u32x4 v = vv[j];
        int64_t yrow = m0 + row;
        if (DG2) {  // phase pixel -> dX pixel (2p + a, 2q + b)
          const int hw = PH * PW, m = m0 + row, b = m / hw, rem = m - b * hw, p = rem / PW, q = rem - p * PW;
          yrow = ((int64_t)b * dg.H + 2 * p + pa) * dg.W + 2 * q + pb;
        }
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(Y + yrow * N + n0 + cc * 8));
        if (STATS) {
          st_n += 1.f;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const float d0 = __uint_as_float(v[h] << 16) - __uint_as_float(st_k[h] << 16);
            const float d1 = __uint_as_float(v[h] & 0xffff0000u) - __uint_as_float(st_k[h] & 0xffff0000u);
            st_s[2 * h] += d0;
            st_s[2 * h + 1] += d1;
            st_ss[2 * h] = fmaf(d0, d0, st_ss[2 * h]);
            st_ss[2 * h + 1] = fmaf(d1, d1, st_ss[2 * h + 1]);
          }
        }
      }
    }
  }
  if (!STATS) return;
  // every thread of the block shifted by the same row-0 values, so the shifted sums simply add:
  // lanes sharing cc (xor over the lane bits above log2(CPR)), then the waves through LDS; one
  // (count, mean, M2) per channel and block, stored group-minor: part[q][N][mtiles]
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1) {
    st_n += __shfl_xor(st_n, o, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      st_s[e] += __shfl_xor(st_s[e], o, 64);
      st_ss[e] += __shfl_xor(st_ss[e], o, 64);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // C tile reads done: reuse smem
  float* red = reinterpret_cast<float*>(smem);                      // [NW][2][BN] sums, [NW][CPR] counts
  float* redn = red + NW * 2 * BN;
  float* redk = redn + NW * CPR;                                    // [BN] the shifts
  if (lane < CPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wid * 2 + 0) * BN + cc * 8 + e] = st_s[e];
      red[(wid * 2 + 1) * BN + cc * 8 + e] = st_ss[e];
      if (wid == 0)
        redk[cc * 8 + e] = __uint_as_float((e & 1) ? (st_k[e >> 1] & 0xffff0000u) : (st_k[e >> 1] << 16));
    }
    redn[wid * CPR + cc] = st_n;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const int G = gridDim.x / ntiles;
  for (int c = tid; c < BN; c += NT) {
    float tn = 0.f, ts = 0.f, tss = 0.f;
    for (int w = 0; w < NW; ++w) {
      tn += redn[w * CPR + c / 8];
      ts += red[(w * 2 + 0) * BN + c];
      tss += red[(w * 2 + 1) * BN + c];
    }
    const float mean_s = ts / tn;  // tn >= 1: row 0 is always valid
    part[((int64_t)0 * N + n0 + c) * G + mt] = tn;
    part[((int64_t)1 * N + n0 + c) * G + mt] = redk[c] + mean_s;
    part[((int64_t)2 * N + n0 + c) * G + mt] = fmaxf(tss - ts * mean_s, 0.f);
  }
}

// W'[c][t][n] = W[n][8 - t][c] (OHWI in, OHWI out): the stride-1 input-gradient weights. One
// 64x64 (n, c) tile of one tap per block, transposed through LDS.
__global__ __launch_bounds__(256) void rot_weight_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ out,
                                                         int N, int C) {
  __shared__ uint16_t tile[64][66];
  const int n0 = blockIdx.x * 64, c0 = blockIdx.y * 64, t = blockIdx.z;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;  // read rows n, contiguous c
    tile[r][c] = w[((int64_t)(n0 + r) * 9 + (8 - t)) * C + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, n = i & 63;  // write rows c, contiguous n
    out[((int64_t)(c0 + r) * 9 + t) * N + n0 + n] = tile[n][r];
  }
}

// Several weights in one launch (the model's 3x3 weights once per step, ops/conv_bn.py): block b
// belongs to the tensor whose first block is the largest start <= b, then runs as above.
constexpr int kRotMax = 32;
struct RotBatch {
  const uint16_t* w[kRotMax];
  uint16_t* out[kRotMax];
  int N[kRotMax], C[kRotMax], start[kRotMax + 1];
  int count;
};

__global__ __launch_bounds__(256) void rot_weights_kernel(RotBatch rb) {
  __shared__ uint16_t tile[64][66];
  int e = 0;
  while (e + 1 < rb.count && (int)blockIdx.x >= rb.start[e + 1]) ++e;
  const int N = rb.N[e], C = rb.C[e], local = (int)blockIdx.x - rb.start[e];
  const int nb = N / 64, cb = C / 64;
  const int t = local / (nb * cb), rem = local - t * nb * cb, c0 = (rem / nb) * 64, n0 = (rem % nb) * 64;
  const uint16_t* w = rb.w[e];
  uint16_t* out = rb.out[e];
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    tile[r][c] = w[((int64_t)(n0 + r) * 9 + (8 - t)) * C + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, n = i & 63;
    out[((int64_t)(c0 + r) * 9 + t) * N + n0 + n] = tile[n][r];
  }
}

const uint16_t* zero_line(const at::Tensor& like) {
  // 256 zero bytes per device that padding lanes read instead of branching; never freed (a
  // static tensor would be destroyed after the HIP runtime at exit)
  static at::Tensor* z[64] = {};
  const int d = like.device().index();
  TORCH_CHECK(d >= 0 && d < 64, "conv3x3: device index out of range");
  if (!z[d]) z[d] = new at::Tensor(at::zeros({128}, like.options().dtype(at::kBFloat16)));
  return reinterpret_cast<const uint16_t*>(z[d]->data_ptr());
}

// Block tile (r1/r2 A/Bs on the ResNet-50 shapes, fixed since): 256x128 (8 waves, one block per
// CU) when N % 128 == 0, else 128x64 (4 waves, two blocks per CU) for the 64-channel layers.
int tile_choice(int N) { return N % 128 == 0 ? 0 : 4; }

}  // namespace

// the band kernel with an explicit band height (timing scripts, tests)
std::vector<at::Tensor> conv3x3_band_forward(const at::Tensor& x, const at::Tensor& w, bool stats, int64_t rows,
                                             int64_t cfg) {
  return conv3x3_band(x, w, stats, rows, zero_line(x), cfg);
}

// x [B, C, IH, IW] bf16 channels_last; w [N, C, 3, 3] bf16 channels_last (OHWI memory);
// returns {y [B, N, OH, OW] channels_last, stats partials [3, N, mtiles] (group-minor; empty if
// !stats)}.
std::vector<at::Tensor> conv3x3_forward(const at::Tensor& x, const at::Tensor& w, int64_t stride, bool stats) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_forward: x must be a bf16 channels_last CUDA tensor");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) == x.size(1),
              "conv3x3_forward: w must be bf16 [N, C, 3, 3] channels_last");
  TORCH_CHECK(stride == 1 || stride == 2, "conv3x3_forward: stride 1 or 2");
  const int64_t B = x.size(0), C = x.size(1), IH = x.size(2), IW = x.size(3), N = w.size(0);
  TORCH_CHECK(C % 64 == 0 && N % 64 == 0, "conv3x3_forward: channel counts must be multiples of 64");
  TORCH_CHECK(x.data_ptr() != nullptr && (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(w.data_ptr()) % 16) == 0,
              "conv3x3_forward: 16-B aligned operands required");
  const int64_t OH = (IH - 1) / stride + 1, OW = (IW - 1) / stride + 1, M = B * OH * OW;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "conv3x3_forward: bad size");
  // stride-1 layers whose rows tile into 224 / 196-pixel bands (W = 56 / 28 / 14): the row-band
  // kernel (conv3x3_band.hip; it replaced r3's whole-row halo kernel: 101 / 62 / 58 vs 108 / 91 /
  // 70 us forward at the ResNet-50 bs256 shapes)
  if (stride == 1 && IW >= 14 && (N == 64 || N % 128 == 0) && conv3x3_band_rows(IW, IH, N == 64 ? 224 : 208) > 0 &&
      x.numel() < (int64_t(1) << 31) && M * N < (int64_t(1) << 31))
    return conv3x3_band(x, w, stats, 0, zero_line(x));
  // N % 128 == 0 (the W = 7 stride-1 layer, the stride-2 layers) on the dense GEMM's 4-phase LDS-DMA
  // pipeline with im2col addressing (gemm.hip ConvGeo)
  // (r5: N = 128 too — the stride-2 layer2.0 conv2, 98.5 vs 105.9 us on conv3x3_fwd_kernel)
  if (N >= 128 && N % 128 == 0 && x.numel() < (int64_t(1) << 31) && ((C / 64) & (C / 64 - 1)) == 0)
    return conv3x3_gemm(x, w, stride, stats, zero_line(x));
  auto y = at::empty({B, N, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int cfg = tile_choice((int)N);
  const int BM = cfg == 1 || cfg == 3 || cfg == 4 ? 128 : 256, BN = cfg <= 1 ? 128 : 64;
  const int mtiles = (int)((M + BM - 1) / BM), ntiles = (int)(N / BN);
  auto part = stats ? at::empty({3, N, mtiles}, x.options().dtype(at::kFloat)) : at::empty({0}, x.options().dtype(at::kFloat));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  Geo3 geo{(int)IH, (int)IW, (int)OH, (int)OW, (int)stride};
  const uint16_t* zeros = zero_line(x);
  auto go = [&](auto kern, int nt, size_t lds) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(mtiles * ntiles), dim3(nt), lds, stream,
                       reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()), zeros, (int)M, (int)N, (int)C, geo,
                       stats ? part.data_ptr<float>() : nullptr, ntiles, Dg2Geo{});
    XDDP_HIP_CHECK(hipGetLastError());
  };
#define XDDP_C3(BM_, BN_, WM_, WN_)                                                                             \
  do {                                                                                                           \
    const size_t lds = (size_t)kStages * (BM_ + BN_) * 128;                                                      \
    if (stats) go(conv3x3_fwd_kernel<BM_, BN_, WM_, WN_, true>, 64 * WM_ * WN_, lds);                           \
    else go(conv3x3_fwd_kernel<BM_, BN_, WM_, WN_, false>, 64 * WM_ * WN_, lds);                                \
  } while (0)
  switch (cfg) {
    case 0: XDDP_C3(256, 128, 4, 2); break;
    case 4: XDDP_C3(128, 64, 2, 2); break;
    default: TORCH_CHECK(false, "conv3x3_forward: bad tile config");
  }
#undef XDDP_C3
  return {y, part};
}

// Stride-2 input gradient of conv3x3_forward(x, w, 2): dy [B, N, OH, OW] bf16 channels_last,
// w_rot = conv3x3_rot_weight(w) ([C, N, 3, 3]); returns dx [B, C, H, W] channels_last (every pixel
// written: each phase covers its pixels, taps past dY read the zero line).
at::Tensor conv3x3_dgrad_s2(const at::Tensor& dy, const at::Tensor& w_rot, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_dgrad_s2: dy must be a bf16 channels_last CUDA tensor");
  TORCH_CHECK(w_rot.scalar_type() == at::kBFloat16 && w_rot.dim() == 4 && w_rot.size(2) == 3 && w_rot.size(3) == 3 &&
                  w_rot.is_contiguous(at::MemoryFormat::ChannelsLast) && w_rot.size(1) == dy.size(1),
              "conv3x3_dgrad_s2: w_rot must be bf16 [C, N, 3, 3] channels_last (conv3x3_rot_weight)");
  const int64_t B = dy.size(0), N = dy.size(1), OH = dy.size(2), OW = dy.size(3), C = w_rot.size(0);
  TORCH_CHECK(H >= 1 && W >= 1 && (H - 1) / 2 + 1 == OH && (W - 1) / 2 + 1 == OW,
              "conv3x3_dgrad_s2: (H, W) must be a stride-2 pad-1 input of dy's size");
  TORCH_CHECK(C % 64 == 0 && N % 64 == 0, "conv3x3_dgrad_s2: channel counts must be multiples of 64");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(w_rot.data_ptr()) % 16) == 0,
              "conv3x3_dgrad_s2: 16-B aligned operands required");
  TORCH_CHECK(B * H * W < (int64_t(1) << 31) && dy.numel() < (int64_t(1) << 40), "conv3x3_dgrad_s2: bad size");
  // even input sizes (every ResNet stride-2 3x3): the four phase GEMMs on the dense GEMM's 4-phase
  // LDS-DMA pipeline, one launch, written straight to the strided pixels (gemm.hip DGS2)
  if (H == 2 * OH && W == 2 * OW && C % 128 == 0 && ((N / 64) & (N / 64 - 1)) == 0 && dy.numel() < (int64_t(1) << 31))
    return conv3x3_dgrad_s2_gemm(dy, w_rot, H, W, zero_line(dy));
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int cfg = tile_choice((int)C);
  const int BM = cfg == 1 || cfg == 3 || cfg == 4 ? 128 : 256, BN = cfg <= 1 ? 128 : 64;
  const int ntiles = (int)(C / BN);
  Dg2Geo dg{(int)B, (int)H, (int)W, {0, 0, 0, 0}};
  int total = 0;
  for (int k = 0; k < 4; ++k) {  // (a, b) = (1,1), (1,0), (0,1), (0,0)
    const int a = k < 2, b = !(k & 1);
    const int64_t mk = B * ((H - a + 1) / 2) * ((W - b + 1) / 2);
    dg.start[k] = total;
    total += (int)((mk + BM - 1) / BM) * ntiles;
  }
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  Geo3 geo{(int)OH, (int)OW, (int)OH, (int)OW, 1};
  const uint16_t* zeros = zero_line(dy);
  auto go = [&](auto kern, int nt, size_t lds) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(total), dim3(nt), lds, stream, reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                       reinterpret_cast<const uint16_t*>(w_rot.data_ptr()), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                       zeros, 0, (int)C, (int)N, geo, nullptr, ntiles, dg);
    XDDP_HIP_CHECK(hipGetLastError());
  };
#define XDDP_D2(BM_, BN_, WM_, WN_) \
  go(conv3x3_fwd_kernel<BM_, BN_, WM_, WN_, false, 9, true>, 64 * WM_ * WN_, (size_t)kStages * (BM_ + BN_) * 128)
  switch (cfg) {
    case 0: XDDP_D2(256, 128, 4, 2); break;
    case 4: XDDP_D2(128, 64, 2, 2); break;
    default: TORCH_CHECK(false, "conv3x3_dgrad_s2: bad tile config");
  }
#undef XDDP_D2
  return dx;
}

// w [N, C, 3, 3] channels_last -> [C, N, 3, 3] channels_last rotated by 180 degrees, so that
// conv3x3_forward(dY, rot, 1) is the stride-1 input gradient of conv3x3_forward(X, w, 1).
at::Tensor conv3x3_rot_weight(const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_rot_weight: w must be bf16 [N, C, 3, 3] channels_last");
  const int64_t N = w.size(0), C = w.size(1);
  TORCH_CHECK(N % 64 == 0 && C % 64 == 0, "conv3x3_rot_weight: channel counts must be multiples of 64");
  auto out = at::empty({C, N, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(w.device().index()).stream();
  hipLaunchKernelGGL(rot_weight_kernel, dim3(N / 64, C / 64, 9), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()),
                     (int)N, (int)C);
  XDDP_HIP_CHECK(hipGetLastError());
  return out;
}

// conv3x3_rot_weight of every tensor in ws (same device) in one launch per 32 tensors
std::vector<at::Tensor> conv3x3_rot_weights(const std::vector<at::Tensor>& ws) {
  std::vector<at::Tensor> outs;
  outs.reserve(ws.size());
  for (size_t i0 = 0; i0 < ws.size(); i0 += kRotMax) {
    RotBatch rb{};
    int total = 0;
    const size_t i1 = std::min(ws.size(), i0 + kRotMax);
    for (size_t i = i0; i < i1; ++i) {
      const at::Tensor& w = ws[i];
      TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 &&
                      w.size(3) == 3 && w.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                      w.device() == ws[i0].device(),
                  "conv3x3_rot_weights: bf16 [N, C, 3, 3] channels_last weights on one device expected");
      const int64_t N = w.size(0), C = w.size(1);
      TORCH_CHECK(N % 64 == 0 && C % 64 == 0, "conv3x3_rot_weights: channel counts must be multiples of 64");
      outs.push_back(at::empty({C, N, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast)));
      const int e = (int)(i - i0);
      rb.w[e] = reinterpret_cast<const uint16_t*>(w.data_ptr());
      rb.out[e] = reinterpret_cast<uint16_t*>(outs.back().data_ptr());
      rb.N[e] = (int)N;
      rb.C[e] = (int)C;
      rb.start[e] = total;
      total += (int)((N / 64) * (C / 64) * 9);
    }
    rb.count = (int)(i1 - i0);
    rb.start[rb.count] = total;
    auto stream = c10::hip::getCurrentHIPStream(ws[i0].device().index()).stream();
    hipLaunchKernelGGL(rot_weights_kernel, dim3(total), dim3(256), 0, stream, rb);
    XDDP_HIP_CHECK(hipGetLastError());
  }
  return outs;
}

}  // namespace kernels
}  // namespace xddp
