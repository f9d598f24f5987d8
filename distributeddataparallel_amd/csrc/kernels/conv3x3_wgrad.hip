// 3x3 convolution weight gradient (NHWC, bf16, pad 1, stride 1 or 2) on gfx950 MFMA.
//
//   dW[n][r][s][c] = sum over output pixels p of dY[p][n] · X[in(p) + (r-1, s-1)][c]
//
// The reduction runs over B·OH·OW output pixels, the output is tiny (N x 9·Cin). MIOpen runs it
// as a split-K implicit GEMM whose column tiles each see one tap, re-reading dY for every tap and
// zero-filling its atomically accumulated output first (~2 ms of a ResNet-50 bs256 step). Here a
// block owns a 64 (n) x 9 (taps) x 64 (c) output tile and walks the pixels in 8x8 output patches:
// per patch it stages the dY patch (64 pixels x 64 n) and the X halo that all 9 taps read
// (10x10 pixels at stride 1, 17x17 at stride 2) ONCE, and every tap's MFMAs read their shifted
// pixel rows out of that halo. Per 64-pixel step: 21 KB (stride 1) staged for 4.7 MFLOP.
//
// * Both operands go global -> LDS with global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip);
//   a wave-instruction fills 8 pixel rows of 128 B (64 channels). Rows outside the image (or past
//   the patch grid) read a zero line instead of branching. Three (stride 1) or two (stride 2)
//   LDS stages, counted `s_waitcnt vmcnt` + raw s_barrier.
// * MFMA operands are read with gfx950's transposing ds_read_b64_tr_b16: the staged rows are
//   pixel-major ([pixel][channel], as in HBM) and the MFMA wants channel-major fragments with the
//   pixels along K. Bank conflicts are avoided by an XOR swizzle of the 32-B chunk pair on the
//   pixel's 2-D coordinates ((x & 3) ^ (y & 1)): the 4 rows one 16-lane group reads land on
//   distinct banks, and the two groups of a half-wave (adjacent pixel rows) on complementary
//   ones. At stride 2 the halo is stored phase-split (even/odd rows and columns), so the 4 pixels
//   a group reads are consecutive LDS rows as at stride 1.
// * 4 waves; wave w owns input channels c0 + 16w..+15 for all 64 n and all 9 taps: 36 MFMA tiles,
//   144 fp32 accumulators per lane (one 256-thread block per SIMD pair).
// * Each block reduces its patch range into an fp32 slab; a second kernel sums the slabs (no
//   zero-fill, no atomics, bitwise reproducible) and casts to the weight dtype.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
using dev::f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kP = 8;  // output patch edge (8x8 = 64 pixels = two 32-deep MFMA k-steps)

__device__ __forceinline__ v4s lds_tr16(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// XOR applied to a row's 32-B chunk-pair index (0..3), from the pixel's 2-D LDS coordinates
__device__ __forceinline__ int swp(int y, int x) { return (x & 3) ^ (y & 1); }

// NB = output channels (n) per block: 64 (4 waves, one 16-channel c slice each) or 128 (stride 2:
// 8 waves, wave w owns n half w >> 2 and c slice w & 3). At stride 2 the staged X halo (289
// pixels per 64 output pixels) dominates the bytes per stage; sharing it between two n halves
// halves the staging per MFMA and puts two waves on each SIMD.
template <int ST, int NB = 64>
struct Halo {
  static constexpr int NW = NB / 16;                     // waves: 4 | 8
  // phases: 1 (stride 1) or 4 (stride 2: (row parity, column parity)); each phase an IYN x 10 grid
  static constexpr int PHASES = ST == 1 ? 1 : 4;
  static constexpr int IYN = ST == 1 ? kP + 2 : kP + 1;  // 10 | 9 (valid columns: the same)
  static constexpr int IXW = 10;                         // row pitch of a phase grid (even: see swp)
  static constexpr int ROWS = PHASES * IYN * IXW;        // 100 | 360 LDS rows
  static constexpr int INSTR = (ROWS + 7) / 8;           // DMA wave-instructions (8 rows each)
  static constexpr int PER_WAVE = (INSTR + NW - 1) / NW; // 4 | 12 (NB 64), 6 (NB 128)
  static constexpr int BROWS = PER_WAVE * NW * 8;        // 128 | 384 rows reserved
  static constexpr int STAGES = ST == 1 ? 3 : 2;
  static constexpr int STAGE = (NB + BROWS) * 128;       // bytes per stage (dY rows: NB / 64 images)
  // LDS row of halo pixel (hy, hx) (0 <= hy < (kP-1)·ST+3)
  __device__ static int row(int hy, int hx) {
    if (ST == 1) return hy * IXW + hx;
    return (((hy & 1) * 2 + (hx & 1)) * IYN + (hy >> 1)) * IXW + (hx >> 1);
  }
  __device__ static int ycoord(int hy) { return ST == 1 ? hy : hy >> 1; }
  __device__ static int xcoord(int hx) { return ST == 1 ? hx : hx >> 1; }
};

template <int ST, int NB = 64>
__global__ __launch_bounds__(NB * 4, ST == 1 ? 2 : 1) void conv3x3_wgrad_kernel(
    const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X, float* __restrict__ ws,
    const uint16_t* __restrict__ zeros, int N, int C, int IH, int IW, int OH, int OW, int pgh, int pgw,
    int npatch, int ntiles, int splits) {
  using H = Halo<ST, NB>;
  constexpr int STG = H::STAGES, LPS = 2 + H::PER_WAVE;  // DMA instructions per stage per wave
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nh = wid >> 2, cw = wid & 3;  // this wave's n half (NB = 128) and 16-channel c slice
  const int wg = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, sidx = wg / ntiles;  // XCD neighbours: same pixels, other tiles
  const int ctiles = C >> 6;
  const int n0 = (tile / ctiles) * NB, c0 = (tile % ctiles) * 64;
  const int p_begin = (int)((int64_t)npatch * sidx / splits), p_end = (int)((int64_t)npatch * (sidx + 1) / splits);

  // per-lane DMA row decode (patch-relative), fixed for the whole kernel
  const int pos = lane & 7;  // 16-B slot this lane fills in its 128-B LDS row
  int a_py[2], a_px[2], a_chunk[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (cw * 2 + i) * 8 + (lane >> 3);  // patch pixel 0..63 (of n half nh)
    a_py[i] = r >> 3;
    a_px[i] = r & 7;
    a_chunk[i] = pos ^ (2 * swp(a_py[i], a_px[i]));
  }
  int b_hy[H::PER_WAVE], b_hx[H::PER_WAVE], b_chunk[H::PER_WAVE];
#pragma unroll
  for (int i = 0; i < H::PER_WAVE; ++i) {
    const int r = (wid * H::PER_WAVE + i) * 8 + (lane >> 3);  // LDS row
    const int ph = r / (H::IYN * H::IXW), rem = r - ph * (H::IYN * H::IXW);
    const int iy = rem / H::IXW, ix = rem - iy * H::IXW;
    const int hy = ST == 1 ? iy : 2 * iy + (ph >> 1), hx = ST == 1 ? ix : 2 * ix + (ph & 1);
    const bool ok = r < H::ROWS && ix < (ST == 1 ? H::IXW : H::IYN) && hy < (kP - 1) * ST + 3 &&
                    hx < (kP - 1) * ST + 3;
    b_hy[i] = ok ? hy : -100000;  // invalid rows always read the zero line
    b_hx[i] = hx;
    b_chunk[i] = pos ^ (2 * swp(iy, ix));
  }

  auto issue = [&](int p, int buf) {
    uint8_t* A = smem + buf * H::STAGE;
    uint8_t* B = A + NB * 128;
    const int per_img = pgh * pgw;
    const int b = p / per_img, pr = p - b * per_img, oy0 = (pr / pgw) * kP, ox0 = (pr % pgw) * kP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int oy = oy0 + a_py[i], ox = ox0 + a_px[i];
      const bool ok = oy < OH && ox < OW;
      const uint16_t* src = ok ? dY + (((int64_t)b * OH + oy) * OW + ox) * N + n0 + 64 * nh + a_chunk[i] * 8 : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(A + nh * 8192 + (cw * 2 + i) * 1024), 16, 0, 0);
    }
    const int gy0 = oy0 * ST - 1, gx0 = ox0 * ST - 1;
#pragma unroll
    for (int i = 0; i < H::PER_WAVE; ++i) {
      const int gy = gy0 + b_hy[i], gx = gx0 + b_hx[i];
      const bool ok = (unsigned)gy < (unsigned)IH && (unsigned)gx < (unsigned)IW;
      const uint16_t* src = ok ? X + (((int64_t)b * IH + gy) * IW + gx) * C + c0 + b_chunk[i] * 8 : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(B + (wid * H::PER_WAVE + i) * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addressing: group g (lane >> 4) = patch row within the k-step, lane (4q + p)
  // supplies pixel column q (+4 for the second read) and bytes 8p of its 32-B chunk pair. The
  // swizzle depends on the lane only through (q + dx) & 3 and (g + dy) & 1, so each read is a
  // per-lane base (4 for A, 6 | 4 for the halo) plus a compile-time offset the ds_read absorbs.
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  constexpr int DXN = ST == 1 ? 3 : 2;
  int a_off[4], b_off[DXN][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a_off[i] = (g * 8 + q4) * 128 + ((i ^ swp(g, q4)) * 32) + 8 * p4;
#pragma unroll
  for (int dx = 0; dx < DXN; ++dx)
#pragma unroll
    for (int dp = 0; dp < 2; ++dp)
      b_off[dx][dp] = (g * H::IXW + q4 + dx) * 128 + ((cw ^ ((q4 + dx) & 3) ^ ((g + dp) & 1)) * 32) + 8 * p4;
  auto read_b = [&](const uint8_t* B, int ks, int t) {
    const int r = t / 3, s = t % 3;
    const int dy = ST == 1 ? r : r >> 1, dx = ST == 1 ? s : s >> 1;
    const int phase = ST == 1 ? 0 : (r & 1) * 2 + (s & 1);
    const uint8_t* p = B + b_off[dx][dy & 1] + (phase * H::IYN * H::IXW + (ks * 4 + dy) * H::IXW) * 128;
    const v4s v8[2] = {lds_tr16(p), lds_tr16(p + 4 * 128)};
    return __builtin_bit_cast(bf16x8, v8);
  };
  const int np = p_end - p_begin;
  for (int k = 0; k < STG - 1 && k < np; ++k) issue(p_begin + k, k);
  for (int k = 0; k < np; ++k) {
    // retire patch k's stage (later stages may stay in flight), then make every wave's DMA visible
    const int ahead = min(STG - 2, np - 1 - k);
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (k + STG - 1 < np) issue(p_begin + k + STG - 1, (k + STG - 1) % STG);
    const uint8_t* A = smem + (k % STG) * H::STAGE + nh * 8192;
    const uint8_t* B = smem + (k % STG) * H::STAGE + NB * 128;
    auto read_a = [&](int ks, bf16x8 (&a)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint8_t* p = A + a_off[i] + ks * 4 * 8 * 128;
        const v4s v8[2] = {lds_tr16(p), lds_tr16(p + 4 * 128)};
        a[i] = __builtin_bit_cast(bf16x8, v8);
      }
    };
    // 18 (k-step, tap) steps; the next step's halo fragment (and, two taps before the end of
    // k-step 0, k-step 1's dY fragments) are read while this step's 4 MFMAs run
    bf16x8 a[4], an[4];
    read_a(0, a);
    bf16x8 b = read_b(B, 0, 0);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int ks = st / 9, t = st % 9;
      bf16x8 bn = b;
      if (st < 17) bn = read_b(B, (st + 1) / 9, (st + 1) % 9);
      if (st == 6) read_a(1, an);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][t], 0, 0, 0);
      b = bn;
      if (st == 8) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = an[i];
      }
      (void)ks;
    }
  }
  // fp32 slab ws[sidx][n][tap][c]: lane holds n = n0 + 64 nh + 16i + 4(lane >> 4) + r, c = c0 + 16 cw + (lane & 15)
  float* out = ws + (int64_t)sidx * N * 9 * C;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 64 * nh + 16 * i + 4 * (lane >> 4) + r;
        out[((int64_t)n * 9 + t) * C + c0 + 16 * cw + (lane & 15)] = acc[i][t][r];
      }
}

// ---------------------------------------------------------------------------------------------
// Stride-1 weight gradient on ROW BANDS (r6): the reduction runs over runs of 224
// consecutive output pixels of the flattened (batch x height) row space — R = 224 / W whole rows
// (W = 56 / 28 / 14 / 7: R = 4 / 8 / 16 / 32; 224 = 7 MFMA k-steps of 32 pixels), bands crossing
// images as in conv3x3_band.hip — instead of 8 x 8 patches, which computed 1.306x the pixels at
// W = 28 / 14 / 7 (a 4 x 4 patch grid over 28 x 28, ...). A band stages its dY rows (224 x 64 n)
// and its input halo (R + 2·segments rows of W + 2 pixels, zero padding rows at image edges, zero
// columns) once per 64 x 64 channel tile, and every tap reads its shifted pixel window from the
// halo: 63 (k-step, tap) steps of 4 MFMAs per wave per band (7x the patch kernel's MFMAs per
// barrier). One block per CU, persistent over a contiguous range of bands, two LDS stages (the next
// band's DMA under this band's MFMAs), both by inline-asm LDS-DMA (hipcc cannot tell the stages apart
// and would drain the prefetch before every fragment read). Eight waves, two per SIMD, split each
// band's 7 k-steps by parity (4 + 3, alternating by band): the first version (4 waves, one per SIMD)
// exposed every fragment-read and DMA-issue latency and ran 137-147 us per ResNet-50 shape.
// LDS image: 128-B rows (one pixel, 64 channels); the 32-B chunk PAIR (16 channels, one wave's or
// one fragment's) of a row is XOR-swizzled by f(v) = ((v >> 1) & 1) | ((v >> 2) & 2) of the pixel's
// virtual index v (dY: the band pixel m; halo: hr·W + hc, which runs on consecutively over the
// output-row wraps of a fragment, and has the parity of the LDS row): the 8 rows one
// ds_read_b64_tr_b16 half-wave reads (two 4-pixel groups 8 pixels apart) land on 8 distinct bank
// octets for any start (checked exhaustively). Same slab layout / slab_sum_kernel as the patch kernel.
__device__ __forceinline__ int bfz(int v) { return ((v >> 1) & 1) | ((v >> 2) & 2); }

// halo row of band-relative output row lr (tap row 0) — conv3x3_band.hip band_hrow
__device__ __forceinline__ int wb_hrow(int lr, int n0, int H) {
  if (lr < n0) return lr;
  const int k = (lr - n0) / H;
  return n0 + 2 + k * (H + 2) + (lr - n0 - k * H);
}

__global__ __launch_bounds__(512, 2) void conv3x3_wgrad_band_kernel(
    const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X, float* __restrict__ ws,
    const uint16_t* __restrict__ zeros, int N, int C, int B, int H, int W, int R, int nbands, int ntiles, int splits,
    int hpix) {
  constexpr int BP = 224;  // band pixels (7 k-steps)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int STAGE = (BP + hpix) * 128;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // 8 waves, two per SIMD: wave w owns c slice cw = w & 3 (16 channels) for all 64 n and 9 taps, and
  // k-step parity group grp = w >> 2 of each band (the two groups alternate the 4-step share by band
  // parity); the groups' accumulators are summed through LDS once, at the end
  const int cw = wid & 3, grp = wid >> 2;
  const int wg = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % ntiles, sidx = wg / ntiles;  // XCD neighbours: same bands, other tiles
  const int ctiles = C >> 6;
  const int n0c = (tile / ctiles) * 64, c0 = (tile % ctiles) * 64;
  const int bb = (int)((int64_t)nbands * sidx / splits), be = (int)((int64_t)nbands * (sidx + 1) / splits);
  const int W2 = W + 2, rows_total = B * H;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem);
  const int uwid = __builtin_amdgcn_readfirstlane(wid);
  auto glds16 = [](const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
  };
  const int pos = lane & 7;  // 16-B slot of the lane's 128-B LDS row in a DMA piece (8 rows)

  auto issue = [&](int band, int slot) {
    const uint32_t st = lbase + slot * STAGE;
    const int g0 = band * R, b0 = g0 / H, h0 = g0 - b0 * H;
    const int n0 = min(H - h0, R), rv = min(R, rows_total - g0), valid = rv * W;
    // dY: 28 pieces of 8 pixel rows; wave w takes pieces w, w + 8, ...
    for (int k = uwid; k < 28; k += 8) {
      const int m = k * 8 + (lane >> 3);
      const bool ok = m < valid;
      const uint16_t* src = ok ? dY + ((int64_t)g0 * W + m) * N + n0c + 8 * (pos ^ (2 * bfz(m))) : zeros;
      glds16(src, __builtin_amdgcn_readfirstlane(st + k * 1024));
    }
    // halo: hpix / 8 pieces (a multiple of 4), rows past the band's halo read the zero line
    const int hlast = wb_hrow(rv - 1, n0, H) + 2;
    for (int k = uwid; k * 8 < hpix; k += 8) {
      const int q = k * 8 + (lane >> 3), hr = q / W2, hc = q - hr * W2;
      int b = b0, ih = h0 - 1 + hr;
      if (hr >= n0 + 2) {  // a later image of the band
        const int r2 = hr - (n0 + 2), kk = r2 / (H + 2);
        b = b0 + 1 + kk;
        ih = r2 - kk * (H + 2) - 1;
      }
      const int iw = hc - 1;
      const bool ok = hr <= hlast && b < B && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint16_t* src =
          ok ? X + (((int64_t)b * H + ih) * W + iw) * C + c0 + 8 * (pos ^ (2 * bfz(hr * W + hc))) : zeros;
      glds16(src, __builtin_amdgcn_readfirstlane(st + (BP + k * 8) * 128));
    }
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed reads: group gq = lane >> 4, lane 4q + p supplies pixel 8gq + q (+4) of the k-step and
  // bytes 8p of its 32-B chunk pair
  const int gq = lane >> 4, q4 = (lane >> 2) & 3, p8 = 8 * (lane & 3);
  if (bb < be) {
    issue(bb, 0);
    for (int band = bb; band < be; ++band) {
      const int slot = (band - bb) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                 // this wave's pieces of the band
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // everyone's; the other slot is free
      issue(band + 1 < be ? band + 1 : band, slot ^ 1);                // (past the end: a re-stage, unused)
      const uint8_t* A = smem + slot * STAGE;
      const uint8_t* Hs = A + BP * 128;
      const int g0 = band * R, b0 = g0 / H, h0 = g0 - b0 * H;
      const int n0 = min(H - h0, R), rv = min(R, rows_total - g0), valid = rv * W;
      // this lane's halo pixel (tap (0, 0)) of pixel m: LDS row and virtual index; past the band's
      // pixels a valid one (its dY row is zero)
      auto hpx = [&](int m, int& hq, int& hv) {
        const int mm = min(m, valid - 1), lr = mm / W, col = mm - lr * W, hr = wb_hrow(lr, n0, H);
        hq = hr * W2 + col;
        hv = hr * W + col;
      };
      auto read_a = [&](int ks, bf16x8 (&a)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v4s v8[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int m = ks * 32 + 8 * gq + q4 + 4 * h;
            v8[h] = lds_tr16(A + m * 128 + 32 * (i ^ bfz(m)) + p8);
          }
          a[i] = __builtin_bit_cast(bf16x8, v8);
        }
      };
      int hq[2], hv[2];
      auto set_k = [&](int ks) {
#pragma unroll
        for (int h = 0; h < 2; ++h) hpx(ks * 32 + 8 * gq + q4 + 4 * h, hq[h], hv[h]);
      };
      auto read_b = [&](int t) {
        const int r = t / 3, sx = t - 3 * r;
        v4s v8[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int q = hq[h] + r * W2 + sx, v = hv[h] + r * W + sx;
          v8[h] = lds_tr16(Hs + q * 128 + 32 * (cw ^ bfz(v)) + p8);
        }
        return __builtin_bit_cast(bf16x8, v8);
      };
#pragma unroll 1
      for (int ks = grp ^ ((band - bb) & 1); ks < 7; ks += 2) {
        bf16x8 a[4];
        read_a(ks, a);
        set_k(ks);
        bf16x8 b = read_b(0);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          bf16x8 bn = b;
          if (t < 8) bn = read_b(t + 1);  // the next tap's fragment under this tap's MFMAs
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][t], 0, 0, 0);
          b = bn;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-stage lands before exit
  }
  // group 1's accumulators -> LDS (144 x 256 floats, element-major: lanes on consecutive words), group 0
  // adds them in a fixed order and writes the fp32 slab ws[sidx][n][tap][c] as the patch kernel: lane
  // holds n = n0c + 16i + 4(lane >> 4) + r, c = c0 + 16 cw + (lane & 15)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* xr = reinterpret_cast<float*>(smem);
  const int xl = cw * 64 + lane;
  if (grp == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) xr[((i * 9 + t) * 4 + r) * 256 + xl] = acc[i][t][r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) return;
  float* out = ws + (int64_t)sidx * N * 9 * C;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0c + 16 * i + 4 * (lane >> 4) + r;
        out[((int64_t)n * 9 + t) * C + c0 + 16 * cw + (lane & 15)] = acc[i][t][r] + xr[((i * 9 + t) * 4 + r) * 256 + xl];
      }
}

// dW = sum of the S slabs, cast to the weight dtype (4 elements per lane, slab sum split 8 ways)
template <typename W>
__global__ __launch_bounds__(512) void slab_sum_kernel(const float* __restrict__ ws, int S, int64_t nk,
                                                       W* __restrict__ dw) {
  __shared__ f32x4 red[8][64];
  const int c = threadIdx.x & 63, gi = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * 64 + c;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (v * 4 < nk) {
    const float* p = ws + v * 4;
    int s = gi;
    for (; s + 8 < S; s += 16) {
      a0 += *reinterpret_cast<const f32x4*>(p + (int64_t)s * nk);
      a1 += *reinterpret_cast<const f32x4*>(p + (int64_t)(s + 8) * nk);
    }
    for (; s < S; s += 8) a0 += *reinterpret_cast<const f32x4*>(p + (int64_t)s * nk);
  }
  red[gi][c] = a0 + a1;
  __syncthreads();
  if (gi == 0 && v * 4 < nk) {
    f32x4 acc = red[0][c];
#pragma unroll
    for (int i = 1; i < 8; ++i) acc += red[i][c];
    dev::Elem<W, float>::st(dw, v * 4 + 0, acc.x);
    dev::Elem<W, float>::st(dw, v * 4 + 1, acc.y);
    dev::Elem<W, float>::st(dw, v * 4 + 2, acc.z);
    dev::Elem<W, float>::st(dw, v * 4 + 3, acc.w);
  }
}

const uint16_t* zero_line_w(const at::Tensor& like) {
  static at::Tensor* z[64] = {};  // never freed: a static tensor would outlive the HIP runtime
  const int d = like.device().index();
  TORCH_CHECK(d >= 0 && d < 64, "conv3x3_wgrad: device index out of range");
  if (!z[d]) z[d] = new at::Tensor(at::zeros({128}, like.options().dtype(at::kBFloat16)));
  return reinterpret_cast<const uint16_t*>(z[d]->data_ptr());
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

}  // namespace

namespace {
// XDDP_WGRAD3_BAND=1: the row-band kernel for stride-1 weight gradients (opt-in: it measured 137-147 us
// vs the patch kernel's 82-87 us per call at every ResNet-50 stage shape, profiles/r6_wgrad3_band_ab.txt)
bool band_wgrad() {
  static const bool v = [] { const char* e = std::getenv("XDDP_WGRAD3_BAND"); return e && e[0] == '1'; }();
  return v;
}

template <typename F>
void slab_sum(const at::Tensor& ws, int splits, int64_t nk, const at::Tensor& dw, hipStream_t stream, F&&) {
  const int grid = (int)((nk / 4 + 63) / 64);
  auto red = [&](auto tag) {
    using W = decltype(tag);
    hipLaunchKernelGGL((slab_sum_kernel<W>), dim3(grid), dim3(512), 0, stream, ws.data_ptr<float>(), splits, nk,
                       reinterpret_cast<W*>(dw.data_ptr()));
    XDDP_HIP_CHECK(hipGetLastError());
  };
  switch (dw.scalar_type()) {
    case at::kBFloat16: red(dev::bf16_t{}); break;
    case at::kFloat: red(float{}); break;
    case at::kHalf: red(dev::f16_t{}); break;
    default: TORCH_CHECK(false, "conv3x3_wgrad: unsupported weight dtype");
  }
}

at::Tensor conv3x3_wgrad_band(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w_like) {
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), N = dy.size(1);
  const int R = (int)(224 / W);
  const int64_t rows_total = B * H, nbands = (rows_total + R - 1) / R;
  TORCH_CHECK(nbands < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "conv3x3_wgrad_band: too large");
  // halo pixels: the most a band needs (a segment per image it touches, two padding rows each)
  int segs = 1;
  for (int64_t k = 0; k < H; ++k) {
    const int64_t h0 = (k * R) % H, n0 = std::min<int64_t>(H - h0, R);
    segs = std::max<int>(segs, (int)(1 + (R - n0 + H - 1) / H));
  }
  segs = (int)std::min<int64_t>(segs, B);
  const int hpix = (int)((((R + 2 * segs) * (W + 2)) + 31) / 32 * 32);
  // two stages; at the end the k-step groups' accumulators are exchanged through the same LDS
  const size_t lds = std::max<size_t>((size_t)2 * (224 + hpix) * 128, (size_t)144 * 256 * sizeof(float));
  TORCH_CHECK(lds <= 160 * 1024, "conv3x3_wgrad_band: LDS budget exceeded (", lds, " B)");
  const int ntiles = (int)((N / 64) * (C / 64));
  const int splits = (int)std::max<int64_t>(1, std::min<int64_t>(nbands, std::max(1, cu_count() / ntiles)));
  auto ws = at::empty({splits, N, 9, C}, dy.options().dtype(at::kFloat));
  auto dw = at::empty({N, C, 3, 3}, dy.options().dtype(w_like.scalar_type()).memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  ensure_dyn_lds((const void*)conv3x3_wgrad_band_kernel, lds);
  hipLaunchKernelGGL(conv3x3_wgrad_band_kernel, dim3(ntiles * splits), dim3(512), lds, stream,
                     reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                     ws.data_ptr<float>(), zero_line_w(x), (int)N, (int)C, (int)B, (int)H, (int)W, R, (int)nbands, ntiles,
                     splits, hpix);
  XDDP_HIP_CHECK(hipGetLastError());
  slab_sum(ws, splits, N * 9 * C, dw, stream, 0);
  return dw;
}
}  // namespace

// dy [B, N, OH, OW], x [B, C, IH, IW] (bf16 channels_last, pad 1, stride 1|2) -> dW [N, C, 3, 3]
// channels_last (OHWI memory) in w_like's dtype. splits_req: < 0 the default kernel (the patch kernel; the
// band kernel at stride 1 with 224 % W == 0 under XDDP_WGRAD3_BAND=1), -2 forces the band kernel there,
// >= 0 forces the patch kernel (0 with its default split): timing scripts / tests.
at::Tensor conv3x3_wgrad_patch(const at::Tensor& dy, const at::Tensor& x, int64_t stride, const at::Tensor& w_like,
                               int64_t splits_req) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 &&
                  dy.dim() == 4 && x.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_wgrad_patch: bf16 channels_last 4-D GPU tensors expected");
  TORCH_CHECK(stride == 1 || stride == 2, "conv3x3_wgrad_patch: stride 1 or 2");
  const int64_t B = x.size(0), C = x.size(1), IH = x.size(2), IW = x.size(3), N = dy.size(1);
  const int64_t OH = (IH - 1) / stride + 1, OW = (IW - 1) / stride + 1;
  TORCH_CHECK(dy.size(0) == B && dy.size(2) == OH && dy.size(3) == OW, "conv3x3_wgrad_patch: dy/x shape mismatch");
  TORCH_CHECK(N % 64 == 0 && C % 64 == 0, "conv3x3_wgrad_patch: channel counts must be multiples of 64");
  TORCH_CHECK(x.numel() < (int64_t(1) << 40) && dy.numel() < (int64_t(1) << 40), "conv3x3_wgrad_patch: too large");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16) == 0,
              "conv3x3_wgrad_patch: 16-B aligned operands required");
  if (stride == 1 && 224 % OW == 0 && (splits_req == -2 || (band_wgrad() && splits_req < 0)))
    return conv3x3_wgrad_band(dy, x, w_like);
  const int pgh = (int)((OH + kP - 1) / kP), pgw = (int)((OW + kP - 1) / kP);
  const int64_t npatch64 = B * pgh * pgw;
  TORCH_CHECK(npatch64 > 0 && npatch64 < (int64_t(1) << 31), "conv3x3_wgrad_patch: bad patch count");
  const int npatch = (int)npatch64;
  // stride 2 with N % 128 == 0: 128-channel n tiles (8 waves sharing one staged halo)
  // (a 128-channel tile at stride 1 measured 3-10 % slower: 96.0 / 97.5 / 93.5 / 91.7 vs
  // 90.4 / 95.0 / 86.3 / 83.1 us on the four stage shapes, scripts/wgrad3_time.py)
  const int nb = stride == 2 && N % 128 == 0 ? 128 : 64;
  const int ntiles = (int)((N / nb) * (C / 64));
  const int per_cu = stride == 1 ? 2 : 1;  // resident blocks per CU (LDS: 72 KB | 112 / 128 KB per block)
  int splits = std::max(1, std::min(npatch, (cu_count() * per_cu + ntiles - 1) / ntiles));
  if (splits_req > 0) splits = (int)std::min<int64_t>(npatch, splits_req);
  auto ws = at::empty({splits, N, 9, C}, dy.options().dtype(at::kFloat));
  auto dw = at::empty({N, C, 3, 3}, dy.options().dtype(w_like.scalar_type()).memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  const uint16_t* zeros = zero_line_w(x);
  auto go = [&](auto kern, size_t lds, int threads) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(ntiles * splits), dim3(threads), lds, stream,
                       reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       ws.data_ptr<float>(), zeros, (int)N, (int)C, (int)IH, (int)IW, (int)OH, (int)OW, pgh, pgw,
                       npatch, ntiles, splits);
    XDDP_HIP_CHECK(hipGetLastError());
  };
  if (stride == 1) go(conv3x3_wgrad_kernel<1>, (size_t)Halo<1>::STAGES * Halo<1>::STAGE, 256);
  else if (nb == 128) go(conv3x3_wgrad_kernel<2, 128>, (size_t)Halo<2, 128>::STAGES * Halo<2, 128>::STAGE, 512);
  else go(conv3x3_wgrad_kernel<2>, (size_t)Halo<2>::STAGES * Halo<2>::STAGE, 256);
  const int64_t nk = N * 9 * C;
  const int grid = (int)((nk / 4 + 63) / 64);
  auto red = [&](auto tag) {
    using W = decltype(tag);
    hipLaunchKernelGGL((slab_sum_kernel<W>), dim3(grid), dim3(512), 0, stream, ws.data_ptr<float>(), splits, nk,
                       reinterpret_cast<W*>(dw.data_ptr()));
    XDDP_HIP_CHECK(hipGetLastError());
  };
  switch (w_like.scalar_type()) {
    case at::kBFloat16: red(dev::bf16_t{}); break;
    case at::kFloat: red(float{}); break;
    case at::kHalf: red(dev::f16_t{}); break;
    default: TORCH_CHECK(false, "conv3x3_wgrad_patch: unsupported weight dtype");
  }
  return dw;
}

}  // namespace kernels
}  // namespace xddp
