// Stride-1 3x3 convolution (NHWC, bf16, pad 1) on row bands: an implicit MFMA GEMM for gfx950
// whose M tiles are runs of R consecutive output rows of the flattened (batch x height) row space,
// with the following BatchNorm's batch statistics optionally produced by its epilogue. The same
// kernel runs the stride-1 input gradient on (dY, rot180(W)ᵀ) (conv3x3.hip conv3x3_rot_weight).
//
// Why bands that cross images: the ResNet-50 3x3 shapes have 56 / 28 / 14 / 7 pixels per row and
// B·H·W = 2^10 · 7^2 · (1, 4, 16, 64) output pixels. Tiles of whole rows inside one image (the
// halo kernel of conv3x3.hip: 256-row tiles holding 224 / 196 valid pixels at W = 56 / 28) compute
// 14-31 % padding rows, and pixel tiles of 256 over the whole batch (conv3x3_gemm) leave 392 / 196
// tiles for 256 CUs (77 % of the last round busy). A band of R rows with R·W = 224 (W = 56: R = 4)
// or 196 (W = 28 / 14 / 7: R = 7 / 14 / 28; one tile = one image at W = 14, four at W = 7) packs
// the band's pixels contiguously into the tile rows: 0 % / 6 % padding rows, and 3584 / 1024 / 512
// / 256 x (N / BN) tiles — whole rounds of 2 blocks per CU. (W = 7 runs the dense-GEMM path of
// conv3x3.hip: 256 tiles of 4-image bands leave one 4-wave block per CU, 73 vs 63 us.)
//
// The input halo of a band is staged ONCE per 64-channel K step and read by all 9 taps (shifted
// windows): a band that spans images is a list of segments, each staged as its rows plus one row
// above and below (the image's zero padding rows where the band meets an image edge), so the
// halo holds R + 2·segments rows of W + 2 pixels (zero columns left and right). Padding pixels
// DMA a zero line. A lane's MFMA rows are output pixels m of the band -> halo pixel
// (hrow(m / W) + r)·(W + 2) + m % W + s for tap (r, s), where hrow skips two halo rows at every
// image boundary. Operands go global -> LDS with global_load_lds_dwordx4 (LDS-DMA, rows of 128 B =
// 64 channels, chunk XOR-swizzled by (row >> 1) & 7 through pre-swizzled source addresses); the
// tap's weights (BN x 64) stream through a RING-slot ring with counted `s_waitcnt vmcnt` + raw
// s_barrier (N = 64), or — N % 128 == 0 — go straight from global memory (L2-resident) into each
// wave's registers per 32-deep half step, three half steps ahead, so the 9 taps of a 64-channel
// step need no barrier at all (only the halo reload between channel steps does). Four waves
// (WM x WN) of TM x TN 16x16x32 MFMA tiles; two blocks per CU, so one block's halo wait and
// epilogue run under the other's MFMAs.
//
// Epilogue as conv3x3.hip: the bf16 C tile through LDS, 16-B row stores of the valid pixels (the
// band's output pixels are contiguous in NHWC memory), BatchNorm (count, mean, M2) partials per
// channel and statistics group, group-minor part[3][N][groups]. With statistics the N = 64
// configuration runs persistent blocks (two per CU, each walking bands wg, wg + grid, ...) whose
// shifted sums stay in registers across bands: the cross-lane reduction and partial writes run
// once per block instead of once per band (r5: 3584 -> 512 groups, C64 forward 108 -> 100 us).
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

__device__ __forceinline__ int swzb(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }

// Halo LDS image: 128-B rows (one pixel, 64 channels), the 16-B chunk of row q XOR-swizzled by
// (v >> 1) & 7 of the pixel's VIRTUAL index v = hr·W + hc (halo row hr, column hc) rather than of q
// = hr·(W + 2) + hc itself: the 16 pixels of an MFMA fragment are consecutive in v whatever image
// rows they wrap over, where q jumps by 2 at every wrap. With the fragment's pixels interleaved
// over its 16 lanes (kPerm: the lanes ds_read_b128 services in one LDS cycle read pixels of one
// parity for one chunk and of the other parity for the other chunk), every read of the halo is
// bank-conflict free (the linear swizzle with lanes in pixel order measured 35-49 % of LDS cycles
// in conflicts: 75-170 % extra cycles per read by the lane-group model of MI355X_MICROARCH.md).
__device__ __forceinline__ int hswz(int q, int v, int chunk) { return q * 128 + 16 * (chunk ^ ((v >> 1) & 7)); }
// fragment pixel of lane x = lane & 15: 0,2,4,6 | 1,3,...,15 | 8,10,12,14
__device__ __forceinline__ int kperm(int x) { return x < 4 ? 2 * x : (x < 12 ? 2 * x - 7 : 2 * x - 16); }

struct BandGeo {
  int B, H, W, C;  // input (= output) batch, rows, columns, channels
  int R;           // output rows per band (tile)
  int rows_total;  // B·H
};

// halo row of band-relative output row lr (tap row 0): the first segment (n0 rows of image b0)
// starts at halo row 0, every later image at a multiple of H + 2 after it
__device__ __forceinline__ int band_hrow(int lr, int n0, int H) {
  if (lr < n0) return lr;
  const int k = (lr - n0) / H;
  return n0 + 2 + k * (H + 2) + (lr - n0 - k * H);
}

// readout rows per batch of LDS reads in the epilogue (issued together, then stored)
#ifndef XDDP_BAND_RB
#define XDDP_BAND_RB 4
#endif

template <int TM, int WM, int TN, int WN, bool STATS, int RING>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv3x3_band_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y,
    const uint16_t* __restrict__ zeros, int N, BandGeo g, float* __restrict__ part, int ntiles, int mtiles,
    int hrows) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
  constexpr int BI = BN / 8 / NW;  // weight DMA wave-instructions per tap
  static_assert(BI * NW * 8 == BN, "weight rows must split evenly over the waves");
  static_assert(RING == 0 || RING == 2 || RING == 3, "weights in registers (0) or a ring of 2 or 3 LDS slots");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* halo = smem;                // hrows x 128 B
  uint8_t* ring = smem + hrows * 128;  // RING x BN x 128 B

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int wg = dev::xcd_remap(blockIdx.x, gridDim.x);
  // persistent over tiles wg, wg + grid, ...: the grid is a multiple of ntiles, so a block keeps one
  // channel tile nt and its statistics accumulate over its bands, reduced and written once
  const int nt = wg % ntiles;
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "readout mapping needs a fixed chunk column per thread");
  const int cc = tid % CPR;
  float st_n = 0.f, st_s[8], st_ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) st_s[e] = st_ss[e] = 0.f;
  u32x4 st_k = u32x4{0u, 0u, 0u, 0u};  // the shift: row 0 (always valid) of the block's first band
  const int prow = kperm(lane & 15);
  const int n0c = nt * BN, pos = lane & 7, cbn = g.C >> 6, K9 = 9 * g.C, W2 = g.W + 2;
  constexpr bool PERSIST = STATS && RING != 0;  // (the register-B configuration has no room for it)
  int wt = wg;
  do {
    const int mt = wt / ntiles;
    if (wt != wg) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // last band's C tile read
    const int g0 = mt * g.R;                       // first output row of the band (flattened b·H + h)
    const int b0 = g0 / g.H, h0 = g0 - b0 * g.H;
    const int n0 = min(g.H - h0, g.R);             // rows of the first segment
    const int rv = min(g.R, g.rows_total - g0);    // valid output rows of the band
    const int valid = rv * g.W;
    const int HP = (band_hrow(rv - 1, n0, g.H) + 3) * W2;  // halo pixels to stage

    // this lane's MFMA A rows -> halo pixel of tap (0, 0) (rows past the band read a valid pixel)
    int hb[TM], vb[TM];  // LDS row and virtual index (hswz) of the pixel's tap (0, 0) halo pixel
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = min(wm * TM * 16 + i * 16 + prow, valid - 1);
      const int lr = m / g.W, hr = band_hrow(lr, n0, g.H), col = m - lr * g.W;
      hb[i] = hr * W2 + col;
      vb[i] = hr * g.W + col;
    }
    int boff[BI];  // (32-bit offsets: host-checked tensors < 2^31 elements)
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int row = (wid * BI + j) * 8 + (lane >> 3);
      boff[j] = (n0c + row) * K9 + 8 * (pos ^ ((row >> 1) & 7));
    }
    auto issue_halo = [&](int cb) {
      for (int k = wid; k * 8 < HP; k += NW) {  // per-wave counts differ: only count-free waits cover it
        const int q = k * 8 + (lane >> 3), hr = q / W2, hc = q - hr * W2;
        int b = b0, ih = h0 - 1 + hr;
        if (hr >= n0 + 2) {  // a later image of the band
          const int r2 = hr - (n0 + 2), kk = r2 / (g.H + 2);
          b = b0 + 1 + kk;
          ih = r2 - kk * (g.H + 2) - 1;
        }
        const int iw = hc - 1;
        const bool ok = q < HP && b < g.B && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        const uint16_t* src =
            ok ? X + (((b * g.H + ih) * g.W + iw) * g.C + cb * 64 + 8 * (pos ^ (((hr * g.W + hc) >> 1) & 7))) : zeros;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(halo + k * 1024), 16, 0, 0);
      }
    };
    auto issue_w = [&](int cb, int t, int slot) {
      uint8_t* Bs = ring + slot * BN * 128;
      const int wk = t * g.C + cb * 64;
#pragma unroll
      for (int j = 0; j < BI; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(Wt + boff[j] + wk), (lds_ptr_t)(Bs + (wid * BI + j) * 1024), 16,
                                         0, 0);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (RING == 0) {
      // B in registers: each wave loads its own TN column tiles straight from global memory (the
      // weights are L2-resident), per 32-deep half step, three half steps deep; taps need no barrier
      // and no ring, only the halo goes through LDS (one barrier per 64-channel step)
      bf16x8 breg[3][TN];
      const uint16_t* wl = Wt + (int64_t)(n0c + wn * TN * 16 + (lane & 15)) * K9 + (lane >> 4) * 8;
      auto load_b = [&](int cb, int u, bf16x8 (&dst)[TN]) {  // half step u = 2·tap + half
        const uint16_t* p = wl + (u >> 1) * g.C + cb * 64 + (u & 1) * 32;
#pragma unroll
        for (int j = 0; j < TN; ++j) dst[j] = *reinterpret_cast<const bf16x8*>(p + j * 16 * K9);
      };
      issue_halo(0);
      load_b(0, 0, breg[0]);
      load_b(0, 1, breg[1]);
      for (int cb = 0; cb < cbn; ++cb) {
        if (cb > 0) {
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done with the halo
          issue_halo(cb);
        }
        const bool last = cb + 1 == cbn;
        // opaque per step: keeps the compiler from hoisting all 18 x TM LDS addresses of the unrolled
        // half steps out of the channel loop (they are loop-invariant; live, they spill)
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(hb[i]), "+v"(vb[i]));
#pragma unroll
        for (int u = 0; u < 18; ++u) {
          __builtin_amdgcn_sched_barrier(0);  // keep each half step's LDS reads in it (register pressure)
          // half step u's B fragments (and at u = 0 the halo) must have landed; the loads issued after
          // them (the next half step's B) may stay in flight
          if (u == 0) {
            if (cb == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TN) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");  // every wave's halo DMA is visible
          } else if (u == 17 && last) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TN) : "memory");
          }
          if (u + 2 < 18) load_b(cb, u + 2, breg[(u + 2) % 3]);
          else if (!last) load_b(cb + 1, u - 16, breg[(u + 2) % 3]);
          const int t = u >> 1, h = u & 1, r = t / 3, sx = t - 3 * r;
          const int toff = r * W2 + sx, tv = r * g.W + sx, ch = h * 4 + (lane >> 4);
          bf16x8 a[TM];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            a[i] = *reinterpret_cast<const bf16x8*>(halo + hswz(hb[i] + toff, vb[i] + tv, ch));
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(breg[u % 3][j], a[i], acc[i][j], 0, 0, 0);
        }
      }
    } else {
      for (int cb = 0; cb < cbn; ++cb) {
        if (cb > 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // halo / ring reads done
        issue_halo(cb);
        issue_w(cb, 0, 0);
        if (RING == 3) issue_w(cb, 1, 1);
#pragma unroll 1
        for (int t = 0; t < 9; ++t) {
          // retire tap t's weights (at t = 0 also the halo issued before them); with three slots the
          // next tap's weights may stay in flight
          if (RING == 3 && t < 8) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BI) : "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (not unrolled: no cross-tap load hoisting)
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          if (t + RING - 1 < 9) issue_w(cb, t + RING - 1, (t + RING - 1) % RING);
          const int r = t / 3, sx = t - 3 * r, toff = r * W2 + sx, tv = r * g.W + sx;
          const uint8_t* Bs = ring + (t % RING) * BN * 128;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int ch = h * 4 + (lane >> 4);
            bf16x8 a[TM], bb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
            a[i] = *reinterpret_cast<const bf16x8*>(halo + hswz(hb[i] + toff, vb[i] + tv, ch));
#pragma unroll
            for (int j = 0; j < TN; ++j)
              bb[j] = *reinterpret_cast<const bf16x8*>(Bs + swzb(wn * TN * 16 + j * 16 + (lane & 15), ch));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j], a[i], acc[i][j], 0, 0, 0);
          }
        }
      }
    }

    // ---- epilogue: bf16 C tile through LDS, 16-B row stores of the valid pixels (+ statistics) ----
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    constexpr int CST = BN * 2 + 16;
    uint8_t* Cs = smem;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wm * TM * 16 + i * 16 + prow;
        const int col = wn * TN * 16 + j * 16 + (lane >> 4) * 4;
        uint2 pk;
        pk.x = dev::pack_bf16x2(acc[i][j][0], acc[i][j][1]);
        pk.y = dev::pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(Cs + row * CST + col * 2) = pk;
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (STATS && wt == wg) st_k = *reinterpret_cast<const u32x4*>(Cs + cc * 16);
    const int64_t y0 = (int64_t)g0 * g.W;                              // the band's first output pixel
    // rows tid / CPR + (NT / CPR)·i; each batch's LDS reads issued before its stores (rows past the
    // band read row valid - 1 and are not stored): a read-then-use per row inside `if (row < valid)`
    // compiled to one ds_read + s_waitcnt lgkmcnt(0) round trip per row
    constexpr int NIT = BM * CPR / NT, RSTR = NT / CPR, EB = NIT < XDDP_BAND_RB ? NIT : XDDP_BAND_RB;
    static_assert(BM * CPR % NT == 0, "readout rows must divide evenly over the threads");
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += EB) {
      u32x4 vv[EB];
#pragma unroll
      for (int j = 0; j < EB; ++j)
        if (i0 + j < NIT) vv[j] = *reinterpret_cast<const u32x4*>(Cs + min(tid / CPR + RSTR * (i0 + j), valid - 1) * CST + cc * 16);
#pragma unroll
      for (int j = 0; j < EB; ++j) {
        const int row = tid / CPR + RSTR * (i0 + j);
        if (i0 + j < NIT && row < valid) {
          const u32x4 v = vv[j];
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(Y + (y0 + row) * N + n0c + cc * 8));
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
  } while (PERSIST && (wt += gridDim.x) < mtiles * ntiles);
  if (!STATS) return;
  // every thread shifted by the same row-0 values, so the shifted sums add: lanes sharing cc, then
  // the waves through LDS; one (count, mean, M2) per channel and tile, part[q][N][tiles]
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1) {
    st_n += __shfl_xor(st_n, o, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      st_s[e] += __shfl_xor(st_s[e], o, 64);
      st_ss[e] += __shfl_xor(st_ss[e], o, 64);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float* red = reinterpret_cast<float*>(smem);
  float* redn = red + NW * 2 * BN;
  float* redk = redn + NW * CPR;
  if (lane < CPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wid * 2 + 0) * BN + cc * 8 + e] = st_s[e];
      red[(wid * 2 + 1) * BN + cc * 8 + e] = st_ss[e];
      if (wid == 0) redk[cc * 8 + e] = __uint_as_float((e & 1) ? (st_k[e >> 1] & 0xffff0000u) : (st_k[e >> 1] << 16));
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
    const float mean_s = tn > 0.f ? ts / tn : 0.f;  // (a block without bands: count 0, M2 0)
    const int grp = wg / ntiles;
    part[((int64_t)0 * N + n0c + c) * G + grp] = tn;
    part[((int64_t)1 * N + n0c + c) * G + grp] = redk[c] + mean_s;
    part[((int64_t)2 * N + n0c + c) * G + grp] = fmaxf(tss - ts * mean_s, 0.f);
  }
}

}  // namespace

// Band geometry for a stride-1 3x3 conv: rows per band for a tile of bm pixels (0: not covered).
// R·W = 224 (W = 56) or 196 (W = 28 / 14 / 7) output pixels (module comment).
int conv3x3_band_rows(int64_t W, int64_t H, int64_t bm) {
  int r = 0;
  if (W == 56) r = (int)(bm / 56);
  else if (W <= 28 && 196 % W == 0) r = (int)(196 / W);
  (void)H;
  return r > 0 && r * W <= bm ? r : 0;
}

// x [B, C, H, W] bf16 channels_last; w [N, C, 3, 3] bf16 channels_last (OHWI memory); stride 1.
// rows: output rows per band (0 = conv3x3_band_rows); returns {y channels_last, stats partials
// [3, N, tiles] group-minor (empty if !stats)}.
std::vector<at::Tensor> conv3x3_band(const at::Tensor& x, const at::Tensor& w, bool stats, int64_t rows,
                                     const uint16_t* zeros, int64_t cfg) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_band: x must be a bf16 channels_last CUDA tensor");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) == x.size(1),
              "conv3x3_band: w must be bf16 [N, C, 3, 3] channels_last");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), N = w.size(0);
  TORCH_CHECK(C % 64 == 0 && (N == 64 || N % 128 == 0), "conv3x3_band: C % 64 == 0 and N = 64 or N % 128 == 0");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31) && B * H * W * N < (int64_t(1) << 31) && N * 9 * C < (int64_t(1) << 31),
              "conv3x3_band: tensors must hold < 2^31 elements");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) % 16) == 0,
              "conv3x3_band: 16-B aligned operands required");
  // configurations {TM, WM, TN, WN, RING}: tile BM = 16·TM·WM pixels x BN = 16·TN·WN channels
  struct Cfg { int tm, wm, tn, wn, ring; };
  // (r5 A/Bs at the ResNet-50 bs256 shapes, scripts/c3_time.py, profiles/r5_conv3x3_band.txt: for N = 64
  // weights in registers (100.7 / 87.2 us) or 448-row tiles (95.9 / 87.1) gained nothing over the
  // ring; for N % 128 == 0 the registers beat the two-slot ring (62.0 / 59.1 vs 67.6 / 63.0 us at
  // C128, 57.7 / 55.4 vs 62.8 / 59.9 at C256: no barrier per tap); 112-row two-image bands at
  // W = 7 lost to the dense-GEMM path, 72.9 vs 63.0 us)
  static constexpr Cfg kCfgs[] = {
      {7, 2, 2, 2, 3},   // 0: N = 64, 224 x 64 tiles, waves 2 x 2 of 112 x 32, three-slot weight ring
      {13, 1, 2, 4, 0},  // 1: N % 128 == 0, 208 x 128 tiles (196-pixel bands), waves 1 x 4 of
                         //    208 x 32, weights in registers (per 32-deep half step, 3 deep)
  };
  if (cfg < 0) cfg = N == 64 ? 0 : 1;
  TORCH_CHECK(cfg < 2, "conv3x3_band: unknown configuration ", cfg);
  const Cfg cf = kCfgs[cfg];
  const int BM = 16 * cf.tm * cf.wm, BN = 16 * cf.tn * cf.wn, ntiles = (int)(N / BN);
  TORCH_CHECK(N % BN == 0, "conv3x3_band: N must be a multiple of the configuration's ", BN, " channels");
  const int R = (int)(rows > 0 ? rows : conv3x3_band_rows(W, H, BM));
  TORCH_CHECK(R > 0 && R * W <= BM, "conv3x3_band: a band of ", R, " rows of ", W, " pixels exceeds the ", BM,
              "-row tile");
  const int64_t rows_total = B * H, mtiles = (rows_total + R - 1) / R;
  TORCH_CHECK(mtiles * ntiles < (int64_t(1) << 31), "conv3x3_band: too many tiles");
  // halo rows: the most a band can need (a segment per image it touches, two padding rows each),
  // over the distinct first rows h0 = (t·R) mod H a band can start at
  int segs = 1;
  for (int64_t k = 0; k < H; ++k) {
    const int64_t h0 = (k * R) % H, n0 = std::min<int64_t>(H - h0, R);
    segs = std::max<int>(segs, (int)(1 + (R - n0 + H - 1) / H));
  }
  segs = (int)std::min<int64_t>(segs, B);
  const int hrows = (((R + 2 * segs) * ((int)W + 2) + 31) / 32) * 32;
  auto y = at::empty({B, N, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  // persistent blocks (stats only): two per CU, a multiple of ntiles, each a fixed channel tile and
  // one statistics group; without statistics one block per tile
  static const int cus = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  const int64_t groups =
      stats && cf.ring != 0 ? std::min<int64_t>(mtiles, std::max(1, 2 * cus / ntiles)) : mtiles;
  const auto fopt = x.options().dtype(at::kFloat);
  auto part = stats ? at::empty({3, N, groups}, fopt) : at::empty({0}, fopt);
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const BandGeo g{(int)B, (int)H, (int)W, (int)C, R, (int)rows_total};
  auto go = [&](auto kern, int ring) {
    const size_t lds = std::max<size_t>((size_t)hrows * 128 + (size_t)ring * BN * 128, (size_t)BM * (BN * 2 + 16) +
                                        (stats ? 0 : 0));
    TORCH_CHECK(lds <= 160 * 1024, "conv3x3_band: LDS budget exceeded (", lds, " B)");
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)(groups * ntiles)), dim3(256), lds, stream,
                       reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                       reinterpret_cast<uint16_t*>(y.data_ptr()), zeros, (int)N, g,
                       stats ? part.data_ptr<float>() : nullptr, ntiles, (int)mtiles, hrows);
    XDDP_HIP_CHECK(hipGetLastError());
  };
#define XDDP_BAND(TM_, WM_, TN_, WN_, RING_)                                      \
  do {                                                                             \
    if (stats) go(conv3x3_band_kernel<TM_, WM_, TN_, WN_, true, RING_>, RING_);    \
    else go(conv3x3_band_kernel<TM_, WM_, TN_, WN_, false, RING_>, RING_);         \
  } while (0)
  if (cfg == 0) XDDP_BAND(7, 2, 2, 2, 3);
  else XDDP_BAND(13, 1, 2, 4, 0);
#undef XDDP_BAND
  return {y, part};
}

}  // namespace kernels
}  // namespace xddp
