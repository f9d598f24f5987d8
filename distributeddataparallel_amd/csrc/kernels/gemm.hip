// Dense bf16 GEMM for the transformer linear layers (ViT-L/16, Llama-3-8B forward projections):
//
//   Y[M, N] = epilogue( A[M, K] · B[N, K]ᵀ )      (torch.nn.Linear: A = activations, B = weight)
//
// with the epilogues that otherwise cost an HBM pass each: + bias, + bias -> GELU (writing both
// the pre-activation the backward needs and the activation), + residual (beta = 1 accumulate).
//
// Structure (gfx950, CDNA4): one 256 x BN block tile per CU (8 waves = 2 (M) x 4 (N), each wave a
// 128 x BN/4 sub-tile = 8 x BN/64 MFMA accumulators of mfma_f32_16x16x32_bf16), BK = 64. Both
// operands go global -> LDS with global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip); each
// wave-instruction fills 8 full 128-B rows, the per-lane SOURCE address is pre-swizzled so the
// lane-linear LDS image has the XOR-swizzled chunk order the ds_read_b128 fragment reads want
// (conflict-free column-slice reads). Two LDS stages of 64 KB; each K-tile runs as four
// 16-MFMA phases whose fragment reads are issued one phase ahead, and the DMA of tile k+2 goes
// out at the one `s_waitcnt vmcnt(0)` + raw s_barrier of tile k, halfway through it (details at
// the loop); nothing else drains the pipeline (all LDS in one dynamic array, no other global
// loads in the loop). The MFMA computes the
// transposed tile (B rows as the first operand), so a lane's four accumulators are four
// consecutive output columns of one row: the C tile goes to LDS as 8-B writes and leaves as full
// 16-B row chunks, where the epilogue math runs. Block ids are remapped XCD-contiguously and
// each XCD's concurrent tiles form a GM x (32 / GM) block that shares A and B panels in its L2.
// Rows past M re-read row M - 1 and are not stored.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <type_traits>

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

constexpr int kBM = 256, kBK = 64, kWM = 2, kWN = 4, NW = kWM * kWN, kThreads = 64 * NW;

enum Epi : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiResidual = 3, kEpiDGelu = 4, kEpiStats = 5 };

// CONV: A is not a matrix but the implicit im2col of a 3x3 pad-1 convolution (NHWC bf16 input
// [B, IH, IW, C], weights OHWI [N][3][3][C] = B[N, 9C]): row m = output pixel (b, oh, ow), K-tile
// kt = tap (kt / (C/64)) x 64-channel block; the DMA source of a row is the input pixel under
// that tap, or a zero line for padding taps (no branch). Same pipeline as the dense GEMM; this is
// the ResNet-50 3x3 forward / stride-1 input gradient for N >= 256, where the 4-phase loop beats
// the 3-stage conv3x3.hip kernel (scripts/conv3x3_ceiling.py).
//
// DGS2 (MODE 2): the input gradient of a stride-2 3x3 pad-1 convolution as four phase GEMMs in one
// launch. dX pixel (2i + ph, 2j + pw) only receives the taps whose stride-2 window lands on it:
// with the 180-degree-rotated weight wr[ci][a][b][co] = w[co][2-a][2-b][ci],
//   dX[2i+ph][2j+pw] = sum over a in A(ph), b in A(pw) of dY[i + r(a)][j + s(b)] · wr[a][b]
// where A(0) = {1} (offset 0) and A(1) = {0 (offset 0), 2 (offset +1)}: phases of 1, 2, 2 and 4
// taps, K = taps x Cout. Row m of phase p = dY-grid pixel (b, i, j); its K-tiles DMA the dY pixels
// under the phase's taps (zero line past the bottom / right edge) and the matching Cout block of
// wr's tap (B = wr viewed [Cin, 9 Cout], ldb = 9 Cout); the C tile is written straight to the
// strided dX pixels — every dX pixel exactly once, no zero-fill, no scatter pass. Blocks are
// phase-major, heaviest phase first (4 taps, then the two 2-tap phases, then the 1-tap one), and
// the XCD remap / grouped tile order run inside each phase.
struct ConvGeo {
  int IH, IW, OH, OW, stride, C;
  const uint16_t* zeros;
  int XH = 0, XW = 0;  // DGS2: dX spatial size (even); IH/IW = OH/OW = the dY grid
};

constexpr int kModeDense = 0, kModeConv = 1, kModeDgS2 = 2;


__device__ __forceinline__ float bf(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

template <int BN, int EPI, int MODE = kModeDense>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_kernel(const uint16_t* __restrict__ A,
                                                              const uint16_t* __restrict__ B,
                                                              uint16_t* Y, uint16_t* __restrict__ Y2,
                                                              const uint16_t* __restrict__ bias,
                                                              const uint16_t* res, float* __restrict__ part,
                                                              int M, int N, int K, int ntiles, int64_t ldr,
                                                              ConvGeo cg) {
  constexpr int AI = kBM / 8 / NW, BI = BN / 8 / NW;  // DMA wave-instructions per stage (8 rows each)
  static_assert(AI * NW * 8 == kBM && BI * NW * 8 == BN, "tile rows must split evenly over the waves");
  constexpr int WTM = kBM / kWM, WTN = BN / kWN, TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE = (kBM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  constexpr bool CONV = MODE != kModeDense;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / kWN, wn = wid % kWN;
  // Tile order: the XCD remap gives each XCD a contiguous run of logical tiles (32 at a time on
  // its 32 CUs); logical tiles go through groups of GM m-tiles, M fastest inside a group, so such
  // a run is a GM x (32 / GM) block of tiles that shares GM A panels and 32 / GM B panels in that
  // XCD's L2 — instead of one A panel and 32 B panels (a full row of N tiles), which made every
  // XCD stream all of B (2.6x hipBLASLt's HBM bytes on 8192^3, profiles/r3_pmc_kernels.txt).
  constexpr int GM = BN == 256 ? 8 : 4;  // 8 x 4 tiles of 256 x 256, 4 x 8 of 256 x 128
  // DGS2: phase-major blocks (heaviest first), each phase a full M x N tile grid
  const int tiles = MODE == kModeDgS2 ? gridDim.x / 4 : gridDim.x;
  const int pidx = MODE == kModeDgS2 ? blockIdx.x / tiles : 0;
  const int ph = pidx == 0 || pidx == 2, pw = pidx <= 1;  // phase order (1,1) (0,1) (1,0) (0,0)
  const int wg = dev::xcd_remap(blockIdx.x - pidx * tiles, tiles);
  const int mtiles = tiles / ntiles, grp = wg / (GM * ntiles), first_m = grp * GM;
  const int gm = min(mtiles - first_m, GM), local = wg - grp * GM * ntiles;
  const int mt = first_m + local % gm, nt = local / gm;
  const int n0 = nt * BN, m0 = mt * kBM;
  const int pos = lane & 7;  // 16-B slot this lane fills in its 128-B LDS row
  // DGS2: the phase's tap count (1 << (ph + pw)) times the Cout blocks; ldb = 9 Cout
  const int nk = MODE == kModeDgS2 ? ((cg.C / kBK) << (ph + pw)) : K / kBK;
  const int ldb = MODE == kModeDgS2 ? 9 * cg.C : K;

  // DMA sources: lane l of wave w fills 16-B slot (l & 7) of rows (w*AI + i)*8 + (l >> 3); the
  // offsets are recomputed per issue from two per-lane values (few live VGPRs: the 4-phase loop
  // needs ~224 for accumulators and fragments). Rows past M re-read row M - 1 (never stored).
  const int drow = wid * 8 + (lane >> 3);                    // + i * 8 NW (A, i < AI) / j * 8 NW (B)
  const int dchunk = 8 * (pos ^ ((drow >> 1) & 7));          // (row >> 1) & 7 is the same for row + 64 i
  // CONV: per A row, the top-left input pixel of its 3x3 window (packed (ih0 + 2) << 16 | (iw0 + 2))
  // and that pixel's element offset (may point before the row for padding windows; never
  // dereferenced then). Host-checked: the input has < 2^31 elements.
  int vmask[CONV ? AI : 1], cbase[CONV ? AI : 1];  // CONV: taps inside the image (bit t), window offset
  if constexpr (MODE == kModeDgS2) {
    // row = dY-grid pixel (b, i, j); tap t of the phase reads dY (i + r_t, j + s_t), r_t, s_t in {0, 1}
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = min(m0 + drow + i * 8 * NW, M - 1);
      const int hw = cg.OH * cg.OW, b = row / hw, rem = row - b * hw, y = rem / cg.OW, x = rem - y * cg.OW;
      int m = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = ph ? (t >> pw) : 0, sx = pw ? (t & 1) : 0;
        m |= (y + r < cg.IH && x + sx < cg.IW) << t;
      }
      vmask[i] = m;
      cbase[i] = ((b * cg.IH + y) * cg.IW + x) * cg.C + dchunk;
    }
  } else if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = min(m0 + drow + i * 8 * NW, M - 1);
      const int hw = cg.OH * cg.OW, b = row / hw, rem = row - b * hw, oh = rem / cg.OW, ow = rem - oh * cg.OW;
      const int st = cg.stride & 0xffff, ih0 = oh * st - 1, iw0 = ow * st - 1;
      int m = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        m |= ((unsigned)(ih0 + t / 3) < (unsigned)cg.IH && (unsigned)(iw0 + t % 3) < (unsigned)cg.IW) << t;
      vmask[i] = m;
      cbase[i] = ((b * cg.IH + ih0) * cg.IW + iw0) * cg.C + dchunk;
    }
  }
  auto issue = [&](int kt, int buf) {
    uint8_t* As = smem + buf * STAGE;
    int boff = kt * kBK;  // B's K offset (DGS2: the tap's block of wr)
    if constexpr (MODE == kModeDgS2) {
      const int lg = cg.stride >> 16, tap = kt >> lg, cb = kt & ((1 << lg) - 1);
      const int tr = pw ? tap >> 1 : tap, tc = pw ? tap & 1 : 0;  // row / column tap of the phase
      const int r = ph ? tr : 0, sx = pw ? tc : 0, a = ph ? 2 * tr : 1, bb = pw ? 2 * tc : 1;
      const int toff = (r * cg.IW + sx) * cg.C + cb * kBK;
      boff = (a * 3 + bb) * cg.C + cb * kBK;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = (vmask[i] >> tap) & 1;
        const uint16_t* src = ok ? A + (cbase[i] + toff) : cg.zeros;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(As + (wid * 8 + i * 8 * NW) * 128), 16, 0, 0);
      }
    } else if constexpr (CONV) {
      // C / 64 is a power of two (host-checked): cg.stride's high half carries its log2
      const int lg = cg.stride >> 16, tap = kt >> lg, cb = kt & ((1 << lg) - 1), r = (tap * 11) >> 5, sx = tap - 3 * r;
      const int toff = (r * cg.IW + sx) * cg.C + cb * kBK;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = (vmask[i] >> tap) & 1;
        const uint16_t* src = ok ? A + (cbase[i] + toff) : cg.zeros;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(As + (wid * 8 + i * 8 * NW) * 128), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int row = min(m0 + drow + i * 8 * NW, M - 1);
        const uint16_t* src = A + (uint32_t)row * (uint32_t)K + (uint32_t)(dchunk + kt * kBK);
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(As + (wid * 8 + i * 8 * NW) * 128), 16, 0, 0);
      }
    }
    uint8_t* Bs = As + kBM * 128;
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const uint16_t* src = B + (uint32_t)(n0 + drow + j * 8 * NW) * (uint32_t)ldb + (uint32_t)(dchunk + boff);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(Bs + (wid * 8 + j * 8 * NW) * 128), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  {
    // 4-phase: each K-tile is 4 phases, one per quadrant (A half x B half) of the wave's output,
    // 16 MFMAs each; the fragments of the next phase are read while the current phase's MFMAs
    // run, so the MFMA pipe never waits on LDS. The phase order alternates between even and odd
    // K-tiles so the last phase of a tile and the first of the next use different fragment
    // registers: even (A0,B0) (A0,B1) (A1,B1) (A1,B0), odd (A0,B1) (A0,B0) (A1,B0) (A1,B1).
    // One barrier per K-tile, between phases 1 and 2: by then this wave's reads of the tile's
    // stage are done (lgkmcnt(0)) and its DMA of tile t+1 (issued after the previous tile's
    // barrier, four phases ago) has landed (vmcnt(0) - nothing else is in flight); after it the
    // DMA of tile t+2 goes into this tile's stage and phases 2-3 read the first fragments of t+1.
    constexpr int HA = TM / 2, HB = TN / 2;
    static_assert(HB >= 1, "B halves need at least one 16-column fragment");
    bf16x8 fa0[2][HA], fa1[2][HA], fb0[2][HB], fb1[2][HB];  // [k-half][fragment]
    // fragment rows of a wave are row0 + 16 i: the XOR term ((row >> 1) & 7) is the same for all
    // of them, so each k-half needs ONE per-lane byte offset; the rest is an immediate
    const int ra = wm * WTM + (lane & 15), rb = wn * WTN + (lane & 15);
    uint32_t a_lds[2], b_lds[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      a_lds[kh] = ra * 128 + 16 * ((kh * 4 + (lane >> 4)) ^ ((ra >> 1) & 7));
      b_lds[kh] = kBM * 128 + rb * 128 + 16 * ((kh * 4 + (lane >> 4)) ^ ((rb >> 1) & 7));
    }
    auto ldA = [&](bf16x8 (&f)[2][HA], int half, int buf) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < HA; ++i)
          f[kh][i] = *reinterpret_cast<const bf16x8*>(smem + buf * STAGE + a_lds[kh] + (half * HA + i) * 16 * 128);
    };
    auto ldB = [&](bf16x8 (&f)[2][HB], int half, int buf) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int j = 0; j < HB; ++j)
          f[kh][j] = *reinterpret_cast<const bf16x8*>(smem + buf * STAGE + b_lds[kh] + (half * HB + j) * 16 * 128);
    };
    auto mma = [&](const bf16x8 (&a)[2][HA], auto ah, const bf16x8 (&b)[2][HB], auto bh) {
      constexpr int AH = decltype(ah)::value, BHV = decltype(bh)::value;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < HA; ++i)
#pragma unroll
          for (int j = 0; j < HB; ++j)
            acc[AH * HA + i][BHV * HB + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[kh][j], a[kh][i], acc[AH * HA + i][BHV * HB + j], 0, 0, 0);
    };
    // One phase = the fragment reads for the NEXT phase interleaved into this phase's MFMAs,
    // MFMA first: the wait the compiler puts before the first MFMA then covers only the reads of
    // the previous phase (whose MFMAs hid them), never the ones just issued. sched_barrier(0)
    // keeps every instruction inside its phase.
    auto interleave = [&](auto nld) {
      constexpr int NLD = decltype(nld)::value, NM = 2 * HA * HB;
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // one MFMA (waits for this phase's fragments)
      __builtin_amdgcn_sched_group_barrier(0x100, NLD, 0);     // the next phase's reads
      __builtin_amdgcn_sched_group_barrier(0x008, NM - 1, 0);  // the rest of the MFMAs
      __builtin_amdgcn_sched_barrier(0);
    };
    using LA = std::integral_constant<int, 2 * HA>;  // reads of an A half (both k-halves)
    using LB = std::integral_constant<int, 2 * HB>;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // The loop runs tile PAIRS and is branch-free: a wait counter cannot be tracked through a
    // conditional load (the compiler then waits for everything), so the last tiles re-read a
    // valid stage and re-stage the last K-tile instead of skipping; those values are never used.
    // An odd tile count gets a zero tile in front (virtual tile 0 = zeros written to stage 0, real
    // tile k = virtual k + 1): its MFMAs add exact zeros, and no tail code raises the register
    // pressure of the loop.
    const int odd = nk & 1, nv = nk + odd;
    auto sync = [&](int t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(min(t + 2, nv - 1) - odd, t & 1);
    };
    if (odd) {
      for (int q = tid; q < STAGE / 16; q += kThreads) reinterpret_cast<u32x4*>(smem)[q] = u32x4{0u, 0u, 0u, 0u};
    } else {
      issue(0, 0);
    }
    issue(1 - odd, 1);  // virtual tile 1: real tile 1 (even count) / 0 (odd count)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AI + BI) : "memory");  // stage 0 ready, stage 1 in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    ldA(fa0, 0, 0);
    ldB(fb0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < nv; t += 2) {
      // even tile t (stage 0): enters with A0, B0 of t
      ldB(fb1, 1, 0);
      mma(fa0, I0{}, fb0, I0{});
      interleave(LB{});
      ldA(fa1, 1, 0);
      mma(fa0, I0{}, fb1, I1{});
      interleave(LA{});
      sync(t);
      __builtin_amdgcn_sched_barrier(0);
      ldA(fa0, 0, 1);  // A0 of t + 1
      mma(fa1, I1{}, fb1, I1{});
      interleave(LA{});
      ldB(fb1, 1, 1);  // B1 of t + 1
      mma(fa1, I1{}, fb0, I0{});
      interleave(LB{});
      // odd tile t + 1 (stage 1): enters with A0, B1 of t + 1
      ldB(fb0, 0, 1);
      mma(fa0, I0{}, fb1, I1{});
      interleave(LB{});
      ldA(fa1, 1, 1);
      mma(fa0, I0{}, fb0, I0{});
      interleave(LA{});
      sync(t + 1);
      __builtin_amdgcn_sched_barrier(0);
      ldA(fa0, 0, 0);  // A0 of t + 2
      mma(fa1, I1{}, fb0, I0{});
      interleave(LA{});
      ldB(fb0, 0, 0);  // B0 of t + 2
      mma(fa1, I1{}, fb1, I1{});
      interleave(LB{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-stage DMAs land before the C tile reuses LDS
  }

  // ---- epilogue: fp32 -> bf16 C tile through LDS (rows padded 16 B), 16-B row chunks out ----
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done reading the stages
  constexpr int CST = BN * 2 + 16;
  uint8_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wm * WTM + i * 16 + (lane & 15);
      const int col = wn * WTN + j * 16 + (lane >> 4) * 4;
      f32x4 v = acc[i][j];
      if (EPI == kEpiBias || EPI == kEpiBiasGelu) {  // bias in fp32 before the one rounding
        const uint2 bb = *reinterpret_cast<const uint2*>(bias + n0 + col);
        v[0] += bf(bb.x & 0xffffu);
        v[1] += bf(bb.x >> 16);
        v[2] += bf(bb.y & 0xffffu);
        v[3] += bf(bb.y >> 16);
      }
      uint2 pk;
      pk.x = dev::pack_bf16x2(v[0], v[1]);
      pk.y = dev::pack_bf16x2(v[2], v[3]);
      *reinterpret_cast<uint2*>(Cs + row * CST + col * 2) = pk;
    }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  constexpr int CPR = BN / 8;
  static_assert(kThreads % CPR == 0, "readout mapping needs a fixed chunk column per thread");
  const int cc = tid % CPR;
  const int rows_valid = min(kBM, M - m0);
  u32x4 rb{};
  if (EPI == kEpiResidual && bias) rb = *reinterpret_cast<const u32x4*>(bias + n0 + cc * 8);
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // kEpiDGelu: this thread's column sums
  // kEpiStats: per-channel shifted sums (shift = the tile's row 0, always valid) for the following
  // BatchNorm's statistics, as conv3x3.hip's epilogue (csum = sum d, cssq = sum d^2)
  float cssq[EPI == kEpiStats ? 8 : 1], st_n = 0.f;
  u32x4 st_k{};
  if (EPI == kEpiStats) {
#pragma unroll
    for (int e = 0; e < 8; ++e) cssq[e] = 0.f;
    st_k = *reinterpret_cast<const u32x4*>(Cs + cc * 16);
  }
  // rows tid / CPR + (kThreads / CPR)·i; each batch's LDS reads issued before its stores (rows past M
  // read row rows_valid - 1 and are skipped): a read-then-use per row compiled to one ds_read +
  // s_waitcnt lgkmcnt(0) round trip per row
  auto out_row = [&](int row, u32x4 v) {
    int64_t off = (int64_t)(m0 + row) * N + n0 + cc * 8;
    if constexpr (MODE == kModeDgS2) {  // dY-grid pixel (b, i, j) -> dX pixel (b, 2i + ph, 2j + pw)
      const int m = m0 + row, hw = cg.OH * cg.OW, b = m / hw, rem = m - b * hw, y = rem / cg.OW, x = rem - y * cg.OW;
      off = (((int64_t)b * cg.XH + 2 * y + ph) * cg.XW + 2 * x + pw) * N + n0 + cc * 8;
    }
    if (EPI == kEpiBiasGelu) {
      *reinterpret_cast<u32x4*>(Y + off) = v;  // pre-activation (the backward's dGELU input)
      u32x4 g;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        g[e] = dev::pack_bf16x2(dev::gelu(bf(v[e] & 0xffffu)), dev::gelu(bf(v[e] >> 16)));
      *reinterpret_cast<u32x4*>(Y2 + off) = g;
    } else if (EPI == kEpiDGelu) {
      // dh = (g·W, the bf16 C tile) · gelu'(h) in fp32; the fp32 dh also feed the column sums
      const u32x4 hv = *reinterpret_cast<const u32x4*>(res + (int64_t)(m0 + row) * ldr + n0 + cc * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = bf(v[e] & 0xffffu) * dev::gelu_grad(bf(hv[e] & 0xffffu));
        const float hi = bf(v[e] >> 16) * dev::gelu_grad(bf(hv[e] >> 16));
        csum[2 * e] += lo;
        csum[2 * e + 1] += hi;
        v[e] = dev::pack_bf16x2(lo, hi);
      }
      *reinterpret_cast<u32x4*>(Y + off) = v;
    } else if (EPI == kEpiStats) {
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(Y + off));
      st_n += 1.f;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float d0 = bf(v[h] & 0xffffu) - bf(st_k[h] & 0xffffu);
        const float d1 = bf(v[h] >> 16) - bf(st_k[h] >> 16);
        csum[2 * h] += d0;
        csum[2 * h + 1] += d1;
        cssq[2 * h] = fmaf(d0, d0, cssq[2 * h]);
        cssq[2 * h + 1] = fmaf(d1, d1, cssq[2 * h + 1]);
      }
    } else if (EPI == kEpiResidual) {
      // y = res + (A·Bᵀ, already rounded to bf16 in the C tile) [+ bias]: one extra rounding of
      // the product against addmm_'s single one (the residual term dominates the sum)
      const u32x4 r = *reinterpret_cast<const u32x4*>(res + (int64_t)(m0 + row) * ldr + n0 + cc * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = bf(r[e] & 0xffffu) + bf(v[e] & 0xffffu), hi = bf(r[e] >> 16) + bf(v[e] >> 16);
        if (bias) {
          lo += bf(rb[e] & 0xffffu);
          hi += bf(rb[e] >> 16);
        }
        v[e] = dev::pack_bf16x2(lo, hi);
      }
      *reinterpret_cast<u32x4*>(Y + off) = v;
    } else {
      *reinterpret_cast<u32x4*>(Y + off) = v;
    }
  };
  constexpr int NIT = kBM * CPR / kThreads, RSTR = kThreads / CPR, EB = NIT < 4 ? NIT : 4;
  static_assert(kBM * CPR % kThreads == 0, "readout rows must divide evenly over the threads");
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
      if (i0 + j < NIT && row < rows_valid) out_row(row, vv[j]);
    }
  }
  if (EPI == kEpiStats) {
    // lanes sharing cc (xor over the lane bits above log2(CPR)), then the waves through LDS; one
    // (count, mean, M2) per channel and tile, group-minor: part[q][N][mtiles] (bn_stats_from_partials)
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
      st_n += __shfl_xor(st_n, o, 64);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        csum[e] += __shfl_xor(csum[e], o, 64);
        cssq[e] += __shfl_xor(cssq[e], o, 64);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // C tile reads done: reuse smem
    float* red = reinterpret_cast<float*>(smem);                      // [NW][2][BN] sums, [NW][CPR] counts
    float* redn = red + NW * 2 * BN;
    float* redk = redn + NW * CPR;                                    // [BN] the shifts
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wid * 2 + 0) * BN + cc * 8 + e] = csum[e];
        red[(wid * 2 + 1) * BN + cc * 8 + e] = cssq[e];
        if (wid == 0) redk[cc * 8 + e] = (e & 1) ? bf(st_k[e >> 1] >> 16) : bf(st_k[e >> 1] & 0xffffu);
      }
      redn[wid * CPR + cc] = st_n;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int G = gridDim.x / ntiles;
    for (int c = tid; c < BN; c += kThreads) {
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
  if (EPI == kEpiDGelu) {
    // column sums of the tile: the kThreads / CPR row groups meet in LDS past the C tile, then
    // thread c < BN writes part[m-tile][n0 + c] (colsum_partials adds the m-tiles up)
    constexpr int RG = kThreads / CPR;
    float* red = reinterpret_cast<float*>(smem + kBM * CST);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid / CPR) * BN + cc * 8 + e] = csum[e];
    __syncthreads();
    if (tid < BN) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < RG; ++r) t += red[r * BN + tid];
      part[(int64_t)mt * N + n0 + tid] = t;
    }
  }
}

template <int BN, int EPI, int MODE = kModeDense>
void launch_gemm(const at::Tensor& a, const at::Tensor& b, uint16_t* y, uint16_t* y2, const uint16_t* bias,
                 const uint16_t* res, float* part, int64_t ldr, int M, int N, int K, hipStream_t stream,
                 const ConvGeo& cg = ConvGeo{}) {
  const int mtiles = (M + kBM - 1) / kBM, ntiles = N / BN, phases = MODE == kModeDgS2 ? 4 : 1;
  // stages | C tile (+ the column-sum exchange of the dGELU epilogue)
  const size_t lds = std::max<size_t>((size_t)2 * (kBM + BN) * 128,
                                      (size_t)kBM * (BN * 2 + 16) + (EPI == kEpiDGelu ? (size_t)2048 * NW : 0));
  static bool attr = false;
  if (!attr) {
    XDDP_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_nt_kernel<BN, EPI, MODE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt_kernel<BN, EPI, MODE>), dim3(phases * mtiles * ntiles), dim3(kThreads), lds, stream,
                     reinterpret_cast<const uint16_t*>(a.data_ptr()), reinterpret_cast<const uint16_t*>(b.data_ptr()),
                     y, y2, bias, res, part, M, N, K, ntiles, ldr, cg);
  XDDP_HIP_CHECK(hipGetLastError());
}

// Tile width: 256 x 256 unless the 256 x 128 grid fills the CUs' last round better (one block
// per CU: a 256 x 256 grid of 800 tiles on 256 CUs runs 4 rounds, the last 1/8 full).
int pick_bn(int64_t M, int64_t N, int cus) {
  if (N % 256) return 128;
  const int64_t mt = (M + kBM - 1) / kBM;
  const int64_t r256 = (mt * (N / 256) + cus - 1) / cus, r128 = (mt * (N / 128) + cus - 1) / cus;
  // a 256 x 128 tile does half the work at ~1.15x the per-FLOP cost (more B traffic per MFMA)
  return 2.0 * r256 <= 1.15 * r128 ? 256 : 128;
}

}  // namespace

// a [M, K] bf16 (row-major, rows 16-B aligned), w [N, K] bf16 -> y [M, N] bf16 = a · wᵀ with
// epilogue `epi`: 0 none, 1 + bias, 2 + bias then GELU (returns {pre-activation, activation}),
// 3 + residual (y may be `out` = the residual itself: the in-place x += a·wᵀ of a pre-norm block;
// + bias if given), 4 the GELU backward of an MLP: `residual` is the pre-activation h and the
// result is {dh = (a·wᵀ)·gelu'(h), Σ_rows dh} (the second in bias's dtype if a bias is passed —
// only its dtype is used — else fp32). K % 64 == 0, N % 128 == 0.
std::vector<at::Tensor> gemm_nt(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                int64_t epi, const c10::optional<at::Tensor>& residual,
                                const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(a.is_cuda() && w.is_cuda() && a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "gemm_nt: bf16 CUDA operands expected");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1) && a.stride(1) == 1 && a.stride(0) == a.size(1) &&
                  w.is_contiguous(),
              "gemm_nt: a [M, K] and w [N, K] must be contiguous with matching K");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31) && K % 64 == 0 && K > 0 && N % 128 == 0 && N > 0,
              "gemm_nt: needs K % 64 == 0 and N % 128 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "gemm_nt: 16-B aligned operands required");
  TORCH_CHECK(epi >= 0 && epi <= 5, "gemm_nt: epi must be 0..5");
  const bool has_bias = bias.has_value() && bias->defined();
  if (has_bias)
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous() &&
                    reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0,
                "gemm_nt: bias must be a contiguous bf16 [N] vector");
  TORCH_CHECK((epi != 1 && epi != 2) || has_bias, "gemm_nt: epilogues 1 and 2 need a bias");
  at::Tensor res;
  int64_t ldr = N;
  if (epi == 3 || epi == 4) {
    TORCH_CHECK(residual.has_value() && residual->defined(), "gemm_nt: epilogues 3 and 4 need a residual / h");
    res = *residual;
    TORCH_CHECK(res.scalar_type() == at::kBFloat16 && res.dim() == 2 && res.size(0) == M && res.size(1) == N &&
                    res.stride(1) == 1 && res.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(res.data_ptr()) % 16 == 0,
                "gemm_nt: residual must be bf16 [M, N] with unit column stride and 16-B aligned rows");
    ldr = res.stride(0);
  }
  at::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 2 && y.size(0) == M && y.size(1) == N && y.is_contiguous(),
                "gemm_nt: out must be a contiguous bf16 [M, N] tensor");
    TORCH_CHECK(epi < 4, "gemm_nt: epilogues 4 and 5 allocate their outputs");
    TORCH_CHECK(epi != 3 || y.data_ptr() == res.data_ptr() || !(y.data_ptr() < (char*)res.data_ptr() + res.nbytes() &&
                                                                  res.data_ptr() < (char*)y.data_ptr() + y.nbytes()),
                "gemm_nt: out may alias the residual only exactly");
  } else {
    y = at::empty({M, N}, a.options());
  }
  at::Tensor y2 = epi == 2 ? at::empty({M, N}, a.options()) : at::Tensor();
  auto stream = c10::hip::getCurrentHIPStream(a.device().index()).stream();
  int cus = 256;
  {
    static int cached = 0;
    if (!cached) {
      int v = 0;
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, a.device().index()) == hipSuccess && v > 0)
        cached = v;
      else
        cached = 256;
    }
    cus = cached;
  }
  const int BN = pick_bn(M, N, cus);
  auto* yp = reinterpret_cast<uint16_t*>(y.data_ptr());
  auto* y2p = epi == 2 ? reinterpret_cast<uint16_t*>(y2.data_ptr()) : nullptr;
  const auto* bp = has_bias ? reinterpret_cast<const uint16_t*>(bias->data_ptr()) : nullptr;
  const auto* rp = (epi == 3 || epi == 4) ? reinterpret_cast<const uint16_t*>(res.data_ptr()) : nullptr;
  at::Tensor part = epi == 4   ? at::empty({(M + kBM - 1) / kBM, N}, a.options().dtype(at::kFloat))
                   : epi == 5 ? at::empty({3, N, (M + kBM - 1) / kBM}, a.options().dtype(at::kFloat))
                              : at::Tensor();
  float* pp = epi >= 4 ? part.data_ptr<float>() : nullptr;
#define XDDP_GEMM(BN_)                                                                                    \
  switch (epi) {                                                                                          \
    case 0: launch_gemm<BN_, kEpiNone>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break;     \
    case 1: launch_gemm<BN_, kEpiBias>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break;     \
    case 2: launch_gemm<BN_, kEpiBiasGelu>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break; \
    case 3: launch_gemm<BN_, kEpiResidual>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break; \
    case 4: launch_gemm<BN_, kEpiDGelu>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break;    \
    default: launch_gemm<BN_, kEpiStats>(a, w, yp, y2p, bp, rp, pp, ldr, (int)M, (int)N, (int)K, stream); break;   \
  }
  if (BN == 256) {
    XDDP_GEMM(256)
  } else {
    XDDP_GEMM(128)
  }
#undef XDDP_GEMM
  if (epi == 2) return {y, y2};
  if (epi == 5) return {y, part};
  if (epi == 4) {
    at::Tensor db = at::empty({N}, has_bias ? bias->options() : a.options().dtype(at::kFloat));
    colsum_partials(part, db);
    return {y, db};
  }
  return {y};
}

// 3x3 pad-1 convolution (stride 1 or 2) on the dense GEMM pipeline (ConvGeo): x [B, C, IH, IW]
// bf16 channels_last, w [N, C, 3, 3] bf16 channels_last (OHWI). Returns {y [B, N, OH, OW]
// channels_last, statistics partials [3, N, mtiles] group-minor (empty without stats)}.
// N % 128 == 0, C % 64 == 0.
std::vector<at::Tensor> conv3x3_gemm(const at::Tensor& x, const at::Tensor& w, int64_t stride, bool stats,
                                     const uint16_t* zeros) {
  const int64_t B = x.size(0), C = x.size(1), IH = x.size(2), IW = x.size(3), N = w.size(0);
  TORCH_CHECK(C % 64 == 0 && N % 128 == 0 && x.numel() < (int64_t(1) << 31), "conv3x3_gemm: unsupported shape");
  const int64_t OH = (IH - 1) / stride + 1, OW = (IW - 1) / stride + 1, M = B * OH * OW;
  auto y = at::empty({B, N, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  // 256 x 128 tiles: the 256-wide tile's conv addressing spills ~60 registers past the 256 the
  // 4-phase loop leaves (kernel_resources.py), the 128-wide one fits in 186
  constexpr int BN = 128;
  const int64_t mtiles = (M + kBM - 1) / kBM;
  at::Tensor part = stats ? at::empty({3, N, mtiles}, x.options().dtype(at::kFloat))
                          : at::empty({0}, x.options().dtype(at::kFloat));
  const int lg = __builtin_ctz((unsigned)(C / 64));
  TORCH_CHECK((C / 64) == (int64_t(1) << lg), "conv3x3_gemm: C / 64 must be a power of two");
  // (stride | log2(C / 64) << 16: the kernel splits K-tiles into tap / channel block by shifts)
  const ConvGeo cg{(int)IH, (int)IW, (int)OH, (int)OW, (int)stride | (lg << 16), (int)C, zeros};
  auto* yp = reinterpret_cast<uint16_t*>(y.data_ptr());
  float* pp = stats ? part.data_ptr<float>() : nullptr;
  const int K = (int)(9 * C);
  if (stats) launch_gemm<BN, kEpiStats, kModeConv>(x, w, yp, nullptr, nullptr, nullptr, pp, N, (int)M, (int)N, K, stream, cg);
  else launch_gemm<BN, kEpiNone, kModeConv>(x, w, yp, nullptr, nullptr, nullptr, pp, N, (int)M, (int)N, K, stream, cg);
  return {y, part};
}

// Input gradient of a stride-2 3x3 pad-1 convolution (DGS2, four phase GEMMs in one launch):
// dy [B, Cout, OH, OW] bf16 channels_last, wr = the rotated weight [Cin, Cout, 3, 3] channels_last
// (OHWI memory: wr[ci][a][b][co] = w[co][2-a][2-b][ci], conv3x3_rot_weight) -> dx [B, Cin, XH, XW]
// channels_last with XH = 2 OH, XW = 2 OW (even input sizes). Cin % 128 == 0, Cout / 64 a power of two.
at::Tensor conv3x3_dgrad_s2_gemm(const at::Tensor& dy, const at::Tensor& wr, int64_t XH, int64_t XW,
                                 const uint16_t* zeros) {
  const int64_t B = dy.size(0), Co = dy.size(1), OH = dy.size(2), OW = dy.size(3), Ci = wr.size(0);
  TORCH_CHECK(wr.size(1) == Co && XH == 2 * OH && XW == 2 * OW, "conv3x3_dgrad_s2_gemm: even input sizes only");
  TORCH_CHECK(Co % 64 == 0 && Ci % 128 == 0 && dy.numel() < (int64_t(1) << 31) && B * XH * XW * Ci < (int64_t(1) << 40),
              "conv3x3_dgrad_s2_gemm: unsupported shape");
  const int lg = __builtin_ctz((unsigned)(Co / 64));
  TORCH_CHECK((Co / 64) == (int64_t(1) << lg), "conv3x3_dgrad_s2_gemm: Cout / 64 must be a power of two");
  const int64_t M = B * OH * OW;
  auto dx = at::empty({B, Ci, XH, XW}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  ConvGeo cg{(int)OH, (int)OW, (int)OH, (int)OW, 2 | (lg << 16), (int)Co, zeros};
  cg.XH = (int)XH;
  cg.XW = (int)XW;
  launch_gemm<128, kEpiNone, kModeDgS2>(dy, wr, reinterpret_cast<uint16_t*>(dx.data_ptr()), nullptr, nullptr, nullptr,
                                        nullptr, Ci, (int)M, (int)Ci, (int)(4 * Co), stream, cg);
  return dx;
}

}  // namespace kernels
}  // namespace xddp
