// 1x1 convolution (NHWC, bf16) as an MFMA GEMM with BatchNorm fused into its prologue and
// epilogue, for gfx950 / CDNA4.
//
//   Y[M, N] = op(X)[M, K] · W[N, K]^T        M = batch·OH·OW pixels, K = Cin, N = Cout
//   op      = identity, or relu(x·s_k + b_k) per input channel (the PREVIOUS BatchNorm's apply,
//             so its normalized activation is never written to HBM)
//   epilogue: bf16 Y plus, per output channel, the batch statistics this conv's own BatchNorm
//             needs, so BN does not re-read Y for its stats pass.
//
// Why this shape (profiles/): at ResNet-50 bs256 the 1x1 convs are
// HBM-bound (K = 64..2048 is short), and every BN pass over an activation costs as much as the
// conv itself. Fusing removes whole activation passes; the GEMM itself only has to stream.
//
// Structure: 256 threads = 4 waves (2 x 2), block tile BM x BN x 64, each wave (BM/2) x (BN/2)
// built from mfma_f32_16x16x32_bf16 tiles. Operands are staged global -> VGPR -> LDS (so the BN
// prologue is applied once per element, in registers), two LDS buffers, the next K-tile's loads
// issued before the current tile's MFMAs (2-phase pipeline). LDS rows are 128 B (64 bf16) with the
// 16-B chunk index XOR-swizzled by (row >> 1) & 7, so the 16 lanes of a ds_read_b128 group hit 16
// distinct bank groups. A block walks several M-tiles of one N-tile (grid sized to the CU count)
// and merges their statistics in registers (Chan's parallel mean/M2), so the per-channel
// partials a finalize kernel has to merge are few. Block ids are remapped XCD-contiguously so
// the blocks sharing an A panel share one L2.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
using dev::f32x4;
using dev::u32x4;

constexpr int kBK = 64;       // K per tile (one 128-B LDS row per operand row)
constexpr bool NTSTORE = true;  // streaming (non-temporal) output stores

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ ((row >> 1) & 7)); }

// LDS-only workgroup barrier: __syncthreads() also waits vmcnt(0), which would drain the
// prefetched global loads that are meant to stay in flight across it (guide §5 "Pipelining
// across barriers"). LDS traffic is ordered by lgkmcnt(0) + s_barrier alone.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float bf16_round(float v) { return __uint_as_float(dev::pack_bf16x2(v, 0.f) << 16); }

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s lds_tr16(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// EPI (input-gradient GEMM of a bottleneck's conv1 whose input is the previous block's output):
// the C tile dX (gradient through conv1) is combined with the gradient the same tensor gets
// through the identity path (add), masked by the previous block's final ReLU (bits), stored as
// g — that block's d(residual) / BN-backward input — and reduced per channel into the previous
// BN's backward partials (sum g, sum g·(y - mean)) in bn_bwd_finalize's [groups][C][2] layout.
// The previous block's separate BN-backward reduce pass (which re-read both gradients) is gone.
// Second form (add = bits = nullptr, ss set): the input-gradient GEMM of a bottleneck's conv3,
// whose input is relu(bn2(y2)) with a single consumer: g = dX masked by relu(y2·s + t) > 0 (the
// mask recomputed from the BN input and its scale/shift), reduced into bn2's backward partials —
// bn2's separate BN-backward reduce pass over (dX, y2) is gone.
// add_h / add_w > 0 (first form): add is the compact input gradient of a stride-2 1x1 conv
// (the downsample branch) over the same tensor — [B][ceil(H/2)][ceil(W/2)][C] — and only the
// even-(h, w) pixels of the H x W output receive it. MIOpen's strided dgrad wrote that gradient
// at full resolution, three quarters of it zeros (plus a separate zero-fill pass).
struct EpiBN {
  const uint16_t* add;
  const uint16_t* y;
  const uint8_t* bits;
  const float* mean;
  float* part;
  const float* ss;  // [2][C] scale, shift (mask recompute form)
  int add_h, add_w;
};

// Prologue side output (PRO 1, 4, 5; forward, stride 1): the staged operand op(X) IS a BatchNorm
// apply's output — BN2's relu(y2·s + t) for a bottleneck's conv3, or a block's final
// relu(y3·s + t + r) for the next block's conv1 — so the blocks of N-tile 0 also store it (and,
// for PRO 4/5, its ReLU bit mask in bn_apply's byte-per-8-channels layout) instead of a separate
// apply pass writing it and this GEMM reading it back. rss: PRO 5's residual is a downsample's raw
// conv output whose BN apply (bf16(r·rs + rh), as that BN's own apply would store it) is folded in
// too. nbt1 / nbt2: the applied BNs' num_batches_tracked, bumped once by block 0.
struct ProOut {
  uint16_t* out;
  uint8_t* bits;
  const float* rss;
  int64_t* nbt1;
  int64_t* nbt2;
};

struct RowMap {  // output pixel m -> input row (strided 1x1 conv reads every stride-th pixel)
  int OH, OW, IH, IW, stride;
  template <bool STRIDED>
  __device__ __forceinline__ int64_t in_row(int m) const {  // M < 2^31 (host-checked)
    if (!STRIDED) return m;
    const int hw = OH * OW;
    const int n = m / hw, r = m - n * hw;
    const int oh = r / OW, ow = r - oh * OW;
    return ((int64_t)n * IH + oh * stride) * IW + (int64_t)ow * stride;
  }
};

// PRO: 0 = plain A; 1 = relu(A·s_k + b_k) (the previous BN's apply); 2 = a_k·A + b_k·X2 + c_k, the
// BatchNorm-backward elementwise pass (A = masked upstream gradient, X2 = the BN input) folded
// into the input-gradient GEMM so that gradient is never written to HBM; 3 = as 2 with the BN's
// ReLU mask recomputed in registers: A -> (X2·s_k + t_k > 0) ? A : 0; 4 = relu(A·s_k + t_k + X2)
// (a bottleneck's final BN + residual + ReLU, X2 = the identity); 5 = as 4 with the identity a
// deferred downsample BN's raw output, X2 -> bf16(X2·rs_k + rh_k) (ProOut::rss).
// BT: the B operand is given K-major (Wt[k][n], e.g. the forward weight W[n_out][k_in] used as Wᵀ by
// the input-gradient GEMM): staged as [64 k][BN n] rows (padded 32 B) and read into fragments with
// the transposing ds_read_b64_tr_b16, so no transposed weight copy is made.
// OCC: waves per SIMD the register budget is sized for. 4 (default) = two 8-wave blocks per CU
// within 128 VGPRs (some variants spill a few registers to scratch); 2 = one block per CU with up
// to 256 VGPRs and no spills (the persistent grid shrinks to one block per CU; the host picks it).
template <int BM, int BN, int WM, int WN, int PRO, bool STATS, bool STRIDED, bool BT = false, bool EPI = false,
          int OCC = 4>
__global__ __launch_bounds__(64 * WM * WN, OCC) void conv1x1_gemm_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, int64_t M, int N,
    int K, RowMap rm, const float* __restrict__ pro_ss, float* __restrict__ part, int mtiles, int ntiles,
    int groups, const uint16_t* __restrict__ X2, EpiBN epi, ProOut po) {
  static_assert(PRO < 4 || (!STRIDED && !BT && !EPI), "the block-output prologue is a stride-1 forward");
  constexpr int NT = 64 * WM * WN, RSTEP = NT / 8;  // threads; rows staged per pass (8 chunks per row)
  constexpr int AR = BM / RSTEP, BR = BN / RSTEP;    // 16-B loads per thread per operand tile
  constexpr int WTM = BM / WM, WTN = BN / WN;        // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;        // 16x16 MFMA tiles per wave
  constexpr int SBT = BN * 2 + 32;                   // BT: LDS row stride of the [64 k][BN n] B tile
  constexpr int ABYTES = BM * 128, BBYTES = BT ? 64 * SBT : BN * 128, BUF = ABYTES + BBYTES;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int wg = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int nt = wg % ntiles, g = wg / ntiles;
  if (g >= groups) return;
  const int n0 = nt * BN;
  const int lc = tid & 7, lr = tid >> 3;  // staging: 16-B chunk (8 k) and first row of this thread
  const int nk = K / kBK;

  // The C-tile readout: each thread stores a fixed 8-channel chunk column (cc) of the tiles it
  // visits (EPI: and keeps that column's BN-backward sums). Statistics (STATS) are shifted sums,
  // the shift a sample of the same channel (the block's first stored row: no cancellation when
  // |mean| >> std), so partials across tiles simply add; threads merge once, at the end.
  constexpr int CPR = BN / 8;                         // 16-B chunks per C-tile row
  static_assert(NT % CPR == 0, "readout mapping needs a fixed chunk column per thread");
  const int cc = tid % CPR;
  float st_s[8], st_ss[8];  // EPI: this thread's 8 channels' BN-backward sums
#pragma unroll
  for (int e = 0; e < 8; ++e) st_s[e] = st_ss[e] = 0.f;
  // STATS: a second pass over the stored C tile in LDS, thread = one channel pair (sp) of rows
  // tid / SPR + SRS·i — 6 registers of state instead of 21 (the 8-channel form spilled at
  // occupancy 4), shifted by the pair's first stored values (row 0 of the block's first tile).
  constexpr int SPR = BN / 2, SRS = NT / SPR;
  static_assert(SPR <= 64 && 64 % SPR == 0 && BM % SRS == 0, "stats pass mapping");
  const int sp = tid % SPR;
  float sn = 0.f, sk[2] = {0.f, 0.f}, ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};

  const uint16_t* wrow[BR];
  constexpr int BCH = BN / 8;  // BT: 16-B chunks per staged k row (64 * BCH == NT * BR)
  static_assert(!BT || 64 * BCH == NT * BR, "BT staging must cover the B tile exactly");
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    if (BT) {
      const int q = tid + NT * i, row = q / BCH, c = q % BCH;
      wrow[i] = Wt + (int64_t)row * N + n0 + c * 8;  // + kt * 64 * N per K-tile
    } else {
      wrow[i] = Wt + (int64_t)(n0 + lr + RSTEP * i) * K + lc * 8;
    }
  }

  u32x4 sa[AR], sb[BR], sa2[PRO >= 2 ? AR : 1];
  // PRO: the per-input-channel coefficients for all K channels, staged once into LDS after the
  // two operand buffers (kept out of the VGPRs that the MFMA phase needs)
  float* pro_lds = reinterpret_cast<float*>(smem + 2 * BUF);
  // EPI mask-recompute form: this N tile's (scale, shift) of the masked BN, after the coefficients
  constexpr int NCOEF = PRO == 3 ? 5 : PRO == 2 ? 3 : PRO == 5 ? 4 : PRO ? 2 : 0;
  float* epi_ss_lds = pro_lds + NCOEF * K;
  // EPI: and this N tile's mean of the previous BN (the shift of the st_ss products; LDS, not VGPRs)
  float* epi_mu_lds = epi_ss_lds + 2 * BN;
  if (EPI && epi.ss) {
    for (int i = tid; i < 2 * BN; i += NT) epi_ss_lds[i] = epi.ss[(i >= BN ? N - BN : 0) + n0 + i];
  }
  if (EPI) {
    for (int i = tid; i < BN; i += NT) epi_mu_lds[i] = epi.mean[n0 + i];
  }
  if (PRO) {
    for (int i = tid; i < (PRO == 5 ? 2 : NCOEF) * K; i += NT) pro_lds[i] = pro_ss[i];
    if (PRO == 5)
      for (int i = tid; i < 2 * K; i += NT) pro_lds[2 * K + i] = po.rss[i];
  }
  if (PRO || EPI) lds_barrier();
  // side output of the staged operand (uniform per block: N-tile 0 writes it, once per element)
  const bool side = (PRO == 1 || PRO >= 4) && po.out != nullptr && nt == 0;
  if ((PRO == 1 || PRO >= 4) && wg == 0 && tid == 0) {
    if (po.nbt1) po.nbt1[0] += 1;
    if (po.nbt2) po.nbt2[0] += 1;
  }
  const uint16_t* arow[AR];
  const int64_t dx2 = PRO >= 2 ? X2 - X : 0;  // the second A source at the same element offsets
  // Rows past M load row M-1 (clamped, branch-free: a per-row "load or zero" select makes hipcc
  // branch around every load); their outputs are neither stored nor counted in the statistics.
  auto set_rows = [&](int mt) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = (int)min<int64_t>((int64_t)mt * BM + lr + RSTEP * i, M - 1);
      arow[i] = X + rm.in_row<STRIDED>(m) * K + lc * 8;
    }
  };
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < AR; ++i) sa[i] = *reinterpret_cast<const u32x4*>(arow[i] + kt * kBK);
    if (PRO >= 2) {
#pragma unroll
      for (int i = 0; i < AR; ++i) sa2[i] = *reinterpret_cast<const u32x4*>(arow[i] + dx2 + kt * kBK);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      sb[i] = *reinterpret_cast<const u32x4*>(wrow[i] + (BT ? (int64_t)kt * kBK * N : (int64_t)kt * kBK));
  };
  auto store = [&](int buf, int kt) {
    uint8_t* A = smem + buf * BUF;
    uint8_t* B = A + ABYTES;
    if (PRO == 2 || PRO == 3) {  // BN backward on this thread's 8 channels: a·g + b·x + c (g masked by ReLU for 3)
      // coefficients two channels at a time (float2 LDS reads): few live VGPRs in this phase
      const int k0 = kt * kBK + lc * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 ca = *reinterpret_cast<const float2*>(pro_lds + k0 + 2 * q);
        const float2 cb = *reinterpret_cast<const float2*>(pro_lds + K + k0 + 2 * q);
        const float2 cc = *reinterpret_cast<const float2*>(pro_lds + 2 * K + k0 + 2 * q);
        float2 ms = {0.f, 0.f}, mt = {0.f, 0.f};
        if (PRO == 3) {
          ms = *reinterpret_cast<const float2*>(pro_lds + 3 * K + k0 + 2 * q);
          mt = *reinterpret_cast<const float2*>(pro_lds + 4 * K + k0 + 2 * q);
        }
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          float g0 = __uint_as_float(sa[i][q] << 16), g1 = __uint_as_float(sa[i][q] & 0xffff0000u);
          const float x0 = __uint_as_float(sa2[i][q] << 16), x1 = __uint_as_float(sa2[i][q] & 0xffff0000u);
          if (PRO == 3) {
            g0 = fmaf(x0, ms.x, mt.x) > 0.f ? g0 : 0.f;
            g1 = fmaf(x1, ms.y, mt.y) > 0.f ? g1 : 0.f;
          }
          sa[i][q] = dev::pack_bf16x2(fmaf(ca.x, g0, fmaf(cb.x, x0, cc.x)), fmaf(ca.y, g1, fmaf(cb.y, x1, cc.y)));
        }
      }
    }
    if (PRO == 1) {  // previous BN's apply + ReLU on this thread's 8 input channels
      const int k0 = kt * kBK + lc * 8;
      float sc[8], sh[8];
      dev::Vec8<float>::ld(pro_lds + k0, sc);
      dev::Vec8<float>::ld(pro_lds + K + k0, sh);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = fmaxf(fmaf(__uint_as_float(sa[i][q] << 16), sc[2 * q], sh[2 * q]), 0.f);
          const float hi = fmaxf(fmaf(__uint_as_float(sa[i][q] & 0xffff0000u), sc[2 * q + 1], sh[2 * q + 1]), 0.f);
          sa[i][q] = dev::pack_bf16x2(lo, hi);
        }
      }
    }
    uint32_t mbits[PRO >= 4 ? AR : 1];
    if (PRO >= 4) {  // block output: relu(y·s + t + r) on this thread's 8 channels, plus its mask bits
      const int k0 = kt * kBK + lc * 8;
#pragma unroll
      for (int i = 0; i < AR; ++i) mbits[i] = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 sc = *reinterpret_cast<const float2*>(pro_lds + k0 + 2 * q);
        const float2 sh = *reinterpret_cast<const float2*>(pro_lds + K + k0 + 2 * q);
        float2 rs = {1.f, 1.f}, rh = {0.f, 0.f};
        if (PRO == 5) {
          rs = *reinterpret_cast<const float2*>(pro_lds + 2 * K + k0 + 2 * q);
          rh = *reinterpret_cast<const float2*>(pro_lds + 3 * K + k0 + 2 * q);
        }
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          float r0 = __uint_as_float(sa2[i][q] << 16), r1 = __uint_as_float(sa2[i][q] & 0xffff0000u);
          if (PRO == 5) {  // the downsample's BN apply, at storage precision (bn_apply_kernel's rss)
            r0 = bf16_round(fmaf(r0, rs.x, rh.x));
            r1 = bf16_round(fmaf(r1, rs.y, rh.y));
          }
          const float o0 = fmaf(__uint_as_float(sa[i][q] << 16), sc.x, sh.x) + r0;
          const float o1 = fmaf(__uint_as_float(sa[i][q] & 0xffff0000u), sc.y, sh.y) + r1;
          mbits[i] |= ((o0 > 0.f ? 1u : 0u) | (o1 > 0.f ? 2u : 0u)) << (2 * q);
          sa[i][q] = dev::pack_bf16x2(fmaxf(o0, 0.f), fmaxf(o1, 0.f));
        }
      }
    }
    if (side) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int64_t e = (arow[i] - X) + (int64_t)kt * kBK;  // element offset of this 8-channel chunk
        *reinterpret_cast<u32x4*>(po.out + e) = sa[i];
        if (PRO >= 4 && po.bits) po.bits[e >> 3] = (uint8_t)mbits[PRO >= 4 ? i : 0];
      }
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) *reinterpret_cast<u32x4*>(A + swz(lr + RSTEP * i, lc)) = sa[i];
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      if (BT) {
        const int q = tid + NT * i, row = q / BCH, c = q % BCH;
        *reinterpret_cast<u32x4*>(B + row * SBT + c * 16) = sb[i];
      } else {
        *reinterpret_cast<u32x4*>(B + swz(lr + RSTEP * i, lc)) = sb[i];
      }
    }
  };

  set_rows(g);
  load(0);
  for (int mt = g; mt < mtiles; mt += groups) {
    const int64_t m0 = (int64_t)mt * BM;
    const int next = mt + groups;
    const int rows_valid = (int)min<int64_t>(BM, M - m0);
    // EPI: every readout row's y / add / mask loads are issued at the start of the tile, so they
    // are in flight during the K loop (rows past M clamped, not used)
    constexpr int RIT = BM * CPR / NT;  // readout rows per thread
    static_assert(BM * CPR % NT == 0, "readout rows must divide evenly over the threads");
    u32x4 e_y[EPI ? RIT : 1], e_ad[EPI ? RIT : 1];
    uint32_t e_mb[EPI ? RIT : 1];
    if (EPI) {
      const bool form1 = epi.bits != nullptr;  // uniform per launch
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        const int row = min((tid + NT * it) / CPR, rows_valid - 1);
        const int64_t e0 = (m0 + row) * N + n0 + cc * 8;
        e_y[it] = *reinterpret_cast<const u32x4*>(epi.y + e0);
        if (form1) {
          int64_t ea = e0;
          bool have = true;
          if (epi.add_w) {  // compact stride-2 addend: pixel (b, h, w) -> (b, h/2, w/2) when h, w even
            const int hw = epi.add_h * epi.add_w;
            const int64_t m = m0 + row;
            const int64_t b = m / hw;
            const int r = (int)(m - b * hw), h = r / epi.add_w, w = r - h * epi.add_w;
            have = ((h | w) & 1) == 0;
            const int ah = (epi.add_h + 1) >> 1, aw = (epi.add_w + 1) >> 1;
            ea = have ? ((b * ah + (h >> 1)) * aw + (w >> 1)) * N + n0 + cc * 8 : 0;
          }
          const u32x4 av = *reinterpret_cast<const u32x4*>(epi.add + ea);
          e_ad[it] = have ? av : u32x4{0, 0, 0, 0};
          e_mb[it] = epi.bits[e0 >> 3];
        } else {
          e_ad[it] = u32x4{0, 0, 0, 0};
          e_mb[it] = 0u;
        }
      }
    }
    store(0, 0);
    lds_barrier();

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      // issue the next K-tile's loads — or, on the last K-tile, the NEXT M-tile's first loads,
      // so they are in flight during these MFMAs and the whole epilogue below
      if (kt + 1 < nk) {
        load(kt + 1);
      } else if (next < mtiles) {
        set_rows(next);
        load(0);
      }
      const uint8_t* A = smem + cur * BUF;
      const uint8_t* B = A + ABYTES;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = s * 4 + (lane >> 4);
        bf16x8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(A + swz(wm * WTM + i * 16 + (lane & 15), ch));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (BT) {  // k rows s*32 + 8*(lane>>4) + 0..3 and + 4..7 of column n, via transposed reads
            const int r0 = s * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
            const int col = wn * WTN + j * 16 + 4 * (lane & 3);
            const v4s v8[2] = {lds_tr16(B + r0 * SBT + col * 2), lds_tr16(B + (r0 + 4) * SBT + col * 2)};
            b[j] = __builtin_bit_cast(bf16x8, v8);
          } else {
            b[j] = *reinterpret_cast<const bf16x8*>(B + swz(wn * WTN + j * 16 + (lane & 15), ch));
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nk) store(cur ^ 1, kt + 1);
      lds_barrier();
    }

    // ---- epilogue: round to bf16 (the stored values are what BN normalizes) ----
    // ---- store Y through LDS: C tile [BM][BN] bf16, rows padded 16 B, then 16-B global stores ----
    // The MFMA computes the transposed tile (W rows as the first operand), so a lane's 4
    // accumulator values are 4 consecutive channels of one pixel row: one 8-B LDS store each
    // instead of four 2-B stores.
    constexpr int CST = BN * 2 + 16;
    uint8_t* Cs = smem;  // the K loop ended with a barrier: the operand buffers are free
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wm * WTM + i * 16 + (lane & 15);
        const int col = wn * WTN + j * 16 + (lane >> 4) * 4;
        uint2 pk;  // one v_cvt_pk_bf16_f32 (RNE) per channel pair
        pk.x = dev::pack_bf16x2(acc[i][j][0], acc[i][j][1]);
        pk.y = dev::pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(Cs + row * CST + col * 2) = pk;
      }
    lds_barrier();
    if (STATS) {
      if (mt == g) {  // row 0: always valid
        const uint32_t k = *reinterpret_cast<const uint32_t*>(Cs + sp * 4);
        sk[0] = __uint_as_float(k << 16);
        sk[1] = __uint_as_float(k & 0xffff0000u);
      }
      // full tiles: every row's LDS read issued before the first use, from one base address plus
      // immediate offsets (a read-then-use per row inside `if (row < rows_valid)` compiled to 16
      // serialized ds_read + s_waitcnt lgkmcnt(0) round trips per tile); the partial last tile
      // keeps the per-row form
      constexpr int NSR = BM / SRS;
      const uint8_t* sbase = Cs + (tid / SPR) * CST + sp * 4;
      auto add_stat = [&](uint32_t v) {
        const float d0 = __uint_as_float(v << 16) - sk[0], d1 = __uint_as_float(v & 0xffff0000u) - sk[1];
        sn += 1.f;
        ssum[0] += d0;
        ssum[1] += d1;
        ssq[0] = fmaf(d0, d0, ssq[0]);
        ssq[1] = fmaf(d1, d1, ssq[1]);
      };
      if (rows_valid == BM) {
        uint32_t sv[NSR];
#pragma unroll
        for (int i = 0; i < NSR; ++i) sv[i] = *reinterpret_cast<const uint32_t*>(sbase + SRS * i * CST);
#pragma unroll
        for (int i = 0; i < NSR; ++i) add_stat(sv[i]);
      } else {
#pragma unroll
        for (int i = 0; i < NSR; ++i)
          if (tid / SPR + SRS * i < rows_valid) add_stat(*reinterpret_cast<const uint32_t*>(sbase + SRS * i * CST));
      }
    }
    if constexpr (EPI) {
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        const int row = (tid + NT * it) / CPR;
        if (row < rows_valid) {
          u32x4 v = *reinterpret_cast<const u32x4*>(Cs + row * CST + cc * 16);
          const u32x4 yv = e_y[EPI ? it : 0], ad = e_ad[EPI ? it : 0];
          const uint32_t mb = e_mb[EPI ? it : 0];
          const bool form1 = epi.bits != nullptr;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            float g0 = __uint_as_float(v[h] << 16) + __uint_as_float(ad[h] << 16);
            float g1 = __uint_as_float(v[h] & 0xffff0000u) + __uint_as_float(ad[h] & 0xffff0000u);
            if (form1) {
              g0 = ((mb >> (2 * h)) & 1u) ? g0 : 0.f;
              g1 = ((mb >> (2 * h + 1)) & 1u) ? g1 : 0.f;
            } else {
              const float2 sc = *reinterpret_cast<const float2*>(epi_ss_lds + cc * 8 + 2 * h);
              const float2 sh = *reinterpret_cast<const float2*>(epi_ss_lds + BN + cc * 8 + 2 * h);
              g0 = fmaf(__uint_as_float(yv[h] << 16), sc.x, sh.x) > 0.f ? g0 : 0.f;
              g1 = fmaf(__uint_as_float(yv[h] & 0xffff0000u), sc.y, sh.y) > 0.f ? g1 : 0.f;
            }
            v[h] = dev::pack_bf16x2(g0, g1);
            g0 = __uint_as_float(v[h] << 16);  // the sums see g at storage precision
            g1 = __uint_as_float(v[h] & 0xffff0000u);
            st_s[2 * h] += g0;
            st_s[2 * h + 1] += g1;
            const float2 mu = *reinterpret_cast<const float2*>(epi_mu_lds + cc * 8 + 2 * h);
            st_ss[2 * h] = fmaf(g0, __uint_as_float(yv[h] << 16) - mu.x, st_ss[2 * h]);
            st_ss[2 * h + 1] = fmaf(g1, __uint_as_float(yv[h] & 0xffff0000u) - mu.y, st_ss[2 * h + 1]);
          }
          if (NTSTORE) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(Y + (m0 + row) * N + n0 + cc * 8));
          else *reinterpret_cast<u32x4*>(Y + (m0 + row) * N + n0 + cc * 8) = v;
        }
      }
    } else {
      // readout of full tiles: every row's LDS read issued before the first store (thread row
      // tid / CPR + (NT / CPR)·it, chunk cc) in the statistics instances; the partial last tile and the
      // other instances keep the per-row form (their batch spilled VGPRs: the BN-backward prologue
      // forms, and the EPI instances with their epilogue operands live)
      constexpr int RSTR = NT / CPR;
      auto st_row = [&](int row, const u32x4& v) {
        if (NTSTORE) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(Y + (m0 + row) * N + n0 + cc * 8));
        else *reinterpret_cast<u32x4*>(Y + (m0 + row) * N + n0 + cc * 8) = v;
      };
      if (STATS && rows_valid == BM) {
        u32x4 rv[RIT];
#pragma unroll
        for (int it = 0; it < RIT; ++it) rv[it] = *reinterpret_cast<const u32x4*>(Cs + (tid / CPR + RSTR * it) * CST + cc * 16);
#pragma unroll
        for (int it = 0; it < RIT; ++it) st_row(tid / CPR + RSTR * it, rv[it]);
      } else {
#pragma unroll
        for (int it = 0; it < RIT; ++it) {
          const int row = (tid + NT * it) / CPR;
          if (row < rows_valid) st_row(row, *reinterpret_cast<const u32x4*>(Cs + row * CST + cc * 16));
        }
      }
    }
    lds_barrier();  // Cs aliases the operand buffers the next tile stores into
  }

  if (EPI) {
    // plain sums: add over the lanes sharing cc, then over the waves through LDS
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        st_s[e] += __shfl_xor(st_s[e], o, 64);
        st_ss[e] += __shfl_xor(st_ss[e], o, 64);
      }
    }
    constexpr int NW = NT / 64;
    float* red = reinterpret_cast<float*>(smem);  // [NW][BN][2]
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wid * BN + cc * 8 + e) * 2 + 0] = st_s[e];
        red[(wid * BN + cc * 8 + e) * 2 + 1] = st_ss[e];
      }
    }
    lds_barrier();
    for (int c = tid; c < BN; c += NT) {
      float sd = 0.f, sdx = 0.f;
      for (int w = 0; w < NW; ++w) {
        sd += red[(w * BN + c) * 2 + 0];
        sdx += red[(w * BN + c) * 2 + 1];
      }
      epi.part[((int64_t)g * N + n0 + c) * 2 + 0] = sd;
      epi.part[((int64_t)g * N + n0 + c) * 2 + 1] = sdx;
    }
    return;
  }

  if (STATS) {
    // per thread (n, mean, M2) of its channel pair, Chan-merged over the lanes sharing sp (xor over
    // the lane bits above log2(SPR)), then over the waves through LDS
    float mean[2], m2[2], n = sn;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      mean[e] = n > 0.f ? sk[e] + ssum[e] / n : 0.f;
      m2[e] = n > 0.f ? fmaxf(ssq[e] - ssum[e] * ssum[e] / n, 0.f) : 0.f;
    }
#pragma unroll
    for (int o = SPR; o < 64; o <<= 1) {
      const float nb = __shfl_xor(n, o, 64), nn = n + nb;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float mb = __shfl_xor(mean[e], o, 64), m2b = __shfl_xor(m2[e], o, 64);
        if (nn > 0.f) {
          const float d = mb - mean[e];
          mean[e] += d * (nb / nn);
          m2[e] += m2b + d * d * (n * nb / nn);
        }
      }
      n = nn;
    }
    constexpr int NW = NT / 64;
    float* red = reinterpret_cast<float*>(smem);  // [NW][3][BN]
    if (lane < SPR) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        red[(wid * 3 + 0) * BN + sp * 2 + e] = n;
        red[(wid * 3 + 1) * BN + sp * 2 + e] = mean[e];
        red[(wid * 3 + 2) * BN + sp * 2 + e] = m2[e];
      }
    }
    lds_barrier();
    for (int c = tid; c < BN; c += NT) {
      float tn = 0.f, tm = 0.f, t2 = 0.f;
      for (int w = 0; w < NW; ++w) {
        const float nb = red[(w * 3 + 0) * BN + c], nn = tn + nb;
        if (nb > 0.f) {
          const float d = red[(w * 3 + 1) * BN + c] - tm;
          tm += d * (nb / nn);
          t2 += red[(w * 3 + 2) * BN + c] + d * d * (tn * nb / nn);
        }
        tn = nn;
      }
      part[((int64_t)g * 3 + 0) * N + n0 + c] = tn;
      part[((int64_t)g * 3 + 1) * N + n0 + c] = tm;
      part[((int64_t)g * 3 + 2) * N + n0 + c] = t2;
    }
  }
}

// Per channel: merge the groups' (count, mean, M2), then the BN coefficients and the running-stat
// update (same outputs as the stats finalize of batch_norm.hip). One 256-thread block per
// channel: threads stride over the groups (element (g, q, c) at g*gs + q*ks + c*cs, so both the
// [groups][3][C] and the group-minor [3][C][groups] layouts are read). The merge is the shifted
// form of Chan's: with K = group 0's mean (a sample of this channel's mean, so |mean_g - K| is
// O(std) and nothing cancels), sum n_g, n_g·(mean_g - K) and M2_g + n_g·(mean_g - K)^2 — plain
// adds, no division per group, so a thread's loads are independent and issue together (the
// divide-per-merge chain made this launch latency-bound: 6-12 us at 64-3136 groups).
template <typename W>
__global__ __launch_bounds__(256) void bn_partial_finalize_kernel(
    const float* __restrict__ part, int groups, int C, int64_t gs, int64_t ks, int64_t cs, int64_t M,
    const W* __restrict__ weight, const W* __restrict__ bias, W* running_mean, W* running_var, const int64_t* nbt,
    float momentum, bool cma, float eps, float* __restrict__ mean_out, float* __restrict__ invstd_out,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float red[3][4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* pc = part + (int64_t)c * cs;
  const float K = pc[ks];  // group 0's mean (group 0 always holds rows)
  // thread 0's per-channel parameters load up front, under the partials (latency-bound launch)
  float gm = 1.f, bb = 0.f, rm = 0.f, rv = 0.f, mom = momentum;
  if (tid == 0) {
    if (weight) gm = dev::Elem<W, float>::ld(weight, c);
    if (bias) bb = dev::Elem<W, float>::ld(bias, c);
    if (running_mean) {
      rm = dev::Elem<W, float>::ld(running_mean, c);
      rv = dev::Elem<W, float>::ld(running_var, c);
      if (cma && nbt) mom = 1.f / (float)(nbt[0] + 1);
    }
  }
  float n = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int gi = tid; gi < groups; gi += 256) {
    const float* q = pc + (int64_t)gi * gs;
    const float nb = q[0], d = q[ks] - K, m2b = q[2 * ks];
    n += nb;
    s1 = fmaf(nb, d, s1);
    s2 += fmaf(nb * d, d, m2b);
  }
  n = dev::wave_sum(n);
  s1 = dev::wave_sum(s1);
  s2 = dev::wave_sum(s2);
  if (lane == 0) {
    red[0][wid] = n;
    red[1][wid] = s1;
    red[2][wid] = s2;
  }
  __syncthreads();
  if (tid != 0) return;
  n = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  s1 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  s2 = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
  const float dm = n > 0.f ? s1 / n : 0.f;
  const float mean = K + dm;
  const float m2 = fmaxf(s2 - s1 * dm, 0.f);
  const float Mf = M > 0 ? (float)M : n;  // M <= 0: the partials' own counts (uneven SyncBN shards)
  const float var = Mf > 0.f ? fmaxf(m2 / Mf, 0.f) : 0.f;
  const float inv = rsqrtf(var + eps);
  mean_out[c] = mean;
  invstd_out[c] = inv;
  scale[c] = gm * inv;
  shift[c] = bb - mean * gm * inv;
  if (running_mean) {
    const float unbiased = Mf > 1.f ? var * Mf / (Mf - 1.f) : var;
    dev::Elem<W, float>::st(running_mean, c, (1.f - mom) * rm + mom * mean);
    dev::Elem<W, float>::st(running_var, c, (1.f - mom) * rv + mom * unbiased);
  }
}


// ---------------------------------------------------------------------------------------------
// Weight gradient of the 1x1 conv: dW[N, K] = sum_m dY[m, n] · X[m, k]  (a "TN" GEMM whose
// reduction runs over the M = batch·OH·OW pixel rows). Both operands are staged row-major
// ([64 pixel rows][n or k], as they lie in HBM) and read into MFMA fragments with gfx950's
// transposing LDS read ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, each lane
// receiving one column), so no register or LDS transposition pass is needed. The reduction is
// split over M across blocks (fp32 slabs), then one small kernel sums the slabs into dW.
// LDS rows are padded by 32 B so the 4 rows of a transposed read fall on distinct banks.

// PRO (2, 3): dY = a_n·G + b_n·Y2 + c_n is formed while staging (the BatchNorm-backward
// elementwise pass folded in; G is the masked upstream gradient, Y2 the BN input; with 3 the ReLU
// mask (Y2·s_n + t_n > 0) is applied to G here).
template <int TN, int TK, bool STRIDED, int PRO>
__global__ __launch_bounds__(256, 2) void conv1x1_wgrad_kernel(const uint16_t* __restrict__ dY,
                                                                const uint16_t* __restrict__ X,
                                                                float* __restrict__ ws, int M, int N, int K,
                                                                RowMap rm, int ntiles, int ktiles, int mchunk,
                                                                const uint16_t* __restrict__ Y2,
                                                                const float* __restrict__ coef) {
  constexpr int BM = 64;                       // pixel rows per step (two 32-deep MFMA k-steps)
  constexpr int SA = TN * 2 + 32, SB = TK * 2 + 32;
  constexpr int ABYTES = BM * SA, BUF = ABYTES + BM * SB;
  constexpr int CA = TN / 8, CB = TK / 8;      // 16-B chunks per staged row
  constexpr int LA = BM * CA / 256, LB = BM * CB / 256;
  constexpr int WTN = TN / 2, WTK = TK / 2, FN = WTN / 16, FK = WTK / 16;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wn = wid >> 1, wk = wid & 1;
  const int tiles = ntiles * ktiles;
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int sidx = bid / tiles, tile = bid % tiles;  // neighbours share the pixel range (L2 reuse)
  const int n0 = (tile % ntiles) * TN, k0 = (tile / ntiles) * TK;
  const int m_begin = sidx * mchunk, m_end = min(M, m_begin + mchunk);

  // Two register slots: the loads of step m + 2·BM go out while step m computes, so each load has
  // two steps of MFMAs (not one) to land. Loads are unconditional (rows clamped to M - 1, always
  // valid memory) and the rows past the range are zeroed when a slot is stored: a conditional
  // load or a select right after it would make the compiler wait for every load in flight.
  u32x4 sa[2][LA], sb[2][LB], sa2[2][PRO ? LA : 1];
  float pa[8], pb[8], pc[8], pms[8], pmt[8];  // this thread's 8 dY channels (fixed: 256 % CA == 0)
  if (PRO) {
    const int c = tid % CA;
    dev::Vec8<float>::ld(coef + n0 + c * 8, pa);
    dev::Vec8<float>::ld(coef + N + n0 + c * 8, pb);
    dev::Vec8<float>::ld(coef + 2 * N + n0 + c * 8, pc);
    if (PRO == 3) {
      dev::Vec8<float>::ld(coef + 3 * N + n0 + c * 8, pms);
      dev::Vec8<float>::ld(coef + 4 * N + n0 + c * 8, pmt);
    }
  }
  auto load = [&](int slot, int m) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + 256 * i, row = q / CA, c = q - (q / CA) * CA;
      const int64_t off = (int64_t)min(m + row, M - 1) * N + n0 + c * 8;
      sa[slot][i] = *reinterpret_cast<const u32x4*>(dY + off);
      if (PRO) sa2[slot][i] = *reinterpret_cast<const u32x4*>(Y2 + off);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + 256 * i, row = q / CB, c = q - (q / CB) * CB;
      sb[slot][i] = *reinterpret_cast<const u32x4*>(X + rm.in_row<STRIDED>(min(m + row, M - 1)) * K + k0 + c * 8);
    }
  };
  auto store = [&](int buf, int slot, int m) {
    uint8_t* A = smem + buf * BUF;
    uint8_t* B = A + ABYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + 256 * i, row = q / CA, c = q - (q / CA) * CA;
      u32x4 t = sa[slot][i];
      if (PRO) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          float g0 = __uint_as_float(sa[slot][i][h] << 16), g1 = __uint_as_float(sa[slot][i][h] & 0xffff0000u);
          const float x0 = __uint_as_float(sa2[slot][i][h] << 16), x1 = __uint_as_float(sa2[slot][i][h] & 0xffff0000u);
          if (PRO == 3) {
            g0 = fmaf(x0, pms[2 * h], pmt[2 * h]) > 0.f ? g0 : 0.f;
            g1 = fmaf(x1, pms[2 * h + 1], pmt[2 * h + 1]) > 0.f ? g1 : 0.f;
          }
          t[h] = dev::pack_bf16x2(fmaf(pa[2 * h], g0, fmaf(pb[2 * h], x0, pc[2 * h])),
                                  fmaf(pa[2 * h + 1], g1, fmaf(pb[2 * h + 1], x1, pc[2 * h + 1])));
        }
      }
      *reinterpret_cast<u32x4*>(A + row * SA + c * 16) = m + row < m_end ? t : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + 256 * i, row = q / CB, c = q - (q / CB) * CB;
      *reinterpret_cast<u32x4*>(B + row * SB + c * 16) = m + row < m_end ? sb[slot][i] : u32x4{0, 0, 0, 0};
    }
  };

  f32x4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addressing: lane (4q + p) of its 16-lane group addresses row q, columns 4p..4p+3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto compute = [&](int cur) {
    const uint8_t* A = smem + cur * BUF;
    const uint8_t* B = A + ABYTES;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r0 = s2 * 32 + 8 * g + q4;
      bf16x8 a[FN], b[FK];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int col = wn * WTN + i * 16 + 4 * p4;
        const v4s lo = lds_tr16(A + r0 * SA + col * 2), hi = lds_tr16(A + (r0 + 4) * SA + col * 2);
        const v4s v8[2] = {lo, hi};
        a[i] = __builtin_bit_cast(bf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < FK; ++j) {
        const int col = wk * WTK + j * 16 + 4 * p4;
        const v4s lo = lds_tr16(B + r0 * SB + col * 2), hi = lds_tr16(B + (r0 + 4) * SB + col * 2);
        const v4s v8[2] = {lo, hi};
        b[j] = __builtin_bit_cast(bf16x8, v8);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  if (m_begin < m_end) {
    // step pairs (slot 0 = even steps, LDS buffer 0; slot 1 = odd steps, buffer 1), branch-free
    // loads; the steps past m_end of the last pair compute on zero rows (stored zeroed)
    load(0, m_begin);
    load(1, m_begin + BM);
    store(0, 0, m_begin);
    lds_barrier();
    for (int m = m_begin; m < m_end; m += 2 * BM) {
      load(0, m + 2 * BM);  // (clamped rows: always valid memory)
      compute(0);
      store(1, 1, m + BM);
      lds_barrier();
      if (m + BM >= m_end) break;  // (uniform) an odd step count: the last odd step is empty
      load(1, m + 3 * BM);
      compute(1);
      store(0, 0, m + 2 * BM);
      lds_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing prefetch loads retire here
  }
  // fp32 slab of this pixel range: ws[sidx][n][k]; lane holds rows n = (lane>>4)*4 + r, col k = lane&15
  float* out = ws + (int64_t)sidx * N * K;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * WTN + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wk * WTK + j * 16 + (lane & 15);
        out[(int64_t)n * K + k] = acc[i][j][r];
      }
}

// Fused backward of a stride-1 1x1 conv whose output gradient dY = k1·G + k2·Y2 + k3 is formed
// while staging (the BN backward folded in, PRO 2 / 3 as above): the input gradient dX = dY·W
// and the weight gradient dW = dYᵀ·X computed from ONE staging of the dY tile. The separate
// dgrad GEMM and wgrad kernel each read G and Y2 (the two largest tensors of the layer): at
// ResNet-50 layer-1 shapes (M = 802816, N·K = 256·64) both sit at the HBM roofline, so sharing
// the read removes a third of the layer's backward traffic.
// One block per CU walks a contiguous pixel range in 64-row steps (two LDS buffers, next step's
// loads in flight): wgrad as conv1x1_wgrad_kernel with the whole N x K as one tile (fp32 slab
// per block, summed by wgrad_reduce_kernel); dgrad on the same step, swapped (dXᵀ = Wᵀ·dYᵀ:
// A = Wᵀ by transposed reads of W [N][K] kept in LDS, B = dY rows), so a lane ends with 4
// consecutive input channels of one pixel — one 8-B store.
template <int N, int K, int PRO>
__global__ __launch_bounds__(256, 1) void conv1x1_bwd_fused_kernel(
    const uint16_t* __restrict__ G, const uint16_t* __restrict__ Y2, const float* __restrict__ coef,
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wg, uint16_t* __restrict__ dX, float* __restrict__ ws,
    int M, int mchunk) {
  constexpr int BM = 64;
  constexpr int SA = N * 2 + 32, SB = K * 2 + 32, SW = K * 2 + 32;
  constexpr int ABYTES = BM * SA, BUF = ABYTES + BM * SB;
  constexpr int CA = N / 8, CB = K / 8;
  constexpr int LA = BM * CA / 256, LB = BM * CB / 256;
  constexpr int WTN = N / 2, WTK = K / 2, FN = WTN / 16, FK = WTK / 16;  // wgrad wave tile (2 x 2 waves)
  constexpr int KW = K / 4, KF = KW / 16;                                // dgrad: k rows per wave
  static_assert(256 % CA == 0 && LA >= 1 && LB >= 1 && KF >= 1, "fused 1x1 backward tile");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* Wl = smem + 2 * BUF;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wn = wid >> 1, wk = wid & 1;
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int m_begin = bid * mchunk, m_end = min(M, m_begin + mchunk);

  // W [N][K] -> LDS rows (padded for the transposed reads)
  for (int q = tid; q < N * CB; q += 256) {
    const int n = q / CB, c = q % CB;
    *reinterpret_cast<u32x4*>(Wl + n * SW + c * 16) = *reinterpret_cast<const u32x4*>(Wg + (int64_t)n * K + c * 8);
  }
  float pa[8], pb[8], pc[8], pms[8], pmt[8];  // this thread's 8 dY channels (fixed: 256 % CA == 0)
  {
    const int c = tid % CA;
    dev::Vec8<float>::ld(coef + c * 8, pa);
    dev::Vec8<float>::ld(coef + N + c * 8, pb);
    dev::Vec8<float>::ld(coef + 2 * N + c * 8, pc);
    if (PRO == 3) {
      dev::Vec8<float>::ld(coef + 3 * N + c * 8, pms);
      dev::Vec8<float>::ld(coef + 4 * N + c * 8, pmt);
    }
  }
  u32x4 sa[LA], sa2[LA], sb[LB];
  auto load = [&](int m) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + 256 * i, row = q / CA, c = q - (q / CA) * CA;
      const int64_t off = (int64_t)min(m + row, M - 1) * N + c * 8;
      sa[i] = *reinterpret_cast<const u32x4*>(G + off);
      sa2[i] = *reinterpret_cast<const u32x4*>(Y2 + off);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + 256 * i, row = q / CB, c = q - (q / CB) * CB;
      const u32x4 v = *reinterpret_cast<const u32x4*>(X + (int64_t)min(m + row, M - 1) * K + c * 8);
      sb[i] = m + row < m_end ? v : u32x4{0, 0, 0, 0};
    }
  };
  auto store = [&](int buf, int m) {
    uint8_t* A = smem + buf * BUF;
    uint8_t* B = A + ABYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + 256 * i, row = q / CA, c = q - (q / CA) * CA;
      u32x4 t;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        float g0 = __uint_as_float(sa[i][h] << 16), g1 = __uint_as_float(sa[i][h] & 0xffff0000u);
        const float x0 = __uint_as_float(sa2[i][h] << 16), x1 = __uint_as_float(sa2[i][h] & 0xffff0000u);
        if (PRO == 3) {
          g0 = fmaf(x0, pms[2 * h], pmt[2 * h]) > 0.f ? g0 : 0.f;
          g1 = fmaf(x1, pms[2 * h + 1], pmt[2 * h + 1]) > 0.f ? g1 : 0.f;
        }
        t[h] = dev::pack_bf16x2(fmaf(pa[2 * h], g0, fmaf(pb[2 * h], x0, pc[2 * h])),
                                fmaf(pa[2 * h + 1], g1, fmaf(pb[2 * h + 1], x1, pc[2 * h + 1])));
      }
      *reinterpret_cast<u32x4*>(A + row * SA + c * 16) = m + row < m_end ? t : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + 256 * i, row = q / CB, c = q - (q / CB) * CB;
      *reinterpret_cast<u32x4*>(B + row * SB + c * 16) = sb[i];
    }
  };

  f32x4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  if (m_begin < m_end) {
    load(m_begin);
    store(0, m_begin);
    lds_barrier();
    int cur = 0;
    for (int m = m_begin; m < m_end; m += BM) {
      const bool more = m + BM < m_end;
      if (more) load(m + BM);  // in flight during the MFMAs below
      const uint8_t* A = smem + cur * BUF;
      const uint8_t* B = A + ABYTES;
      // ---- wgrad: acc[n][k] += dYᵀ·X over this step's 64 pixel rows
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int r0 = s2 * 32 + 8 * g + q4;
        bf16x8 a[FN], b[FK];
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int col = wn * WTN + i * 16 + 4 * p4;
          const v4s v8[2] = {lds_tr16(A + r0 * SA + col * 2), lds_tr16(A + (r0 + 4) * SA + col * 2)};
          a[i] = __builtin_bit_cast(bf16x8, v8);
        }
#pragma unroll
        for (int j = 0; j < FK; ++j) {
          const int col = wk * WTK + j * 16 + 4 * p4;
          const v4s v8[2] = {lds_tr16(B + r0 * SB + col * 2), lds_tr16(B + (r0 + 4) * SB + col * 2)};
          b[j] = __builtin_bit_cast(bf16x8, v8);
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      // ---- dgrad: dXᵀ[k][m] = Σ_n W[n][k]·dY[m][n] for this step's rows; wave owns k rows wid·KW..
      {
        f32x4 d[KF][4];
#pragma unroll
        for (int kf = 0; kf < KF; ++kf)
#pragma unroll
          for (int mf = 0; mf < 4; ++mf) d[kf][mf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
        for (int ns = 0; ns < N / 32; ++ns) {
          const int r0 = ns * 32 + 8 * g + q4;
          bf16x8 a[KF], b[4];
#pragma unroll
          for (int kf = 0; kf < KF; ++kf) {
            const int col = wid * KW + kf * 16 + 4 * p4;
            const v4s v8[2] = {lds_tr16(Wl + r0 * SW + col * 2), lds_tr16(Wl + (r0 + 4) * SW + col * 2)};
            a[kf] = __builtin_bit_cast(bf16x8, v8);
          }
#pragma unroll
          for (int mf = 0; mf < 4; ++mf)
            b[mf] = *reinterpret_cast<const bf16x8*>(A + (mf * 16 + (lane & 15)) * SA + (ns * 32 + 8 * g) * 2);
#pragma unroll
          for (int kf = 0; kf < KF; ++kf)
#pragma unroll
            for (int mf = 0; mf < 4; ++mf) d[kf][mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kf], b[mf], d[kf][mf], 0, 0, 0);
        }
        // lane: k = wid·KW + kf·16 + 4g + r (r = 0..3), pixel m + mf·16 + (lane & 15)
#pragma unroll
        for (int mf = 0; mf < 4; ++mf) {
          const int mm = m + mf * 16 + (lane & 15);
          if (mm < m_end) {
#pragma unroll
            for (int kf = 0; kf < KF; ++kf) {
              uint2 pk;
              pk.x = dev::pack_bf16x2(d[kf][mf][0], d[kf][mf][1]);
              pk.y = dev::pack_bf16x2(d[kf][mf][2], d[kf][mf][3]);
              *reinterpret_cast<uint2*>(dX + (int64_t)mm * K + wid * KW + kf * 16 + 4 * g) = pk;
            }
          }
        }
      }
      if (more) store(cur ^ 1, m + BM);
      lds_barrier();
      cur ^= 1;
    }
  }
  float* out = ws + (int64_t)bid * N * K;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wn * WTN + i * 16 + (lane >> 4) * 4 + r;
        const int k = wk * WTK + j * 16 + (lane & 15);
        out[(int64_t)n * K + k] = acc[i][j][r];
      }
}

// dW = sum over the S slabs, cast to the weight dtype; 4 elements per lane.
template <typename W>
__global__ __launch_bounds__(512) void wgrad_reduce_kernel(const float* __restrict__ ws, int S, int64_t nk,
                                                           W* __restrict__ dw) {
  // block = 64 float4 columns x 8 slab groups: the slab sum is split 8 ways (4 independent
  // accumulators each) so a small weight with hundreds of slabs is not one long dependent chain
  __shared__ f32x4 red[8][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * 64 + c;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (v * 4 < nk) {
    const float* p = ws + v * 4;
    int s = g;
    for (; s + 24 < S; s += 32) {
      a0 += *reinterpret_cast<const f32x4*>(p + (int64_t)s * nk);
      a1 += *reinterpret_cast<const f32x4*>(p + (int64_t)(s + 8) * nk);
      a2 += *reinterpret_cast<const f32x4*>(p + (int64_t)(s + 16) * nk);
      a3 += *reinterpret_cast<const f32x4*>(p + (int64_t)(s + 24) * nk);
    }
    for (; s < S; s += 8) a0 += *reinterpret_cast<const f32x4*>(p + (int64_t)s * nk);
  }
  red[g][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (g == 0 && v * 4 < nk) {
    f32x4 acc = red[0][c];
#pragma unroll
    for (int i = 1; i < 8; ++i) acc += red[i][c];
    dev::Elem<W, float>::st(dw, v * 4 + 0, acc.x);
    dev::Elem<W, float>::st(dw, v * 4 + 1, acc.y);
    dev::Elem<W, float>::st(dw, v * 4 + 2, acc.z);
    dev::Elem<W, float>::st(dw, v * 4 + 3, acc.w);
  }
}

int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int BM, int BN, int WM, int WN, int OCC>
void launch_gemm(int pro, bool stats, bool bt, dim3 grid, size_t lds, hipStream_t s, const uint16_t* x,
                 const uint16_t* w, uint16_t* y, int64_t M, int N, int K, RowMap rm, const float* pss, float* part,
                 int mt, int nt, int groups, const uint16_t* x2, const EpiBN& epi, const ProOut& po) {
  auto go = [&](auto kern) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, grid, dim3(64 * WM * WN), lds, s, x, w, y, M, N, K, rm, pss, part, mt, nt, groups, x2,
                       epi, po);
  };
#define XDDP_G(P, S)                                                                                       \
  if (rm.stride > 1) go(conv1x1_gemm_kernel<BM, BN, WM, WN, P, S, true, false, false, OCC>);                \
  else go(conv1x1_gemm_kernel<BM, BN, WM, WN, P, S, false, false, false, OCC>)
  if (bt) {  // input gradient on the untransposed weight: stride 1, no statistics
    if (epi.part && pro == 2) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 2, false, false, true, true, OCC>);
    else if (epi.part) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 0, false, false, true, true, OCC>);
    else if (pro == 3) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 3, false, false, true, false, OCC>);
    else if (pro == 2) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 2, false, false, true, false, OCC>);
    else go(conv1x1_gemm_kernel<BM, BN, WM, WN, 0, false, false, true, false, OCC>);
  } else if (pro == 3) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 3, false, false, false, false, OCC>);  // stride-1 dgrad only
  else if (pro == 2) go(conv1x1_gemm_kernel<BM, BN, WM, WN, 2, false, false, false, false, OCC>);
  else if (pro == 1) { if (stats) XDDP_G(1, true); else XDDP_G(1, false); }
  else { if (stats) XDDP_G(0, true); else XDDP_G(0, false); }
#undef XDDP_G
  XDDP_HIP_CHECK(hipGetLastError());
}

}  // namespace

// x: [B, K, IH, IW] channels_last bf16; w: [N, K, 1, 1] bf16 (contiguous == [N][K]).
// prologue_ss: optional float [2, K] (scale, shift) -> op(x) = relu(x*scale + shift).
// Returns (y [B, N, OH, OW] channels_last, partials [groups, 3, N] or undefined).
std::vector<at::Tensor> conv1x1_gemm(const at::Tensor& x, const at::Tensor& w, int64_t stride,
                                     const c10::optional<at::Tensor>& prologue_ss, bool stats,
                                     const c10::optional<at::Tensor>& prologue_y, bool w_t,
                                     const c10::optional<at::Tensor>& epi_add, const c10::optional<at::Tensor>& epi_y,
                                     const c10::optional<at::Tensor>& epi_bits, const c10::optional<at::Tensor>& epi_mean,
                                     const c10::optional<at::Tensor>& epi_ss, int64_t epi_add_stride,
                                     const c10::optional<at::Tensor>& pro_out, const c10::optional<at::Tensor>& pro_bits,
                                     const c10::optional<at::Tensor>& pro_res, const c10::optional<at::Tensor>& pro_res_ss,
                                     const c10::optional<at::Tensor>& pro_nbt, const c10::optional<at::Tensor>& pro_res_nbt) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16, "conv1x1_gemm: x must be 4-D bf16 on GPU");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv1x1_gemm: x must be channels_last");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 1 && w.size(3) == 1 && w.scalar_type() == at::kBFloat16,
              "conv1x1_gemm: w must be [N, K, 1, 1] bf16");
  TORCH_CHECK(stride >= 1, "conv1x1_gemm: bad stride");
  // w_t: w is [K, N, 1, 1] (the forward weight of the conv whose input gradient this is), used as Wᵀ
  const int64_t B = x.size(0), K = x.size(1), IH = x.size(2), IW = x.size(3), N = w.size(w_t ? 1 : 0);
  TORCH_CHECK(w.size(w_t ? 0 : 1) == K, "conv1x1_gemm: channel mismatch");
  TORCH_CHECK(!w_t || (stride == 1 && !stats), "conv1x1_gemm: w_t is for stride-1 input gradients without stats");
  TORCH_CHECK(K % kBK == 0 && N % 64 == 0, "conv1x1_gemm: needs Cin % 64 == 0 and Cout % 64 == 0");
  auto wc = w.contiguous();  // [N][K] row-major for either weight memory format (1x1: same bytes)
  const int64_t OH = (IH - 1) / stride + 1, OW = (IW - 1) / stride + 1;
  const int64_t M = B * OH * OW;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31), "conv1x1_gemm: bad M");
  const bool has_y2 = prologue_y.has_value() && prologue_y->defined();
  const bool has_ss = prologue_ss.has_value() && prologue_ss->defined();
  auto def = [](const c10::optional<at::Tensor>& t) { return t.has_value() && t->defined(); };
  const bool has_res = def(pro_res), has_rss = def(pro_res_ss);
  const int pro = has_res ? (has_rss ? 5 : 4)
                          : has_y2 ? (has_ss && prologue_ss->numel() == 5 * K ? 3 : 2) : (has_ss ? 1 : 0);
  const int ncoef = pro == 3 ? 5 : pro == 2 ? 3 : 2;  // (PRO 5's residual coefficients come in pro_res_ss)
  if (has_res || def(pro_out) || def(pro_bits)) {
    TORCH_CHECK(!has_y2 && !w_t && stride == 1 && !(epi_add.has_value() && epi_add->defined()) &&
                    !(epi_ss.has_value() && epi_ss->defined()),
                "conv1x1_gemm: the apply prologue's side output / residual is for stride-1 forwards");
    TORCH_CHECK(has_ss, "conv1x1_gemm: the apply prologue needs prologue_ss");
    if (has_res)
      TORCH_CHECK(pro_res->sizes() == x.sizes() && pro_res->scalar_type() == at::kBFloat16 &&
                      pro_res->is_contiguous(at::MemoryFormat::ChannelsLast),
                  "conv1x1_gemm: pro_res must match x (bf16 channels_last)");
    if (has_rss)
      TORCH_CHECK(pro_res_ss->is_cuda() && pro_res_ss->scalar_type() == at::kFloat && pro_res_ss->numel() == 2 * K &&
                      pro_res_ss->is_contiguous(),
                  "conv1x1_gemm: pro_res_ss must be float [2, K]");
    if (def(pro_out))
      TORCH_CHECK(pro_out->sizes() == x.sizes() && pro_out->scalar_type() == at::kBFloat16 &&
                      pro_out->is_contiguous(at::MemoryFormat::ChannelsLast),
                  "conv1x1_gemm: pro_out must match x (bf16 channels_last)");
    if (def(pro_bits))
      TORCH_CHECK(has_res && def(pro_out) && pro_bits->scalar_type() == at::kByte && pro_bits->numel() * 8 == x.numel(),
                  "conv1x1_gemm: pro_bits needs the residual form and pro_out (uint8, one byte per 8 elements)");
    for (const auto* t : {&pro_nbt, &pro_res_nbt})
      if (def(*t)) TORCH_CHECK((*t)->scalar_type() == at::kLong && (*t)->numel() == 1, "conv1x1_gemm: bad nbt");
  }
  if (pro) TORCH_CHECK(has_ss && prologue_ss->scalar_type() == at::kFloat && prologue_ss->numel() == ncoef * K &&
                           prologue_ss->is_contiguous(),
                       "conv1x1_gemm: prologue coefficients must be float [2, K] (or [3|5, K] with prologue_y)");
  if (pro == 2 || pro == 3)
    TORCH_CHECK(prologue_y->sizes() == x.sizes() && prologue_y->scalar_type() == at::kBFloat16 &&
                    prologue_y->is_contiguous(at::MemoryFormat::ChannelsLast) && stride == 1 && !stats,
                "conv1x1_gemm: prologue_y must match x (bf16 channels_last), stride 1, no stats");
  auto y = at::empty({B, N, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const bool epi_form1 = epi_add.has_value() && epi_add->defined();
  const bool epi_form2 = !epi_form1 && epi_ss.has_value() && epi_ss->defined();
  const bool epi_on = epi_form1 || epi_form2;
  if (epi_on) {
    TORCH_CHECK(w_t && (pro == 0 || (epi_form2 && pro == 2)),
                "conv1x1_gemm: the BN-reduce epilogue needs w_t (and no prologue, or the BN-backward one with "
                "the mask-recompute epilogue)");
    TORCH_CHECK(epi_y.has_value() && epi_y->sizes() == y.sizes() && epi_y->scalar_type() == at::kBFloat16 &&
                    epi_y->is_contiguous(at::MemoryFormat::ChannelsLast) && epi_mean.has_value() &&
                    epi_mean->scalar_type() == at::kFloat && epi_mean->numel() == N && epi_mean->is_contiguous(),
                "conv1x1_gemm: epilogue y / mean must match the output (bf16 channels_last, float mean)");
    if (epi_form1) {
      TORCH_CHECK(epi_add_stride == 1 || epi_add_stride == 2, "conv1x1_gemm: epi_add_stride must be 1 or 2");
      const std::vector<int64_t> asz = epi_add_stride == 1 ? y.sizes().vec()
                                                           : std::vector<int64_t>{B, N, (OH + 1) / 2, (OW + 1) / 2};
      TORCH_CHECK(epi_add->sizes() == at::IntArrayRef(asz) && epi_add->scalar_type() == at::kBFloat16 &&
                      epi_add->is_contiguous(at::MemoryFormat::ChannelsLast) && epi_bits.has_value() &&
                      epi_bits->scalar_type() == at::kByte && epi_bits->numel() * 8 == y.numel(),
                  "conv1x1_gemm: epilogue add / bits must match the output (bf16 channels_last, uint8 bits)");
    } else {
      TORCH_CHECK(epi_ss->scalar_type() == at::kFloat && epi_ss->numel() >= 2 * N && epi_ss->is_contiguous(),
                  "conv1x1_gemm: epilogue scale/shift must be float [2, N]");
    }
  }
  const int BN = (N % 128 == 0) ? 128 : 64;
  // Tile / occupancy choices, each measured on ResNet-50 bs256 (r2 A/Bs, now fixed):
  // * the BN-reduce epilogue GEMM (EPI) runs 64x128 tiles (8 waves of 32x32, two blocks per CU,
  //   128 VGPRs without spills): half the live epilogue registers of the 128x128 tile, so two
  //   tiles' loads are in flight per CU — 271/157/89/73 vs 337/190/104/79 us on the stage shapes
  //   (profiles/r2_epi_dgrad_shapes.txt), 12,418-12,422 vs 12,120-12,154 img/s; the forward and
  //   BN-backward-prologue GEMMs on 64x128 measured no gain (12,304 / 12,446 vs 12,438-12,454);
  // * a 64-wide EPI tile (N % 128 != 0) runs at occupancy 2 (one block per CU, 190 VGPRs): its
  //   epilogue loads stay live across the K loop and spill 76 registers within the 128 of
  //   occupancy 4 (331/189/105/78 vs 614/334/200/96 us, 11,969 vs 10,915 img/s);
  // * everything else at occupancy 4, persistent grid of 2 blocks per CU (one resident round).
  // * the block-output prologue (pro 4 / 5: two A sources, the mask bits and the statistics live
  //   together) on 128-wide N tiles runs 64-row tiles at occupancy 4 (its 128-row tile spills
  //   35-41 registers there); on 64-wide N tiles the 128-row tile fits (124 VGPRs), the same tile
  //   and grid as the plain statistics GEMM, so those statistics partials are bitwise the same
  const bool bm64 = (epi_on && BN == 128) || (pro >= 4 && BN == 128);
  const int BM = bm64 ? 64 : 128;
  const int mtiles = (int)((M + BM - 1) / BM), ntiles = (int)(N / BN);
  const int kocc = bm64 ? 4 : (epi_on ? 2 : 4);
  constexpr int blocks_per_cu = 2;
  const int target = num_cus() * (kocc == 2 ? 1 : blocks_per_cu);
  int groups = std::max(1, std::min(mtiles, (target + ntiles - 1) / ntiles));
  at::Tensor part = stats ? at::empty({groups, 3, N}, x.options().dtype(at::kFloat))
                          : (epi_on ? at::empty({groups, N, 2}, x.options().dtype(at::kFloat)) : at::Tensor());
  EpiBN epi{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0};
  if (epi_form1)
    epi = EpiBN{reinterpret_cast<const uint16_t*>(epi_add->data_ptr()), reinterpret_cast<const uint16_t*>(epi_y->data_ptr()),
                epi_bits->data_ptr<uint8_t>(), epi_mean->data_ptr<float>(), part.data_ptr<float>(), nullptr,
                epi_add_stride == 2 ? (int)OH : 0, epi_add_stride == 2 ? (int)OW : 0};
  else if (epi_form2)
    epi = EpiBN{nullptr, reinterpret_cast<const uint16_t*>(epi_y->data_ptr()), nullptr, epi_mean->data_ptr<float>(),
                part.data_ptr<float>(), epi_ss->data_ptr<float>(), 0, 0};
  RowMap rm{(int)OH, (int)OW, (int)IH, (int)IW, (int)stride};
  const dim3 grid(groups * ntiles);
  const size_t bbytes = w_t ? (size_t)64 * (BN * 2 + 32) : (size_t)BN * 128;
  const size_t lds = 2 * ((size_t)BM * 128 + bbytes) + (pro ? (pro == 5 ? 4 : ncoef) * K * sizeof(float) : 0) +
                     (epi_on ? 3 * (size_t)BN * sizeof(float) : 0);
  const auto* x2p = pro >= 4 ? reinterpret_cast<const uint16_t*>(pro_res->data_ptr())
                   : pro >= 2 ? reinterpret_cast<const uint16_t*>(prologue_y->data_ptr()) : nullptr;
  const ProOut po{def(pro_out) ? reinterpret_cast<uint16_t*>(pro_out->data_ptr()) : nullptr,
                  def(pro_bits) ? pro_bits->data_ptr<uint8_t>() : nullptr,
                  has_rss ? pro_res_ss->data_ptr<float>() : nullptr,
                  def(pro_nbt) ? pro_nbt->data_ptr<int64_t>() : nullptr,
                  def(pro_res_nbt) ? pro_res_nbt->data_ptr<int64_t>() : nullptr};
  const auto* xp = reinterpret_cast<const uint16_t*>(x.data_ptr());
  const auto* wp = reinterpret_cast<const uint16_t*>(wc.data_ptr());
  auto* yp = reinterpret_cast<uint16_t*>(y.data_ptr());
  const float* pss = pro ? prologue_ss->data_ptr<float>() : nullptr;
  float* pp = stats ? part.data_ptr<float>() : nullptr;  // (EPI partials travel in epi)
#define XDDP_LG(BN_, WM_, WN_, OCC_)                                                                            \
  launch_gemm<128, BN_, WM_, WN_, OCC_>(pro, stats, w_t, grid, lds, stream, xp, wp, yp, M, (int)N, (int)K, rm, pss, pp, \
                                        mtiles, ntiles, groups, x2p, epi, po)
  if (pro >= 4) {
    auto go = [&](auto kern) {
      ensure_dyn_lds((const void*)kern, lds);
      hipLaunchKernelGGL(kern, grid, dim3(512), lds, stream, xp, wp, yp, M, (int)N, (int)K, rm, pss, pp, mtiles, ntiles,
                         groups, x2p, epi, po);
    };
#define XDDP_P45(BM_, BN_, WM_, WN_)                                                                     \
    if (pro == 5) { if (stats) go(conv1x1_gemm_kernel<BM_, BN_, WM_, WN_, 5, true, false, false, false, 4>);    \
                    else go(conv1x1_gemm_kernel<BM_, BN_, WM_, WN_, 5, false, false, false, false, 4>); }   \
    else { if (stats) go(conv1x1_gemm_kernel<BM_, BN_, WM_, WN_, 4, true, false, false, false, 4>);             \
           else go(conv1x1_gemm_kernel<BM_, BN_, WM_, WN_, 4, false, false, false, false, 4>); }
    if (BN == 128) { XDDP_P45(64, 128, 2, 4) } else { XDDP_P45(128, 64, 8, 1) }
#undef XDDP_P45
    XDDP_HIP_CHECK(hipGetLastError());
  } else if (bm64) {  // (EPI implies w_t; pro is 0 or the BN-backward form 2)
    auto kern = pro == 2 ? conv1x1_gemm_kernel<64, 128, 2, 4, 2, false, false, true, true, 4>
                         : conv1x1_gemm_kernel<64, 128, 2, 4, 0, false, false, true, true, 4>;
    hipLaunchKernelGGL(kern, grid, dim3(512), lds, stream, xp, wp, yp, M, (int)N, (int)K, rm, pss, pp, mtiles, ntiles,
                       groups, x2p, epi, po);
    XDDP_HIP_CHECK(hipGetLastError());
  } else if (BN == 128) { if (kocc == 2) XDDP_LG(128, 4, 2, 2); else XDDP_LG(128, 4, 2, 4); }
  else { if (kocc == 2) XDDP_LG(64, 8, 1, 2); else XDDP_LG(64, 8, 1, 4); }
#undef XDDP_LG
  return {y, part};
}


// dY: [B, N, OH, OW] channels_last bf16; x: [B, K, IH, IW] channels_last bf16 (the conv input);
// returns dW [N, K, 1, 1] in w_like's dtype (fp32 accumulation, split over pixel rows).
// With prologue_y/coef: dY = coef[0]·dy + coef[1]·prologue_y + coef[2] per dY channel (stride 1).
at::Tensor conv1x1_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t stride, const at::Tensor& w_like,
                         const c10::optional<at::Tensor>& prologue_y, const c10::optional<at::Tensor>& coef) {
  const auto wdtype = w_like.scalar_type();
  const bool has_y2 = prologue_y.has_value() && prologue_y->defined();
  const int pro = has_y2 ? (coef.has_value() && coef->defined() && coef->numel() == 5 * dy.size(1) ? 3 : 2) : 0;
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16,
              "conv1x1_wgrad: bf16 GPU tensors expected");
  TORCH_CHECK(dy.dim() == 4 && x.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv1x1_wgrad: channels_last 4-D tensors expected");
  const int64_t B = x.size(0), K = x.size(1), IH = x.size(2), IW = x.size(3), N = dy.size(1);
  const int64_t OH = (IH - 1) / stride + 1, OW = (IW - 1) / stride + 1;
  TORCH_CHECK(dy.size(0) == B && dy.size(2) == OH && dy.size(3) == OW, "conv1x1_wgrad: dy/x shape mismatch");
  TORCH_CHECK(N % 64 == 0 && K % 64 == 0, "conv1x1_wgrad: channel counts must be multiples of 64");
  const int64_t M = B * OH * OW;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31), "conv1x1_wgrad: bad M");
  if (pro)
    TORCH_CHECK(prologue_y->sizes() == dy.sizes() && prologue_y->scalar_type() == at::kBFloat16 &&
                    prologue_y->is_contiguous(at::MemoryFormat::ChannelsLast) && stride == 1 && coef.has_value() &&
                    coef->defined() && coef->scalar_type() == at::kFloat && coef->numel() == (pro == 3 ? 5 : 3) * N &&
                    coef->is_contiguous(),
                "conv1x1_wgrad: prologue_y must match dy (bf16 channels_last, stride 1) with float coef [3|5, N]");
  const auto* y2p = pro ? reinterpret_cast<const uint16_t*>(prologue_y->data_ptr()) : nullptr;
  const float* cfp = pro ? coef->data_ptr<float>() : nullptr;
  const int TN = N % 128 == 0 ? 128 : 64, TK = K % 128 == 0 ? 128 : 64;
  const int ntiles = (int)(N / TN), ktiles = (int)(K / TK), tiles = ntiles * ktiles;
  const int64_t steps = (M + 63) / 64;
  int S = (int)std::max<int64_t>(1, std::min<int64_t>(steps, (int64_t)num_cus() * 2 / tiles));
  const int64_t mchunk = ((steps + S - 1) / S) * 64;
  S = (int)((M + mchunk - 1) / mchunk);
  auto ws = at::empty({S, N, K}, dy.options().dtype(at::kFloat));
  auto dw = at::empty({N, K, 1, 1}, dy.options().dtype(wdtype));
  auto stream = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  RowMap rm{(int)OH, (int)OW, (int)IH, (int)IW, (int)stride};
  const size_t lds = 2 * (size_t)64 * ((TN * 2 + 32) + (TK * 2 + 32));
  auto go = [&](auto kern) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(S * tiles), dim3(256), lds, stream,
                       reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                       ws.data_ptr<float>(), (int)M, (int)N, (int)K, rm, ntiles, ktiles, (int)mchunk, y2p, cfp);
    XDDP_HIP_CHECK(hipGetLastError());
  };
  const bool strided = stride > 1;
#define XDDP_W(A, Bk) \
  if (pro == 3) go(conv1x1_wgrad_kernel<A, Bk, false, 3>);                                         \
  else if (pro == 2) go(conv1x1_wgrad_kernel<A, Bk, false, 2>);                                    \
  else if (strided) go(conv1x1_wgrad_kernel<A, Bk, true, 0>); else go(conv1x1_wgrad_kernel<A, Bk, false, 0>)
  if (TN == 128 && TK == 128) { XDDP_W(128, 128); }
  else if (TN == 128) { XDDP_W(128, 64); }
  else if (TK == 128) { XDDP_W(64, 128); }
  else { XDDP_W(64, 64); }
#undef XDDP_W
  const int64_t nk = N * K;
  const int grid = (int)((nk / 4 + 63) / 64);
  auto red = [&](auto tag) {
    using W = decltype(tag);
    hipLaunchKernelGGL((wgrad_reduce_kernel<W>), dim3(grid), dim3(512), 0, stream, ws.data_ptr<float>(), S, nk,
                       reinterpret_cast<W*>(dw.data_ptr()));
    XDDP_HIP_CHECK(hipGetLastError());
  };
  switch (wdtype) {
    case at::kBFloat16: red(dev::bf16_t{}); break;
    case at::kFloat: red(float{}); break;
    case at::kHalf: red(dev::f16_t{}); break;
    default: TORCH_CHECK(false, "conv1x1_wgrad: unsupported weight dtype");
  }
  return dw;
}

// Fused stride-1 1x1 backward (see conv1x1_bwd_fused_kernel): g, y2 [B, N, H, W], coef [3|5, N]
// (dY = k1·g + k2·y2 + k3', with the ReLU mask recomputed from y2 for 5 rows), x [B, K, H, W],
// w [N, K, 1, 1] -> (dx [B, K, H, W], dw like w). (N, K) in {(256, 64), (64, 256)}.
bool conv1x1_bwd_fused_supported(int64_t N, int64_t K) { return (N == 256 && K == 64) || (N == 64 && K == 256); }

std::vector<at::Tensor> conv1x1_bwd_fused(const at::Tensor& g, const at::Tensor& y2, const at::Tensor& coef,
                                          const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kBFloat16 && g.dim() == 4 &&
                  g.is_contiguous(at::MemoryFormat::ChannelsLast) && y2.sizes() == g.sizes() &&
                  y2.scalar_type() == at::kBFloat16 && y2.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv1x1_bwd_fused: g, y2 must be matching bf16 channels_last tensors");
  const int64_t B = x.size(0), K = x.size(1), H = x.size(2), Wd = x.size(3), N = g.size(1);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  g.size(0) == B && g.size(2) == H && g.size(3) == Wd,
              "conv1x1_bwd_fused: x must be bf16 channels_last with g's batch and spatial size (stride 1)");
  TORCH_CHECK(conv1x1_bwd_fused_supported(N, K), "conv1x1_bwd_fused: unsupported (N, K)");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.numel() == N * K && w.size(0) == N && w.is_contiguous(),
              "conv1x1_bwd_fused: w must be contiguous bf16 [N, K, 1, 1]");
  const int pro = coef.numel() == 5 * N ? 3 : 2;
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && (coef.numel() == 3 * N || pro == 3),
              "conv1x1_bwd_fused: coef must be float [3|5, N]");
  const int64_t M = B * H * Wd;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 31), "conv1x1_bwd_fused: bad M");
  const int64_t steps = (M + 63) / 64;
  int S = (int)std::max<int64_t>(1, std::min<int64_t>(steps, (int64_t)num_cus()));
  const int64_t mchunk = ((steps + S - 1) / S) * 64;
  S = (int)((M + mchunk - 1) / mchunk);
  auto dx = at::empty({B, K, H, Wd}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto ws = at::empty({S, N, K}, x.options().dtype(at::kFloat));
  auto dw = at::empty({N, K, 1, 1}, w.options().memory_format(at::MemoryFormat::Contiguous));
  auto stream = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  const size_t lds = 2 * (size_t)64 * ((N * 2 + 32) + (K * 2 + 32)) + (size_t)N * (K * 2 + 32);
  auto go = [&](auto kern) {
    ensure_dyn_lds((const void*)kern, lds);
    hipLaunchKernelGGL(kern, dim3(S), dim3(256), lds, stream, reinterpret_cast<const uint16_t*>(g.data_ptr()),
                       reinterpret_cast<const uint16_t*>(y2.data_ptr()), coef.data_ptr<float>(),
                       reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                       reinterpret_cast<uint16_t*>(dx.data_ptr()), ws.data_ptr<float>(), (int)M, (int)mchunk);
    XDDP_HIP_CHECK(hipGetLastError());
  };
  if (N == 256) { if (pro == 3) go(conv1x1_bwd_fused_kernel<256, 64, 3>); else go(conv1x1_bwd_fused_kernel<256, 64, 2>); }
  else { if (pro == 3) go(conv1x1_bwd_fused_kernel<64, 256, 3>); else go(conv1x1_bwd_fused_kernel<64, 256, 2>); }
  const int64_t nk = N * K;
  hipLaunchKernelGGL((wgrad_reduce_kernel<dev::bf16_t>), dim3((unsigned)((nk / 4 + 63) / 64)), dim3(512), 0, stream,
                     ws.data_ptr<float>(), S, nk, reinterpret_cast<dev::bf16_t*>(dw.data_ptr()));
  XDDP_HIP_CHECK(hipGetLastError());
  return {dx, dw};
}


// partials [groups, 3, N] (or [3, N, groups] when group_minor) -> (mean, invstd, scale_shift
// [2, N]); updates running stats. M = rows behind the partials; M <= 0 = sum the partials' counts.
std::vector<at::Tensor> bn_stats_from_partials(const at::Tensor& part, int64_t M,
                                               const c10::optional<at::Tensor>& weight,
                                               const c10::optional<at::Tensor>& bias,
                                               const c10::optional<at::Tensor>& running_mean,
                                               const c10::optional<at::Tensor>& running_var,
                                               const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                               bool cumulative, double eps, bool group_minor) {
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.size(group_minor ? 0 : 1) == 3 &&
                  part.scalar_type() == at::kFloat && part.is_contiguous(),
              "bn_stats_from_partials: partials must be float [groups, 3, C] (or [3, C, groups])");
  const int groups = (int)part.size(group_minor ? 2 : 0), C = (int)part.size(group_minor ? 1 : 2);
  const int64_t gs = group_minor ? 1 : 3 * C, ks = group_minor ? (int64_t)C * groups : C,
                cs = group_minor ? groups : 1;
  auto fopt = part.options();
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt), ss = at::empty({2, C}, fopt);
  auto stream = c10::hip::getCurrentHIPStream(part.device().index()).stream();
  auto opt = [](const c10::optional<at::Tensor>& t) { return t.has_value() && t->defined(); };
  const auto wdt = opt(weight) ? weight->scalar_type() : (opt(running_mean) ? running_mean->scalar_type() : at::kFloat);
  auto go = [&](auto tag) {
    using W = decltype(tag);
    auto P = [&](const c10::optional<at::Tensor>& t) { return opt(t) ? reinterpret_cast<W*>(t->data_ptr()) : nullptr; };
    hipLaunchKernelGGL((bn_partial_finalize_kernel<W>), dim3(C), dim3(256), 0, stream, part.data_ptr<float>(), groups,
                       C, gs, ks, cs, M, P(weight), P(bias), P(running_mean), P(running_var),
                       opt(num_batches_tracked) ? num_batches_tracked->data_ptr<int64_t>() : nullptr, (float)momentum,
                       cumulative, (float)eps, mean.data_ptr<float>(), invstd.data_ptr<float>(), ss.data_ptr<float>(),
                       ss.data_ptr<float>() + C);
    XDDP_HIP_CHECK(hipGetLastError());
  };
  switch (wdt) {
    case at::kFloat: go(float{}); break;
    case at::kBFloat16: go(dev::bf16_t{}); break;
    case at::kHalf: go(dev::f16_t{}); break;
    default: TORCH_CHECK(false, "bn_stats_from_partials: unsupported weight dtype");
  }
  return {mean, invstd, ss};
}

}  // namespace kernels
}  // namespace xddp
