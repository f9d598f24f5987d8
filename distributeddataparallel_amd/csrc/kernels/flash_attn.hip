// Flash attention (forward + backward) for gfx950 MFMA, bf16 in/out, fp32 softmax statistics:
// the ViT-L/16 (D = 64, 197 tokens, non-causal) and Llama-3-8B (D = 128, causal, GQA 32:8)
// configs of BASELINE.json. torch's SDPA on this ROCm build runs AOTriton kernels at ~13 % (fwd)
// and ~7 % (bwd) of the MI355X bf16 MFMA peak at Llama's shape; these are written for CDNA4
// directly.
//
// Layout: q, k, v, o are [B, S, H, D] with D contiguous and any B/S/H strides (so the projection
// outputs are used as views and o comes out ready for the output projection, no transposes).
// GQA: q head h reads kv head h / (Hq / Hkv).
//
// Forward (one workgroup = 8 waves = 256 query rows of one (batch, head); wave = 32 rows; two
// waves per SIMD so one wave's softmax / LDS / load waits hide under the other's MFMAs):
// * swapped scores: S^T = K·Q^T on mfma_f32_32x32x16_bf16 with K as the A operand (from LDS) and
//   Q^T as the B operand (Q kept in registers), so a lane owns ONE query row (lane & 31) and half
//   of a 32-key tile: the row max / sum are in-lane plus one exchange with lane ^ 32;
// * O is accumulated transposed, O^T = V^T·P^T, with V^T as the A operand read by gfx950's
//   transposing ds_read_b64_tr_b16 and P^T (the score accumulator, rounded to bf16) as the B
//   operand: the accumulator layout of S^T IS the B-operand layout when the PV reduction walks
//   the keys in the order the lanes hold them (lane group g holds keys 4g..4g+3, 8+4g..8+4g+3 of
//   each 16), and V's rows are read in that same order. O^T's lane also owns one query row, so
//   the online-softmax rescale is a per-lane scalar;
// * K/V tiles (64 keys) are register-staged: the next tile's global loads are issued before the
//   current tile's MFMAs and written to LDS after them (one LDS buffer, two barriers per tile).
//   Every LDS tile uses one XOR chunk swizzle (uswz) that is conflict-free for both the b128 row
//   reads and the transposed reads, so a tile is staged once whichever way it is read;
// * softmax in the exp2 domain (scale·log2 e folded in, v_exp_f32), LSE = m + log2(l) saved.
//
// Backward: preprocess delta = rowsum(dO·O); dK/dV kernel (one workgroup = 128 keys of one
// (batch, kv head) and a share of the GQA group's query heads; D = 128: one 4-wave group, two
// workgroups per CU; D = 64: two 4-wave groups splitting the (query head, 32-row query tile)
// items), LDS-DMA double-buffered Q / dO tiles; S = Q·K^T and dP = dO·V^T with the KEY on the lane, so P and dS are directly the B operands of dV^T += dO^T·P and
// dK^T += Q^T·dS); dQ kernel (8 waves x 32 query rows; S^T and dP^T with the query on the lane,
// dQ^T += K^T·dS^T). No atomics: dQ and dK/dV are separate passes (S and dP are recomputed in
// both), each bitwise reproducible — except when one workgroup holds every key of a head (D = 64,
// non-causal, Sk <= 256: ViT), where the dK/dV kernel also produces dQ from its dS (FQ below).
//
// MI355X, Llama-3-8B shape (B1 S4096 H32/8 D128 causal): fwd 0.174 ms, fwd+bwd 0.939 ms vs torch
// SDPA (AOTriton) 0.423 / 2.286 ms; ViT-L/16 (B64 S197 H16 D64): 0.043 / 0.190 vs 0.062 / 0.352 ms
// (profiles/r2_flash_attn_v3.txt).
#include <cstdlib>

#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "common.h"
#include "kernels/dev_utils.h"
#include "kernels/norm.h"

namespace xddp {
namespace kernels {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
using dev::u32x4;

constexpr int kBK = 64;   // keys per K/V tile
constexpr float kNegInf = -1e30f;
constexpr float kLazy = 8.f;  // log2-domain headroom before the running max is raised

__device__ __forceinline__ v4s lds_tr16(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

// 16-B chunk XOR swizzle of a row-major [rows][D] LDS tile, conflict-free for BOTH read patterns
// used on it: ds_read_b128 row fragments (16 consecutive rows at one chunk) and ds_read_b64_tr_b16
// transposed fragments (4 consecutive rows x 4 consecutive chunks per half-wave). So a tile is
// staged once and read both ways (the dQ / dK,dV GEMMs read the same Q, dO, K tiles transposed).
template <int D>
__device__ __forceinline__ int uswz(int row, int chunk) {
  return chunk ^ (D == 128 ? (4 * (row & 3) | ((row >> 2) & 3)) : (4 * ((row >> 1) & 1) | ((row >> 2) & 3)));
}

// keys (or queries) held by lane group g (= lane >> 5) in element e (0..7) of a 16-wide k-step
// of a 32x32 accumulator: 4g + (e & 3) + 8 (e >> 2)
__device__ __forceinline__ int kappa(int g, int e) { return 4 * g + (e & 3) + 8 * (e >> 2); }

struct Strides {
  int64_t b, s, h;
};

// A fragment of a row-major tile in LDS: rows r0 + (lane & 31), 8 elements from column 16 ks + 8 (lane >> 5)
template <int D>
__device__ __forceinline__ bf16x8 ld_rowfrag(const uint8_t* T, int r, int ks, int lane) {
  const int chunk = 2 * ks + (lane >> 5);
  return *reinterpret_cast<const bf16x8*>(T + r * (D * 2) + uswz<D>(r, chunk) * 16);
}

// transposed fragment: element e of lane l = T[rows rbase + kappa(g, e)][col cbase + (l & 31)]
template <int D>
__device__ __forceinline__ bf16x8 ld_trfrag(const uint8_t* T, int rbase, int cbase, int lane) {
  const int g = lane >> 5, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * p4;  // 4 bf16 = 8 B per lane
  const int r0 = rbase + 4 * g + q4, r1 = r0 + 8;
  const int c0 = col >> 3, off = (col & 7) * 2;
  const v4s lo = lds_tr16(T + r0 * (D * 2) + uswz<D>(r0, c0) * 16 + off);
  const v4s hi = lds_tr16(T + r1 * (D * 2) + uswz<D>(r1, c0) * 16 + off);
  const v4s v8[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v8);
}

// register-staged tile load: rows [r0, r0 + 64) of a [B, S, H, D] tensor (zero past `rows`)
template <int D, int NTH = 256>
struct TileRegs {
  static constexpr int CH = kBK * D / 8 / NTH;  // 16-B chunks per thread
  u32x4 v[CH];
  __device__ void load(const uint16_t* base, int64_t ss, int r0, int rows, int tid) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int q = tid + NTH * i, r = q / (D / 8), c = q % (D / 8);
      v[i] = (r0 + r < rows) ? *reinterpret_cast<const u32x4*>(base + (int64_t)(r0 + r) * ss + c * 8)
                             : u32x4{0, 0, 0, 0};
    }
  }
  __device__ void store(uint8_t* T, int tid) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int q = tid + NTH * i, r = q / (D / 8), c = q % (D / 8);
      *reinterpret_cast<u32x4*>(T + r * (D * 2) + uswz<D>(r, c) * 16) = v[i];
    }
  }
};

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// every wave's LDS-DMA for the current stage has landed and every wave is done with the previous
// stage (whose buffer the next DMA overwrites)
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// K/V tile rows [r0, r0 + 64) of a [B, S, H, D] tensor -> LDS by LDS-DMA (1 KB per wave
// instruction, lane i -> 16 B at slot i; the source chunk is pre-swizzled so the LDS image is the
// uswz layout). Rows past `rows` read row rows - 1 (finite; the caller masks those keys).
template <int D, int NW>
__device__ __forceinline__ void dma_tile(const uint16_t* base, int64_t ss, int r0, int rows, uint8_t* T, int w,
                                         int lane) {
  constexpr int RPI = 512 / D, NI = kBK / RPI, PER = NI / NW;
  static_assert(PER * NW == NI, "tile pieces must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int ins = w * PER + i, r = ins * RPI + lane / (D / 8);
    const int c = uswz<D>(r, lane % (D / 8));
    const int64_t row = min(r0 + r, rows - 1);
    __builtin_amdgcn_global_load_lds((const void*)(base + row * ss + c * 8), (lds_ptr_t)(T + ins * 1024), 16, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------ fwd
// NW waves x 32 query rows per workgroup. At NW = 8 two waves share each SIMD, so one wave's
// softmax, LDS reads and global-load waits overlap the other's MFMAs (at 4 waves, one per SIMD,
// the kernel ran ~12K cycles per K/V tile against ~1K of MFMA work).
// WH (whole K/V, non-causal D = 64 with Sk <= 256: ViT's 197 tokens): every K/V tile of the head
// is DMA'd up front (64 KB of LDS) and the tile loop runs without barriers; waves whose 32 query
// rows all lie past Sq skip the math.
template <int D, bool CAUSAL, int NW, bool WH = false>
__global__ __launch_bounds__(64 * NW, WH && NW == 8 ? 4 : 1) void fa_fwd_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                        const uint16_t* __restrict__ V, uint16_t* __restrict__ O,
                                                        float* __restrict__ LSE, int Sq, int Sk, int Hq, int Hkv,
                                                        Strides qs, Strides ks, Strides vs, Strides os,
                                                        float scale_log2, int nqb) {
  constexpr int KS = D / 16, NT = D / 32, BQ = 32 * NW;
  static_assert(!WH || (!CAUSAL && D == 64), "whole-K/V staging is the non-causal D = 64 form");
  __shared__ __attribute__((aligned(16))) uint8_t KVs[WH ? 4 : 2][2][kBK * D * 2];  // [stage or tile][K, V]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 5;
  const int bh = blockIdx.y, b = bh / Hq, h = bh % Hq, hk = h / (Hq / Hkv);
  const uint16_t* Qb = Q + b * qs.b + h * qs.h;
  const uint16_t* Kb = K + b * ks.b + hk * ks.h;
  const uint16_t* Vb = V + b * vs.b + hk * vs.h;
  // causal: a workgroup takes query blocks (nqb - 1 - x, x) — a heavy and a light one, the same
  // total number of K/V tiles for every workgroup (one pass when they coincide)
  const int npass = CAUSAL && (int)blockIdx.x != nqb - 1 - (int)blockIdx.x ? 2 : 1;
#pragma unroll 1
  for (int pass = 0; pass < npass; ++pass) {
    const int qb = CAUSAL ? (pass == 0 ? nqb - 1 - (int)blockIdx.x : (int)blockIdx.x) : (int)blockIdx.x;
    const int q0 = qb * BQ, qw = q0 + 32 * w;  // wave rows [qw, qw + 32)
    const int qrow = qw + (lane & 31);
    bf16x8 qf[KS];
    f32x16 acc_o[NT];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
      qf[s2] = qrow < Sq ? *reinterpret_cast<const bf16x8*>(Qb + (int64_t)qrow * qs.s + 16 * s2 + 8 * g) : bf16x8{};
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc_o[n][i] = 0.f;
    // m_run: the (scaled, log2-domain) reference max the accumulators are relative to. It is only
    // raised when a row max exceeds it by more than kLazy (wave-uniform test), so most tiles skip
    // the 64-multiply rescale; P = exp2(s - m_run) then stays below 2^kLazy (exact in fp32 / bf16 range).
    float m_run = kNegInf, l_run = 0.f;

    const int kend = CAUSAL ? min(Sk, q0 + BQ) : Sk;
    const int ntiles = (kend + kBK - 1) / kBK;
    if (WH) {
      for (int j = 0; j < ntiles; ++j) {
        dma_tile<D, NW>(Kb, ks.s, j * kBK, Sk, KVs[j][0], w, lane);
        dma_tile<D, NW>(Vb, vs.s, j * kBK, Sk, KVs[j][1], w, lane);
      }
      dma_barrier();
    } else {
      dma_tile<D, NW>(Kb, ks.s, 0, Sk, KVs[0][0], w, lane);
      dma_tile<D, NW>(Vb, vs.s, 0, Sk, KVs[0][1], w, lane);
    }
    for (int j = 0; j < ntiles; ++j) {
      const int k0 = j * kBK;
      if (!WH) {
        dma_barrier();
        if (j + 1 < ntiles) {  // next tile in flight during this tile's math
          dma_tile<D, NW>(Kb, ks.s, k0 + kBK, Sk, KVs[(j + 1) & 1][0], w, lane);
          dma_tile<D, NW>(Vb, vs.s, k0 + kBK, Sk, KVs[(j + 1) & 1][1], w, lane);
        }
      }
      const uint8_t* Kt = KVs[WH ? j : (j & 1)][0];
      const uint8_t* Vt = KVs[WH ? j : (j & 1)][1];
      if (WH ? qw < Sq : (!CAUSAL || k0 <= qw + 31)) {  // a wave whose rows all precede the tile skips it
        f32x16 sc[2];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) sc[t][i] = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2) sc[t] = mfma32(ld_rowfrag<D>(Kt, 32 * t + (lane & 31), s2, lane), qf[s2], sc[t]);
        // masks only on the tiles that need them (the causal diagonal, the key tail): wave-uniform
        const bool masked = k0 + kBK > Sk || (CAUSAL && k0 + kBK - 1 > qw);
        float mx = kNegInf;
        {  // last visible key of this lane's row, tile-relative (no limit off the boundary)
          const int lim = masked ? (CAUSAL ? min(qrow, Sk - 1) : Sk - 1) - k0 : (1 << 30);
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (32 * t + kappa(g, i & 7) + 16 * (i >> 3) > lim) sc[t][i] = kNegInf;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[t][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;  // the scale is positive: max commutes
        const bool raise = mx > m_run + kLazy;
        if (__builtin_amdgcn_ballot_w64(raise) != 0) {  // some row of the wave needs a new reference
          const float m_new = fmaxf(m_run, mx);
          const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
          l_run *= alpha;
#pragma unroll
          for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc_o[n][i] *= alpha;
          m_run = m_new;
        }
        bf16x8 pf[4];
        float ls = 0.f;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int t = kk >> 1, hh = kk & 1;
          uint32_t pk[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float p0 = __builtin_amdgcn_exp2f(fmaf(sc[t][8 * hh + 2 * e], scale_log2, -m_run));
            const float p1 = __builtin_amdgcn_exp2f(fmaf(sc[t][8 * hh + 2 * e + 1], scale_log2, -m_run));
            ls += p0 + p1;
            pk[e] = dev::pack_bf16x2(p0, p1);
          }
          pf[kk] = __builtin_bit_cast(bf16x8, pk);
        }
        l_run += ls;
        // O^T += V^T P^T over the 4 16-key steps of the tile
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int n = 0; n < NT; ++n) acc_o[n] = mfma32(ld_trfrag<D>(Vt, 16 * kk, 32 * n, lane), pf[kk], acc_o[n]);
      }
    }
    lds_barrier();  // (causal pairs) every wave is done with the stages before the next pass refills them
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    if (qrow < Sq) {
      const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
      uint16_t* Ob = O + b * os.b + h * os.h + (int64_t)qrow * os.s;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // 4 consecutive d per store: d = 32n + 4g + 8q + 0..3
          uint2 pk;
          pk.x = dev::pack_bf16x2(acc_o[n][4 * q] * inv, acc_o[n][4 * q + 1] * inv);
          pk.y = dev::pack_bf16x2(acc_o[n][4 * q + 2] * inv, acc_o[n][4 * q + 3] * inv);
          *reinterpret_cast<uint2*>(Ob + 32 * n + 4 * g + 8 * q) = pk;
        }
      if (g == 0) LSE[(int64_t)bh * Sq + qrow] = m_run + log2f(fmaxf(l_tot, 1e-30f));
    }
  }
}

// ------------------------------------------------------------------------------------------ bwd
// delta[bh][q] = sum_d dO[q][d] · O[q][d] (fp32): D / 8 lanes per query row, 16-B loads, a
// shuffle reduction inside each lane group (64 / (D / 8) rows per wave)
template <int D>
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(const uint16_t* __restrict__ O, const uint16_t* __restrict__ dO,
                                                         float* __restrict__ delta, int64_t rows, int Sq, int Hq,
                                                         Strides os, Strides dos) {
  constexpr int LPR = D / 8;  // lanes per row
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / LPR;
  const int c = (int)(t % LPR) * 8;
  float s = 0.f;
  if (row < rows) {
    const int q = (int)(row % Sq);
    const int64_t bh = row / Sq;
    const int b = (int)(bh / Hq), h = (int)(bh % Hq);
    const dev::u32x4 ov = *reinterpret_cast<const dev::u32x4*>(O + b * os.b + h * os.h + (int64_t)q * os.s + c);
    const dev::u32x4 dv = *reinterpret_cast<const dev::u32x4*>(dO + b * dos.b + h * dos.h + (int64_t)q * dos.s + c);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      s += bf2f(ov[e] & 0xffff) * bf2f(dv[e] & 0xffff) + bf2f(ov[e] >> 16) * bf2f(dv[e] >> 16);
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) s += __shfl_xor(s, o, 64);
  if (row < rows && t % LPR == 0) delta[row] = s;
}

// dQ: one workgroup = NW waves x 32 query rows of one (batch, q head); S^T and dP^T with the
// query on the lane (as the forward), dQ^T += K^T · dS^T. NW = 8 pairs two waves per SIMD.
template <int D, bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW) void fa_bwd_dq_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    uint16_t* __restrict__ dQ, int Sq, int Sk, int Hq, int Hkv, Strides qs, Strides ks, Strides vs, Strides dos,
    Strides dqs, float scale_log2, float scale, int nqb) {
  constexpr int KS = D / 16, NT = D / 32, BQ = 32 * NW;
  // [stage][K (row reads for S^T, transposed reads for dQ), V (row reads for dP^T)]
  __shared__ __attribute__((aligned(16))) uint8_t KVs[2][2][kBK * D * 2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 5;
  const int bh = blockIdx.y, b = bh / Hq, h = bh % Hq, hk = h / (Hq / Hkv);
  const uint16_t* Kb = K + b * ks.b + hk * ks.h;
  const uint16_t* Vb = V + b * vs.b + hk * vs.h;
  // causal: query blocks (nqb - 1 - x, x) per workgroup, as the forward
  const int npass = CAUSAL && (int)blockIdx.x != nqb - 1 - (int)blockIdx.x ? 2 : 1;
#pragma unroll 1
  for (int pass = 0; pass < npass; ++pass) {
    const int qb = CAUSAL ? (pass == 0 ? nqb - 1 - (int)blockIdx.x : (int)blockIdx.x) : (int)blockIdx.x;
    const int q0 = qb * BQ, qw = q0 + 32 * w;
    const int qrow = qw + (lane & 31);
    const bool ok = qrow < Sq;
    bf16x8 qf[KS], dof[KS];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      qf[s2] = ok ? *reinterpret_cast<const bf16x8*>(Q + b * qs.b + h * qs.h + (int64_t)qrow * qs.s + 16 * s2 + 8 * g)
                  : bf16x8{};
      dof[s2] = ok ? *reinterpret_cast<const bf16x8*>(dO + b * dos.b + h * dos.h + (int64_t)qrow * dos.s + 16 * s2 + 8 * g)
                   : bf16x8{};
    }
    const float lse = ok ? LSE[(int64_t)bh * Sq + qrow] : 0.f;
    const float dl = ok ? delta[(int64_t)bh * Sq + qrow] : 0.f;
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[n][i] = 0.f;
    const int kend = CAUSAL ? min(Sk, q0 + BQ) : Sk;
    const int ntiles = (kend + kBK - 1) / kBK;
    dma_tile<D, NW>(Kb, ks.s, 0, Sk, KVs[0][0], w, lane);
    dma_tile<D, NW>(Vb, vs.s, 0, Sk, KVs[0][1], w, lane);
    for (int j = 0; j < ntiles; ++j) {
      const int k0 = j * kBK;
      dma_barrier();
      if (j + 1 < ntiles) {
        dma_tile<D, NW>(Kb, ks.s, k0 + kBK, Sk, KVs[(j + 1) & 1][0], w, lane);
        dma_tile<D, NW>(Vb, vs.s, k0 + kBK, Sk, KVs[(j + 1) & 1][1], w, lane);
      }
      const uint8_t* Kt = KVs[j & 1][0];
      const uint8_t* Vt = KVs[j & 1][1];
      if (!CAUSAL || k0 <= qw + 31) {
        const bool masked = k0 + kBK > Sk || (CAUSAL && k0 + kBK - 1 > qw);  // wave-uniform
        // one 32-key half at a time keeps S^T / dP^T at 32 live registers
#pragma unroll 1
        for (int t = 0; t < 2; ++t) {
          f32x16 sc, dp;
#pragma unroll
          for (int i = 0; i < 16; ++i) sc[i] = dp[i] = 0.f;
#pragma unroll
          for (int s2 = 0; s2 < KS; ++s2) {
            sc = mfma32(ld_rowfrag<D>(Kt, 32 * t + (lane & 31), s2, lane), qf[s2], sc);
            dp = mfma32(ld_rowfrag<D>(Vt, 32 * t + (lane & 31), s2, lane), dof[s2], dp);
          }
          // dS^T = P^T (dP^T - delta), P^T = exp2(S^T c - lse); the softmax scale of dS folds into the end
          // last visible key of this lane's row, relative to the half tile (no limit off the boundary)
          const int lim = masked ? (CAUSAL ? min(qrow, Sk - 1) : Sk - 1) - k0 - 32 * t : (1 << 30);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float p = __builtin_amdgcn_exp2f(fmaf(sc[i], scale_log2, -lse));
            if (kappa(g, i & 7) + 16 * (i >> 3) > lim) p = 0.f;
            sc[i] = p * (dp[i] - dl);
          }
          bf16x8 sf[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            uint32_t pk[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) pk[e] = dev::pack_bf16x2(sc[8 * hh + 2 * e], sc[8 * hh + 2 * e + 1]);
            sf[hh] = __builtin_bit_cast(bf16x8, pk);
          }
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = mfma32(ld_trfrag<D>(Kt, 32 * t + 16 * hh, 32 * n, lane), sf[hh], acc[n]);
        }
      }
    }
    lds_barrier();  // (causal pairs) every wave is done with the stages before the next pass refills them
    if (ok) {
      uint16_t* out = dQ + b * dqs.b + h * dqs.h + (int64_t)qrow * dqs.s;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint2 pk;
          pk.x = dev::pack_bf16x2(acc[n][4 * q] * scale, acc[n][4 * q + 1] * scale);
          pk.y = dev::pack_bf16x2(acc[n][4 * q + 2] * scale, acc[n][4 * q + 3] * scale);
          *reinterpret_cast<uint2*>(out + 32 * n + 4 * g + 8 * q) = pk;
        }
    }
  }
}

// dK, dV: one workgroup = 32·KW keys of one (batch, kv head), 8 waves in NG = 8 / KW groups of KW.
// KW = 8 (D = 64, Sk <= 256: ViT's 197 tokens): ONE 256-key block and one group, so a (batch,
// head) is one workgroup that reads each Q / dO tile once and needs no cross-group reduction.
// Wave (group G, index wq) owns keys k0 + 32 wq .. +31; the groups split the (query head of the
// GQA group, 32-row query tile) work items (G takes items G, G + NG, ...), so two waves share each
// SIMD, and sum their dK^T / dV^T accumulators through LDS at the end. KW = 4 (128-key blocks) is
// the default; KW = 2 balanced causal work better (twice as many half-size blocks) but re-read
// every Q / dO tile per 64 keys: Llama-shape fwd+bwd 1.30 vs 1.16 ms (r2), so it was dropped. Per item: S = Q·K^T and
// dP = dO·V^T with the KEY on the lane (K fragments in registers, the V block in LDS), then
// dV^T += dO^T·P and dK^T += Q^T·dS with P / dS as the B operands straight from their
// accumulators. Q / dO / lse / delta tiles go global -> LDS by LDS-DMA (no VGPR staging), two
// stages per group: item k + 1 is in flight while item k is computed; one barrier per item.
// Registers: K 32 + dK^T 64 + dV^T 64 + S, dP 32 (D = 128) stay under the 256 of two waves/SIMD.
//
// FQ (KW = 8 only: every key of the head is in this workgroup) also produces dQ, so the separate
// dQ pass — a second read of Q, K, V, dO and a second S / dP evaluation — is skipped: each item's
// dS (bf16, [32 queries][256 keys]) goes to one of two LDS buffers next to K^T ([64][256], staged
// once from the K registers), and after the NEXT item's barrier (no extra one) every wave computes
// one 16 x 16 tile of that item's dQ^T = K^T · dS^T on mfma_f32_16x16x32_bf16 over all 256 keys
// (d = 16 (w & 3).., q = 16 (w >> 2)..): no cross-wave reduction, no atomics. Both LDS images are [row][256] bf16 with the 16-B chunk index XOR'd by
// row & 15, so the 16 rows a b128 lane group reads sit in 16 distinct bank groups.
// FQ with dbp: the packed qkv projection's bias gradient too ([B][3][H][D] partials, the host sums
// the batches): Σ dQ from the dQ tiles, Σ dV from the dV^T accumulators after they are stored,
// Σ dK = 0 exactly (Σ_k dS[q][k] = δ_q - δ_q) — the separate pass re-read all of dQKV (r5: 62.5 us
// per ViT-L layer against +12 us here).
template <int D, bool CAUSAL, int KW, bool FQ = false, int NG_ = 8 / KW>
__global__ __launch_bounds__(64 * KW * NG_, 8 / (KW * NG_)) void fa_bwd_dkdv_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int Sq, int Sk, int Hq, int Hkv, Strides qs, Strides ks,
    Strides vs, Strides dos, Strides dks, Strides dvs, float scale_log2, float scale, int nsplit,
    float* __restrict__ wsk, float* __restrict__ wsv, uint16_t* __restrict__ dQo, Strides dqs,
    float* __restrict__ dbp) {
  constexpr int NG = NG_, BK = 32 * KW;             // groups; keys per workgroup
  constexpr int KS = D / 16, NT = D / 32, QB = 32;  // query rows per work item
  constexpr int TILE = QB * D * 2;                  // bytes of one Q (or dO) tile
  constexpr int STAGE = 2 * TILE + 2 * QB * 4;      // Q, dO, lse, delta
  constexpr int VBLK = BK * D * 2;                  // the workgroup's V rows
  // rows per 1-KB DMA instruction; instructions per tile; per wave (KW = 8 at D = 64: half the
  // waves issue one each)
  constexpr int RPI = 512 / D, NIT = QB / RPI, NI = NIT >= KW ? NIT / KW : 1;
  constexpr int ACC = NT * 16 * 64;                 // floats of one wave's dK^T (or dV^T)
  static_assert(KW >= 2 && 8 % (KW * NG) == 0 && NIT % NI == 0 && (NIT < KW || NI * KW == NIT), "wave split");
  static_assert((NG - 1) * KW * ACC * 4 <= VBLK + 2 * NG * STAGE, "group reduction must fit the LDS");
  static_assert(!FQ || (KW == 8 && D == 64 && !CAUSAL), "fused dQ: one 256-key block, D = 64, non-causal");
  constexpr int DSB = QB * BK * 2;                   // (FQ) one dS [QB][BK] bf16 buffer
  constexpr int FQB = FQ ? D * BK * 2 + 2 * DSB : 0;  // K^T [D][BK] + two dS buffers
  __shared__ __attribute__((aligned(16))) uint8_t smem[VBLK + 2 * NG * STAGE + FQB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wq = w % KW, G = w / KW, g = lane >> 5;
  // blockIdx.x = (batch, kv head, head split), blockIdx.y = key block: the dispatcher walks x
  // first, so every workgroup of key block 0 (the heaviest under a causal mask) starts first.
  // nsplit > 1 splits the query heads of a GQA group over workgroups (fp32 partial dK/dV summed
  // by fa_dkdv_sum_kernel): 4x the workgroups, each a quarter of the work, so the heavy-first
  // dispatch balances the CUs (one workgroup per (key block, kv head) left a 2x work spread).
  const int split = (int)blockIdx.x % nsplit, bhk = (int)blockIdx.x / nsplit;
  const int b = bhk / Hkv, hk = bhk % Hkv, grp = Hq / Hkv, hpw = grp / nsplit;
  const int kb = (int)blockIdx.y;
  const int k0 = kb * BK, kw = k0 + 32 * wq, krow = kw + (lane & 31);
  uint8_t* Vblk = smem;
  {  // V rows [k0, k0 + BK) -> LDS (rows past Sk read row Sk - 1; their P, dS are masked to 0)
    constexpr int VI = BK / RPI / (KW * NG);  // per wave
    static_assert(VI * KW * NG * RPI == BK, "the V block must split evenly over the waves");
    const uint16_t* Vb = V + b * vs.b + hk * vs.h;
#pragma unroll
    for (int i = 0; i < VI; ++i) {
      const int ins = w * VI + i, r = ins * RPI + lane / (D / 8);
      const int c = uswz<D>(r, lane % (D / 8));
      const int64_t row = min(k0 + r, Sk - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + row * vs.s + c * 8), (lds_ptr_t)(Vblk + ins * 1024), 16, 0,
                                       0);
    }
  }
  bf16x8 kf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    kf[s] = krow < Sk ? *reinterpret_cast<const bf16x8*>(K + b * ks.b + hk * ks.h + (int64_t)krow * ks.s + 16 * s + 8 * g)
                      : bf16x8{};
  // (FQ) byte offset of element [row][col] of a [row][BK] bf16 LDS image, chunk-swizzled
  auto fq_off = [](int row, int col) { return row * (BK * 2) + (((col >> 3) ^ (row & 15)) << 4) + (col & 7) * 2; };
  uint8_t* KT = smem + VBLK + 2 * NG * STAGE;
  uint8_t* DSl = KT + D * BK * 2;
  const int kl = 32 * wq + (lane & 31);  // this lane's key within the block
  if constexpr (FQ) {  // K^T image from the K registers (zero rows past Sk come along)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u32x4 kv = __builtin_bit_cast(u32x4, kf[s]);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<uint16_t*>(KT + fq_off(16 * s + 8 * g + e, kl)) = (uint16_t)(kv[e >> 1] >> (16 * (e & 1)));
    }
  }
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int i = 0; i < 16; ++i) adk[n][i] = adv[n][i] = 0.f;
  const int qstart = CAUSAL ? (k0 / QB) * QB : 0;
  const int nqt = (Sq - qstart + QB - 1) / QB;
  const int total = hpw * nqt, niter = (total + NG - 1) / NG;
  uint8_t* gsm = smem + VBLK + G * 2 * STAGE;
  auto issue = [&](int it, int st) {  // rows past Sq read row Sq - 1 (masked below)
    const int h = hk * grp + split * hpw + it / nqt, qt0 = qstart + (it % nqt) * QB;
    uint8_t* S = gsm + st * STAGE;
    const uint16_t* Qb = Q + b * qs.b + h * qs.h;
    const uint16_t* Db = dO + b * dos.b + h * dos.h;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int ins = wq * NI + i, r = ins * RPI + lane / (D / 8);
      if (NIT < KW && ins >= NIT) break;  // (wave-uniform)
      const int c = uswz<D>(r, lane % (D / 8));  // the logical chunk that lands at this lane's slot
      const int64_t row = min(qt0 + r, Sq - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Qb + row * qs.s + c * 8), (lds_ptr_t)(S + ins * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Db + row * dos.s + c * 8), (lds_ptr_t)(S + TILE + ins * 1024), 16,
                                       0, 0);
    }
    if (wq < 2) {  // 32 lse / delta values: lanes 32..63 duplicate the last row (harmless, in bounds)
      const float* src = (wq == 0 ? LSE : delta) + ((int64_t)b * Hq + h) * Sq + min(qt0 + (lane & 31), Sq - 1);
      if (lane < 32)
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(S + 2 * TILE + wq * QB * 4), 4, 0, 0);
    }
  };
  // (FQ, dbp) the qkv bias gradient's partial of this (batch, head): Σ dQ from the dQ tiles, Σ dV
  // from the dV^T accumulators at the end, Σ dK = 0 (Σ_k dS = 0: a per-query constant added to the
  // logits changes nothing)
  float qsum[4] = {0.f, 0.f, 0.f, 0.f};
  // (FQ) dQ of item itq from its dS buffer: wave w owns the 16 x 16 tile d = 16 (w & 3).., q = 16 (w >> 2)..
  auto dq_tile = [&](int itq, const uint8_t* dsb) {
    const int d0 = 16 * (w & 3), q0 = 16 * (w >> 2), r16 = lane & 15, kq = lane >> 4;
    f32x4v aq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int col = 32 * s + 8 * kq;
      aq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(KT + fq_off(d0 + r16, col)),
                                                   *reinterpret_cast<const bf16x8*>(dsb + fq_off(q0 + r16, col)), aq,
                                                   0, 0, 0);
    }
    // lane: dQ[query q0 + r16][d0 + 4 kq .. + 3]
    const int h = hk * grp + split * hpw + itq / nqt, qrow = qstart + (itq % nqt) * QB + q0 + r16;
    if (qrow < Sq) {
      uint2 o;
      o.x = dev::pack_bf16x2(aq[0] * scale, aq[1] * scale);
      o.y = dev::pack_bf16x2(aq[2] * scale, aq[3] * scale);
      *reinterpret_cast<uint2*>(dQo + b * dqs.b + h * dqs.h + (int64_t)qrow * dqs.s + d0 + 4 * kq) = o;
#pragma unroll
      for (int j = 0; j < 4; ++j) qsum[j] += aq[j] * scale;
    }
  };
  if (G < total) issue(G, 0);
  for (int k = 0; k < niter; ++k) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int it = G + NG * k;
    if (it + NG < total) issue(it + NG, (k + 1) & 1);  // into the stage item k - 1 was computed from
    // (FQ: one group, non-causal, so every item is computed) item k - 1's dQ: its dS landed before
    // the barrier above; the buffer is rewritten at item k + 1, after the next barrier
    if constexpr (FQ)
      if (k > 0) dq_tile(it - 1, DSl + ((k - 1) & 1) * DSB);
    const int qt0 = qstart + (it % nqt) * QB;
    if (it < total && (!CAUSAL || qt0 + QB - 1 >= kw)) {
      const uint8_t* Qt = gsm + (k & 1) * STAGE;
      const uint8_t* Dt = Qt + TILE;
      const float* lse_s = reinterpret_cast<const float*>(Qt + 2 * TILE);
      const float* dl_s = lse_s + QB;
      f32x16 sc, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = dp[i] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        sc = mfma32(ld_rowfrag<D>(Qt, lane & 31, s, lane), kf[s], sc);
        dp = mfma32(ld_rowfrag<D>(Dt, lane & 31, s, lane), ld_rowfrag<D>(Vblk, 32 * wq + (lane & 31), s, lane), dp);
      }
      // element i: query qt0 + kappa(g, i&7) + 16(i>>3), key krow; visible iff lo <= ql < hi
      const int lo = krow >= Sk ? (1 << 30) : (CAUSAL ? krow - qt0 : -1), hi = Sq - qt0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = kappa(g, i & 7) + 16 * (i >> 3);
        float p = __builtin_amdgcn_exp2f(fmaf(sc[i], scale_log2, -lse_s[ql]));
        if (ql < lo || ql >= hi) p = 0.f;
        sc[i] = p;
        dp[i] = p * (dp[i] - dl_s[ql]);
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        uint32_t pk[4], dk4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pk[e] = dev::pack_bf16x2(sc[8 * hh + 2 * e], sc[8 * hh + 2 * e + 1]);
          dk4[e] = dev::pack_bf16x2(dp[8 * hh + 2 * e], dp[8 * hh + 2 * e + 1]);
        }
        const bf16x8 pf = __builtin_bit_cast(bf16x8, pk), sf = __builtin_bit_cast(bf16x8, dk4);
        if constexpr (FQ) {  // dS[query][key] -> LDS (element 8 hh + 2 e + j: query kappa(g, 2 e + j) + 16 hh)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              *reinterpret_cast<uint16_t*>(DSl + (k & 1) * DSB + fq_off(kappa(g, 2 * e + j) + 16 * hh, kl)) =
                  (uint16_t)(dk4[e] >> (16 * j));
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          adv[n] = mfma32(ld_trfrag<D>(Dt, 16 * hh, 32 * n, lane), pf, adv[n]);
          adk[n] = mfma32(ld_trfrag<D>(Qt, 16 * hh, 32 * n, lane), sf, adk[n]);
        }
      }
    }
  }
  if constexpr (FQ) {  // the last item's dQ
    if (niter > 0) {
      lds_barrier();
      dq_tile(niter - 1, DSl + ((niter - 1) & 1) * DSB);
    }
  }
  // groups 1..NG-1 hand their partial dK^T, then dV^T, to group 0 through the (now idle) LDS
  float* red = reinterpret_cast<float*>(smem) + lane;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    f32x16* acc = pass == 0 ? adk : adv;
    if (G > 0) {
      float* r = red + ((G - 1) * KW + wq) * ACC;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) r[(n * 16 + i) * 64] = acc[n][i];
    }
    __syncthreads();
    if (G == 0) {
      const float* r = red + wq * ACC;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float v = 0.f;
#pragma unroll
          for (int gg = 1; gg < NG; ++gg) v += r[(gg - 1) * KW * ACC + (n * 16 + i) * 64];
          acc[n][i] += v;
        }
    }
  }
  const bool rows_out = G == 0 && krow < Sk;  // (FQ with dbp: every lane goes on to the sums below)
  if (!rows_out && !(FQ && dbp)) return;
  if (rows_out && nsplit > 1) {  // fp32 partials [split][B][Sk][Hkv][D], summed (and dK scaled) later
    const int64_t base = ((((int64_t)split * (gridDim.x / nsplit) + bhk) / Hkv * Sk + krow) * Hkv + hk) * D;
    float* pk = wsk + base;
    float* pv = wsv + base;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *reinterpret_cast<float4*>(pk + 32 * n + 4 * g + 8 * q) =
            make_float4(adk[n][4 * q], adk[n][4 * q + 1], adk[n][4 * q + 2], adk[n][4 * q + 3]);
        *reinterpret_cast<float4*>(pv + 32 * n + 4 * g + 8 * q) =
            make_float4(adv[n][4 * q], adv[n][4 * q + 1], adv[n][4 * q + 2], adv[n][4 * q + 3]);
      }
  } else if (rows_out) {
    uint16_t* ok = dK + b * dks.b + hk * dks.h + (int64_t)krow * dks.s;
    uint16_t* ov = dV + b * dvs.b + hk * dvs.h + (int64_t)krow * dvs.s;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint2 a, c;
        a.x = dev::pack_bf16x2(adk[n][4 * q] * scale, adk[n][4 * q + 1] * scale);
        a.y = dev::pack_bf16x2(adk[n][4 * q + 2] * scale, adk[n][4 * q + 3] * scale);
        c.x = dev::pack_bf16x2(adv[n][4 * q], adv[n][4 * q + 1]);
        c.y = dev::pack_bf16x2(adv[n][4 * q + 2], adv[n][4 * q + 3]);
        *reinterpret_cast<uint2*>(ok + 32 * n + 4 * g + 8 * q) = a;
        *reinterpret_cast<uint2*>(ov + 32 * n + 4 * g + 8 * q) = c;
      }
  }
  if constexpr (FQ) {
    if (dbp) {
      static_assert(NT * 16 == 32, "the key-sum butterfly below is written for D = 64");
      // Σ_keys dV: halving butterfly over lane bits 0..4, in place on the (stored) accumulators,
      // value j = adv[j >> 4][j & 15]: each exchange trades half the live values, so lane l ends with
      // the 32-lane total of value index l & 31 in adv[0][0] (31 shuffles; keys past Sk hold zeros)
#pragma unroll
      for (int st = 0, width = 16; st < 5; ++st, width >>= 1) {
        const int o = 16 >> st;
        const bool hi = lane & o;
#pragma unroll
        for (int i = 0; i < width; ++i) {
          const float lo_v = adv[i >> 4][i & 15], hi_v = adv[(i + width) >> 4][(i + width) & 15];
          const float recv = __shfl_xor(hi ? lo_v : hi_v, o, 64);
          adv[i >> 4][i & 15] = (hi ? hi_v : lo_v) + recv;
        }
      }
      // Σ_queries dQ: the 16 lanes r16 = lane & 15 of a dQ column set; bits 3, 2 halve the 4 values
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool hi = lane & 8;
        const float recv = __shfl_xor(hi ? qsum[i] : qsum[i + 2], 8, 64);
        qsum[i] = (hi ? qsum[i + 2] : qsum[i]) + recv;
      }
      {
        const bool hi = lane & 4;
        const float recv = __shfl_xor(hi ? qsum[0] : qsum[1], 4, 64);
        qsum[0] = (hi ? qsum[1] : qsum[0]) + recv;
      }
      qsum[0] += __shfl_xor(qsum[0], 2, 64);
      qsum[0] += __shfl_xor(qsum[0], 1, 64);
      float* rb = reinterpret_cast<float*>(smem);  // [8][D] per-wave dV sums, [2][D] dQ sums (LDS idle)
      {
        const int j = lane & 31, n = j >> 4, i = j & 15;
        rb[w * D + 32 * n + 8 * (i >> 2) + 4 * g + (i & 3)] = adv[0][0];
      }
      // lane (kq = lane >> 4) holds dQ column 16 (w & 3) + 4 kq + 2·(bit 3) + (bit 2) of query half w >> 2
      if ((lane & 3) == 0)
        rb[(8 + (w >> 2)) * D + 16 * (w & 3) + 4 * (lane >> 4) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1)] = qsum[0];
      __syncthreads();
      if (tid < 3 * D) {
        const int t = tid / D, d = tid - t * D;
        float sum = 0.f;
        if (t == 0) {
          sum = rb[8 * D + d] + rb[9 * D + d];
        } else if (t == 2) {
#pragma unroll
          for (int ww = 0; ww < 8; ++ww) sum += rb[ww * D + d];
        }
        dbp[((int64_t)b * 3 + t) * Hq * D + (int64_t)hk * D + d] = sum;
      }
    }
  }
}

// dK = scale · sum_s wsk[s], dV = sum_s wsv[s] (fp32 head-split partials, [nsplit][B·Sk·Hkv·D]);
// 8 elements per thread, output [B, Sk, Hkv, D] contiguous
__global__ __launch_bounds__(256) void fa_dkdv_sum_kernel(const float* __restrict__ wsk, const float* __restrict__ wsv,
                                                          uint16_t* __restrict__ dK, uint16_t* __restrict__ dV,
                                                          int64_t n8, int nsplit, float scale) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float k[8] = {0, 0, 0, 0, 0, 0, 0, 0}, v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int sp = 0; sp < nsplit; ++sp) {
    const float4* a = reinterpret_cast<const float4*>(wsk + ((int64_t)sp * n8 + i) * 8);
    const float4* c = reinterpret_cast<const float4*>(wsv + ((int64_t)sp * n8 + i) * 8);
    const float4 a0 = a[0], a1 = a[1], c0 = c[0], c1 = c[1];
    k[0] += a0.x; k[1] += a0.y; k[2] += a0.z; k[3] += a0.w; k[4] += a1.x; k[5] += a1.y; k[6] += a1.z; k[7] += a1.w;
    v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w; v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
  }
  uint4 ko, vo;
  ko.x = dev::pack_bf16x2(k[0] * scale, k[1] * scale);
  ko.y = dev::pack_bf16x2(k[2] * scale, k[3] * scale);
  ko.z = dev::pack_bf16x2(k[4] * scale, k[5] * scale);
  ko.w = dev::pack_bf16x2(k[6] * scale, k[7] * scale);
  vo.x = dev::pack_bf16x2(v[0], v[1]);
  vo.y = dev::pack_bf16x2(v[2], v[3]);
  vo.z = dev::pack_bf16x2(v[4], v[5]);
  vo.w = dev::pack_bf16x2(v[6], v[7]);
  reinterpret_cast<uint4*>(dK)[i] = ko;
  reinterpret_cast<uint4*>(dV)[i] = vo;
}

Strides strides_of(const at::Tensor& t) { return Strides{t.stride(0), t.stride(1), t.stride(2)}; }

void check_bshd(const at::Tensor& t, const char* name, int64_t D) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4, "flash_attn: ", name,
              " must be a bf16 [B, S, H, D] GPU tensor");
  TORCH_CHECK(t.size(3) == D && t.stride(3) == 1, "flash_attn: ", name, " must have a contiguous last dim of ", D);
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "flash_attn: ", name, " needs 16-B aligned rows");
}

}  // namespace

// q [B, Sq, Hq, D], k / v [B, Sk, Hkv, D] -> (o [B, Sq, Hq, D], lse [B, Hq, Sq] fp32, log2 domain)
std::vector<at::Tensor> flash_attn_forward(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal,
                                           double scale) {
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "flash_attn: head dim 64 or 128");
  check_bshd(q, "q", D);
  check_bshd(k, "k", D);
  check_bshd(v, "v", D);
  const int64_t B = q.size(0), Sq = q.size(1), Hq = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.sizes() == v.sizes() && k.size(0) == B && Hq % Hkv == 0, "flash_attn: q/k/v shape mismatch");
  TORCH_CHECK(!causal || Sq == Sk, "flash_attn: causal needs Sq == Sk");
  TORCH_CHECK(Sq > 0 && Sk > 0 && B * Hq < 65536 && Sq < (1 << 30), "flash_attn: bad size");
  auto o = at::empty({B, Sq, Hq, D}, q.options());
  auto lse = at::empty({B, Hq, Sq}, q.options().dtype(at::kFloat));
  auto stream = c10::hip::getCurrentHIPStream(q.device().index()).stream();
  // 8 waves (256 query rows) per workgroup; 4 when 256-row blocks would leave CUs idle
  const int64_t wg8 = ((Sq + 255) / 256) * B * Hq;
  const int nw = wg8 >= 256 ? 8 : 4;
  const int nqb = (int)((Sq + 32 * nw - 1) / (32 * nw));
  const dim3 grid((unsigned)(causal ? (nqb + 1) / 2 : nqb), (unsigned)(B * Hq));
  const float sl2 = (float)(scale * 1.4426950408889634);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(64 * nw), 0, stream, reinterpret_cast<const uint16_t*>(q.data_ptr()),
                       reinterpret_cast<const uint16_t*>(k.data_ptr()), reinterpret_cast<const uint16_t*>(v.data_ptr()),
                       reinterpret_cast<uint16_t*>(o.data_ptr()), lse.data_ptr<float>(), (int)Sq, (int)Sk, (int)Hq,
                       (int)Hkv, strides_of(q), strides_of(k), strides_of(v), strides_of(o), sl2, nqb);
    XDDP_HIP_CHECK(hipGetLastError());
  };
#define XDDP_FA(D_, C_) \
  if (nw == 8) go(fa_fwd_kernel<D_, C_, 8>); else go(fa_fwd_kernel<D_, C_, 4>)
  // short non-causal D = 64 heads (ViT: 197 keys) stage all of K / V at once (r3 A/B vs the
  // double-buffered tile loop: profiles/r3_flash_whole_kv_ab.txt)
  const bool whole = D == 64 && !causal && Sk <= 4 * kBK;
  if (D == 128) { if (causal) { XDDP_FA(128, true); } else { XDDP_FA(128, false); } }
  else if (whole) { if (nw == 8) go(fa_fwd_kernel<64, false, 8, true>); else go(fa_fwd_kernel<64, false, 4, true>); }
  else { if (causal) { XDDP_FA(64, true); } else { XDDP_FA(64, false); } }
#undef XDDP_FA
  return {o, lse};
}

// -> (dq, dk, dv) in the layouts of q, k, v ([B, S, H, D] contiguous)
std::vector<at::Tensor> flash_attn_backward(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                            const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                                            bool causal, double scale, const c10::optional<at::Tensor>& dq_out,
                                            const c10::optional<at::Tensor>& dk_out,
                                            const c10::optional<at::Tensor>& dv_out,
                                            const c10::optional<at::Tensor>& bias_like) {
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "flash_attn: head dim 64 or 128");
  check_bshd(q, "q", D);
  check_bshd(k, "k", D);
  check_bshd(v, "v", D);
  check_bshd(o, "o", D);
  check_bshd(dout, "dout", D);
  const int64_t B = q.size(0), Sq = q.size(1), Hq = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && lse.is_contiguous() &&
                  lse.numel() == B * Hq * Sq && lse.scalar_type() == at::kFloat,
              "flash_attn backward: shape mismatch");
  // optional caller-provided outputs (e.g. strided views of one packed [B, S, 3, H, D] gradient, so
  // a fused qkv projection gets its gradient without a gather)
  auto out_or = [&](const c10::optional<at::Tensor>& o_, const at::Tensor& like, int64_t S_, int64_t H_) {
    if (o_.has_value() && o_->defined()) {
      check_bshd(*o_, "dq/dk/dv out", D);
      TORCH_CHECK(o_->sizes() == like.sizes(), "flash_attn backward: output shape mismatch");
      return *o_;
    }
    return at::empty({B, S_, H_, D}, like.options());
  };
  auto dq = out_or(dq_out, q, Sq, Hq);
  auto dk = out_or(dk_out, k, Sk, Hkv);
  auto dv = out_or(dv_out, v, Sk, Hkv);
  auto delta = at::empty({B, Hq, Sq}, q.options().dtype(at::kFloat));
  auto stream = c10::hip::getCurrentHIPStream(q.device().index()).stream();
  const int64_t rows = B * Hq * Sq;
  {  // delta: D / 8 lanes per query row
    auto go = [&](auto kern, int lpr) {
      const int64_t threads = rows * lpr;
      hipLaunchKernelGGL(kern, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream,
                         reinterpret_cast<const uint16_t*>(o.data_ptr()),
                         reinterpret_cast<const uint16_t*>(dout.data_ptr()), delta.data_ptr<float>(), rows, (int)Sq,
                         (int)Hq, strides_of(o), strides_of(dout));
      XDDP_HIP_CHECK(hipGetLastError());
    };
    if (D == 128) go(fa_bwd_pre_kernel<128>, 16); else go(fa_bwd_pre_kernel<64>, 8);
  }
  const float sl2 = (float)(scale * 1.4426950408889634), sc = (float)scale;
  // short non-causal D = 64 sequences (ViT): the whole key range in one 8-wave block, which then
  // also computes dQ (r2: measured faster than two 128-key blocks + the separate dQ pass)
  const int kwv = D == 64 && !causal && Sk <= 256 ? 8 : 4;
  const bool fused_dq = kwv == 8;
  if (!fused_dq) {
    const int64_t wg8 = ((Sq + 255) / 256) * B * Hq;
    const int nw = wg8 >= 256 ? 8 : 4;
    const int nqb = (int)((Sq + 32 * nw - 1) / (32 * nw));
    const dim3 grid((unsigned)(causal ? (nqb + 1) / 2 : nqb), (unsigned)(B * Hq));
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(64 * nw), 0, stream, reinterpret_cast<const uint16_t*>(q.data_ptr()),
                         reinterpret_cast<const uint16_t*>(k.data_ptr()), reinterpret_cast<const uint16_t*>(v.data_ptr()),
                         reinterpret_cast<const uint16_t*>(dout.data_ptr()), lse.data_ptr<float>(),
                         delta.data_ptr<float>(), reinterpret_cast<uint16_t*>(dq.data_ptr()), (int)Sq, (int)Sk,
                         (int)Hq, (int)Hkv, strides_of(q), strides_of(k), strides_of(v), strides_of(dout),
                         strides_of(dq), sl2, sc, nqb);
      XDDP_HIP_CHECK(hipGetLastError());
    };
#define XDDP_FA(D_, C_) \
  if (nw == 8) go(fa_bwd_dq_kernel<D_, C_, 8>); else go(fa_bwd_dq_kernel<D_, C_, 4>)
    if (D == 128) { if (causal) { XDDP_FA(128, true); } else { XDDP_FA(128, false); } }
    else { if (causal) { XDDP_FA(64, true); } else { XDDP_FA(64, false); } }
#undef XDDP_FA
  }
  {
    const int nkb = (int)((Sk + 32 * kwv - 1) / (32 * kwv));
    // GQA head split for causal attention (balance, see the kernel)
    const int grp = (int)(Hq / Hkv);
    // D = 128: one 4-wave group per workgroup, two workgroups per CU (NG = 1; r5: the per-item
    // barrier of a two-group workgroup kept both groups' softmax phases in step, 1,435 vs 1,345 us
    // at Llama B2 S4096). Causal: the smallest GQA head split that still gives two rounds of
    // workgroups (heavy key blocks first, so the second round evens out the causal 2x work spread)
    // — fewer fp32 partials to write and sum: B2 splits in two (1,311 vs 1,345 us four-way; one-way,
    // a single round: 1,611), B1 (the Llama bench) in four (18,190 / 18,229 tok/s vs 17,629 /
    // 17,658 two-way)
    static const int cus = [] {
      int dev = 0, v = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
      return v > 0 ? v : 256;
    }();
    const int ng = D == 128 && kwv == 4 ? 1 : 8 / kwv;
    int nsplit = 1;
    if (causal && ng == 1) {
      nsplit = grp;
      for (int sp = 1; sp < grp; sp *= 2)
        if (grp % sp == 0 && B * Hkv * sp * nkb >= 4LL * cus) {
          nsplit = sp;
          break;
        }
    } else if (causal) {
      nsplit = grp;
    }
    if (nsplit < 1 || grp % nsplit != 0) nsplit = 1;
    at::Tensor wsk, wsv;
    if (nsplit > 1) {
      wsk = at::empty({nsplit, B, Sk, Hkv, D}, q.options().dtype(at::kFloat));
      wsv = at::empty({nsplit, B, Sk, Hkv, D}, q.options().dtype(at::kFloat));
    }
    const dim3 grid((unsigned)(B * Hkv * nsplit), (unsigned)nkb);
    // bias_like (the fused-dQ path: one workgroup per (batch, head), non-causal, every key in it): the
    // column sums of dQ, dK, dV ([3][Hq][D], the packed qkv projection's bias gradient) from the kernel
    const bool want_db =
        bias_like.has_value() && bias_like->defined() && fused_dq && Hq == Hkv && nsplit == 1 && nkb == 1;
    if (want_db)
      TORCH_CHECK(bias_like->numel() == 3 * Hq * D, "flash_attn backward: bias_like must hold 3·H·D elements");
    at::Tensor dbp = want_db ? at::empty({B, 3 * Hq * D}, q.options().dtype(at::kFloat)) : at::Tensor();
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(64 * kwv * ng), 0, stream, reinterpret_cast<const uint16_t*>(q.data_ptr()),
                         reinterpret_cast<const uint16_t*>(k.data_ptr()), reinterpret_cast<const uint16_t*>(v.data_ptr()),
                         reinterpret_cast<const uint16_t*>(dout.data_ptr()), lse.data_ptr<float>(),
                         delta.data_ptr<float>(), reinterpret_cast<uint16_t*>(dk.data_ptr()),
                         reinterpret_cast<uint16_t*>(dv.data_ptr()), (int)Sq, (int)Sk, (int)Hq, (int)Hkv, strides_of(q),
                         strides_of(k), strides_of(v), strides_of(dout), strides_of(dk), strides_of(dv), sl2, sc,
                         nsplit, nsplit > 1 ? wsk.data_ptr<float>() : nullptr,
                         nsplit > 1 ? wsv.data_ptr<float>() : nullptr, reinterpret_cast<uint16_t*>(dq.data_ptr()),
                         strides_of(dq), dbp.defined() ? dbp.data_ptr<float>() : nullptr);
      XDDP_HIP_CHECK(hipGetLastError());
    };
    if (D == 128) {
      if (causal) go(fa_bwd_dkdv_kernel<128, true, 4, false, 1>); else go(fa_bwd_dkdv_kernel<128, false, 4, false, 1>);
    }
    else if (kwv == 8) go(fa_bwd_dkdv_kernel<64, false, 8, true>);
    else { if (causal) go(fa_bwd_dkdv_kernel<64, true, 4>); else go(fa_bwd_dkdv_kernel<64, false, 4>); }
    if (nsplit > 1) {  // the split-sum writes dense [B, Sk, Hkv, D]: strided outputs get a copy
      const int64_t n8 = B * Sk * Hkv * D / 8;
      auto dkc = dk.is_contiguous() ? dk : at::empty({B, Sk, Hkv, D}, k.options());
      auto dvc = dv.is_contiguous() ? dv : at::empty({B, Sk, Hkv, D}, v.options());
      hipLaunchKernelGGL(fa_dkdv_sum_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, stream,
                         wsk.data_ptr<float>(), wsv.data_ptr<float>(), reinterpret_cast<uint16_t*>(dkc.data_ptr()),
                         reinterpret_cast<uint16_t*>(dvc.data_ptr()), n8, nsplit, sc);
      XDDP_HIP_CHECK(hipGetLastError());
      if (!dk.is_same(dkc)) dk.copy_(dkc);
      if (!dv.is_same(dvc)) dv.copy_(dvc);
    }
    if (bias_like.has_value()) {  // a 4th output: the bias gradient, or None (not covered: bias_grad)
      at::Tensor db;
      if (want_db) {
        db = at::empty({3 * Hq * D}, bias_like->options());
        colsum_partials(dbp, db);
      }
      return {dq, dk, dv, db};
    }
  }
  return {dq, dk, dv};
}

}  // namespace kernels
}  // namespace xddp
