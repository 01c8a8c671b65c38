// Small GEMMs on f32-input MFMA: the block body shared by k_tgemm / k_tgemm2 (tail.hip) and the
// fused user-tower forward k_user_fwd (adam.hip). Only the TA / TB = 0 / 1 paths contain no
// contractible multiply-add, so the body computes the same bits under either file's fp-contract
// setting for them (adam.hip, -ffp-contract=off, instantiates only those).
#pragma once
#include "dcue_internal.h"

namespace dcue {

// ------------------------------------------------------------ small GEMMs on f32-input MFMA
// C(m,n) = sum_k TA(A(m,k)) TB(B(k,n)) (+ bias[n]) (* [cmask(m,n) > 0]) on v_mfma_f32_16x16x4_f32.
// A workgroup owns a 16 (m) x 64 (n) output block; K is staged through LDS 128 at a time with every
// load of a stage issued at once (these operands are <= 1.2 MB and L2/MALL resident: the cost is
// load latency, so the chain of dependent load rounds is kept to ceil(K/128)). Each wave computes
// one 16x16 tile from the k-major LDS images (conflict-free ds_read_b32). Optional row gathers
// (arow: A rows, brow: B rows along K, cmrow: mask rows) and per-row sums of TA(A) (bias grads).
constexpr int kTgKC = 128;
// AKF: A is k-contiguous (sak == 1); BNF: B is n-contiguous (sbn == 1) -- picks the staging thread
// map that keeps global reads coalesced. All staging addresses are clamped in-range and loaded
// unconditionally (no per-element branch), row gathers resolved before the data loads.
// The block (bx, by) of one GEMM, as a device function: k_tgemm runs it on its own grid, k_tgemm2
// runs two independent GEMMs' blocks in one launch (same arithmetic, so the same bits).
// LDS images: odd pitches, the k-major staging stores hit 64 distinct banks.
struct TgLds {
  float As[kTgKC][17];
  float Bs[kTgKC][81];
};
template <int TA, int TB, int AKF, int BNF>
__device__ __forceinline__ void tgemm_block(const TGemmArgs& g, int bx, int by, TgLds& L, int t) {
  float (*As)[17] = L.As;
  float (*Bs)[81] = L.Bs;
  const int wave = t >> 6, lane = t & 63;
  const int m0 = bx * 16, nb0 = by * 64, n0 = nb0 + 16 * wave;
  const int l16 = lane & 15, kq = lane >> 4;
  const int n = n0 + l16;
  const bool nok = n < g.N;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float rsum = 0.f;
  constexpr int NA = 16 * kTgKC / 256, NB = 64 * kTgKC / 256;  // staged elements per thread
  constexpr int NAR = AKF ? NA : 1;
  // A rows (fixed over K): AKF -> rows (t>>7)+2j, k = t&127; else row t&15, k = (t>>4)+16j
  // Rows m >= M / columns n >= N are clamped onto real data and never stored; only the K tail of
  // the A image is zeroed (a zero A column annihilates whatever finite B value sits beside it).
  long abase[NAR];
#pragma unroll
  for (int j = 0; j < NAR; ++j) {
    const int mc = min(m0 + (AKF ? (t >> 7) + 2 * j : (t & 15)), g.M - 1);
    abase[j] = (g.arow ? g.arow[mc] : mc) * g.sam;
  }
  // B columns: BNF -> column t&63 (fixed), k = (t>>6)+4j; else columns (t>>7)+2j, k = t&127 (fixed)
  const long bcol0 = (long)min(nb0 + (BNF ? (t & 63) : (t >> 7)), g.N - 1) * g.sbn;
  // register-staged K chunks: chunk k0 + kTgKC's loads are issued right after chunk k0 is in LDS,
  // so they fly during its MFMAs (one load latency per GEMM instead of one per chunk)
  float ra[NA], rb[NB];
  auto load = [&](int k0) {
    long brk[BNF ? NB : 1];
#pragma unroll
    for (int j = 0; j < (BNF ? NB : 1); ++j) {
      const int k = min(k0 + (BNF ? (t >> 6) + 4 * j : (t & 127)), g.K - 1);
      brk[j] = (long)(g.brow ? g.brow[k] : k) * g.sbk;
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {  // every load of the stage issued before any is used
      const int k = min(k0 + (AKF ? (t & 127) : (t >> 4) + 16 * j), g.K - 1);
      ra[j] = g.A[abase[AKF ? j : 0] + (long)k * g.sak];
    }
    if constexpr (BNF) {
#pragma unroll
      for (int j = 0; j < NB; ++j) rb[j] = g.B[brk[j] + bcol0];
    } else {
      const float* bp = g.B + brk[0];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int nc = min(nb0 + (t >> 7) + 2 * j, g.N - 1);
        rb[j] = bp[(long)nc * g.sbn];
      }
    }
  };
  load(0);
  for (int k0 = 0; k0 < g.K; k0 += kTgKC) {
    // TA == 2 / TB == 2 affine operands, per column: gathered before the conversion loops (their
    // loads issued together; the acc-finalize branch is uniform, hoisted out of the loop)
    constexpr int NAC = TA == 2 ? NA : 1, NBC = TB == 2 ? NB : 1;
    float amu[NAC], asc[NAC], abt[NAC], bmu[NBC], bsc[NBC], bbt[NBC];
    if constexpr (TA == 2) {
      int kcs[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) kcs[j] = min(k0 + (AKF ? (t & 127) : (t >> 4) + 16 * j), g.K - 1);
      if (g.abn.acc) {  // train: BatchNorm of A's columns finalized from its accumulators
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          const BnChan st = bn_chan_train(g.abn.acc, g.K, kcs[j], g.abn.count, g.abn.inv_count);
          amu[j] = st.mean;
          asc[j] = g.abn.gamma[kcs[j]] * st.invstd;
          abt[j] = g.abn.beta[kcs[j]];
        }
      } else {
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          amu[j] = g.amean[kcs[j]];
          asc[j] = g.aa[kcs[j]];
          abt[j] = g.abeta[kcs[j]];
        }
      }
    }
    if constexpr (TB == 2) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int nc = min(nb0 + (BNF ? (t & 63) : (t >> 7) + 2 * j), g.N - 1);
        bmu[j] = g.bmean[nc];
        bsc[j] = g.ba[nc];
        bbt[j] = g.bbeta[nc];
      }
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int kk = AKF ? (t & 127) : (t >> 4) + 16 * j, mm = AKF ? (t >> 7) + 2 * j : (t & 15);
      const int k = k0 + kk;
      float a = ra[j];
      if constexpr (TA == 1) a = a > 0.f ? a : 0.f;
      if constexpr (TA == 2) a = (a - amu[j]) * asc[j] + abt[j];
      As[kk][mm] = k < g.K ? a : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int kk = BNF ? (t >> 6) + 4 * j : (t & 127), nn = BNF ? (t & 63) : (t >> 7) + 2 * j;
      float b = rb[j];
      if constexpr (TB == 1) b = b > 0.f ? b : 0.f;
      if constexpr (TB == 2) b = (b - bmu[j]) * bsc[j] + bbt[j];
      Bs[kk][nn] = b;
    }
    __syncthreads();
    if (k0 + kTgKC < g.K) load(k0 + kTgKC);
    const int kn = min(kTgKC, g.K - k0);
    for (int kk = 0; kk < kn; kk += 4) {
      const float a = As[kk + kq][l16];
      acc = mfma4(a, Bs[kk + kq][16 * wave + l16], acc);
      rsum += a;
    }
    __syncthreads();
  }
  if constexpr (TA == 2)
    if (bx == 0 && by == 0) bn_publish(g.abn, t);
  const int m = m0 + l16;
  const bool mok = m < g.M;
  if (g.rowsum && n0 == 0) {  // sum_k TA(A(m,k)) for the tile's rows: lanes with equal l16
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    if (kq == 0 && mok) g.rowsum[m] = rsum;
  }
  // epilogue operands: every load issued (at clamped, in-bounds indices) before any is used -- a
  // per-element conditional load makes hipcc wait for each one in turn
  float cs = 0.f, csx = 0.f, cmx = 0.f;
  const int nc = min(n, g.N - 1);
  float bn = 0.f, xmu = 0.f, xis = 0.f;
  float cmv[4] = {1.f, 1.f, 1.f, 1.f}, xyv[4] = {0.f, 0.f, 0.f, 0.f};
  int mrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) mrow[j] = min(m0 + 4 * kq + j, g.M - 1);
  if (g.bias) bn = g.bias[nc];
  if (g.cmask) {
    long cr[4];
    if (g.cmrow) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cr[j] = g.cmrow[mrow[j]];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) cr[j] = mrow[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) cmv[j] = g.cmask[cr[j] * g.smm + (long)nc * g.smn];
  }
  if (g.colacc) {
    xmu = g.xmean[nc];
    xis = g.xinvstd[nc];
#pragma unroll
    for (int j = 0; j < 4; ++j) xyv[j] = g.xy[(long)mrow[j] * g.N + nc];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int mm = m0 + 4 * kq + j;
    if (mm < g.M && nok) {
      float v = acc[j] + bn;
      if (g.cmask && !(cmv[j] > 0.f)) v = 0.f;
      g.C[(long)mm * g.scm + (long)n * g.scn] = v;
      cmx = fmaxf(cmx, fabsf(v));
      if (g.colacc) {
        cs += v;
        csx += v * ((xyv[j] - xmu) * xis);
      }
    }
  }
  if (g.colacc) {  // this tile's share of the column sums (BN backward of C's channels)
    cs += __shfl_xor(cs, 16, 64); cs += __shfl_xor(cs, 32, 64);
    csx += __shfl_xor(csx, 16, 64); csx += __shfl_xor(csx, 32, 64);
    if (kq == 0 && nok) {
      acc128_add(acc_at(g.colacc, g.N, 0, n), cs);
      acc128_add(acc_at(g.colacc, g.N, 1, n), csx);
    }
  }
  if (g.colmax) {  // max |C| per column over the tile
    cmx = fmaxf(cmx, __shfl_xor(cmx, 16, 64));
    cmx = fmaxf(cmx, __shfl_xor(cmx, 32, 64));
    if (kq == 0 && nok) atomicMax(g.colmax + n, ord_key(cmx));
  }
}


}  // namespace dcue
