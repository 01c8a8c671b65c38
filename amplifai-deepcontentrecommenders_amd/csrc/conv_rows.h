// Row-GEMM conv kernels shared by the forward (conv_fwd.hip) and input-gradient (conv_dgrad.hip)
// translation units.
// Item-tower convolutions on f32-input MFMA (v_mfma_f32_16x16x4_f32), gfx950.
//
// Reference ops replaced (dcrecommend/dcue/audiomodels/truedcuemel1dbn.py):
//   forward  bn_{l-1} -> Conv1d_l -> MaxPool1d -> ReLU   (:77-99), with BN_l batch statistics
//   backward Conv1d weight/bias grads, input grads, MaxPool1d/ReLU/BatchNorm backward (autograd of
//            the same ops, nn/dcue.py:208)
//
// Data layout in HBM (all fp32 unless noted):
//   tracks   [n_tracks][131][128] fp16|fp32      frame-major rows of mel bins (one 256/512-B row per frame)
//   y_l      [M][Lp_l][C_l]   ReLU(maxpool(conv_l)) = input of BN_l;  idx_l same shape, uint8 argmax
//   g_l      [M][Lp_l][C_l]   dL/d(BN_l output), summed over an item's copies
//   wpack    [ks][cin/4][cout][4] forward B operand; [ks][cout/4][cin][4] (taps reversed) dgrad B
// Rows of the GEMM are (item, position) pairs packed densely over items; a workgroup owns 16*TW rows
// and all 128 output channels of its column block (8 waves x 16). Its A operand is an LDS slab of
// the input positions those rows touch (taps + zero halos), built once with the neighbouring
// elementwise op fused into the load, then read with ds_read_b128 (4 consecutive K per lane; the
// four MFMA k-steps of a 16-deep K chunk take one component each).
#pragma once
#include "dcue_internal.h"

namespace dcue {

// Slab fill: every thread owns one channel quad (threads % (KC/4) == 0), so the per-channel operands
// of the fused elementwise op are loaded once; the raw global reads of a batch of slab slots are
// issued branch-free (clamped addresses, masked afterwards) before any is used -- the loads are the
// latency of these small kernels, not the math.
struct ChanOps {        // per-channel constants of the fused op for one channel quad
  float4 mu, sc, be;    // forward: (x - mu) * sc + be
  float4 inv, sd, sdx;  // dgrad: BN_l backward (mu = mean_l, sc = a_l)
};

// Per-channel constants of the fused op, finalized once per channel per workgroup (thread t owns
// channel t) into LDS, then read by quad: the fp64 finalize is one short chain per thread.
struct ChanLds {
  float v[5][256];
  float wmax[4];  // split-f16 forward: the per-wave maxima of the channels' value bounds
};

// The global inputs of chan_stage / range_stage for thread t's channel, loaded at the kernel's
// entry before the weight prefetch and the slab reads: loads return in issue order, so loaded after
// those (as they were) the fp64 finalize and the split-scale bound waited for the whole first slab
// batch and then added their own chain (kernel-phase traces).
struct ChanPre {
  unsigned long long w[4];  // forward train: the input BN's (sum, sum sq) words; dgrad: (sD, sDx)
  float f[3];               // forward: gamma | (mean, a), beta; dgrad: mean_l, a_l, invstd_l
  unsigned r[2];            // split-f16: range keys (forward hi / -lo; dgrad max|g|, y_l's max)
  double count, inv_count;
  bool train;
};
template <int SRC, bool F16>
__device__ __forceinline__ ChanPre chan_preload(const RowsArgs& a, int KC) {
  ChanPre q;
  const int t = threadIdx.x;
  q.w[0] = q.w[1] = q.w[2] = q.w[3] = 0;
  q.f[0] = q.f[1] = q.f[2] = 0.f;
  q.r[0] = q.r[1] = 0u;
  q.count = a.in_bn.count;
  q.inv_count = a.in_bn.inv_count;
  q.train = SRC != SRC_DZ && a.in_bn.acc != nullptr;
  if (t >= KC) return q;
  const unsigned long long* acc = SRC == SRC_DZ ? a.dz_acc : a.in_bn.acc;
  if (SRC == SRC_DZ || q.train) {
    q.w[0] = acc[(size_t)t * 2];
    q.w[1] = acc[(size_t)t * 2 + 1];
    q.w[2] = acc[((size_t)KC + t) * 2];
    q.w[3] = acc[((size_t)KC + t) * 2 + 1];
  }
  if constexpr (SRC != SRC_DZ) {
    if (q.train) {
      q.f[0] = a.in_bn.gamma[t];
    } else {
      q.f[0] = a.in_mean[t];
      q.f[1] = a.in_a[t];
    }
    q.f[2] = a.in_beta ? a.in_beta[t] : 0.f;
    if constexpr (F16)
      if (a.in_range) {
        q.r[0] = a.in_range[t];
        q.r[1] = a.in_range[kRngC + t];
      }
  } else {
    q.f[0] = a.mean_l[t];
    q.f[1] = a.a_l[t];
    q.f[2] = a.invstd_l[t];
    if constexpr (F16)
      if (a.in_range) {
        q.r[0] = a.in_range[t];
        q.r[1] = a.y_range ? a.y_range[t] : 0u;
      }
  }
  return q;
}

// Split-f16 forward operand scale. Every slab value v is stored as v*S = hi + lo in
// fp16, S a power of two, and the epilogue multiplies the accumulators by 1/S: exact, so the result
// is what the unscaled split computes wherever that one is in range. S puts the largest |v| the layer
// can produce in [2^14, 2^15): no fp16 overflow (65504) whatever the input magnitudes, and small
// activations (unnormalised towers, tiny inputs) keep hi/lo out of fp16's subnormals, so the split
// stays ~2^-22 relative to the layer's scale. The bound of channel c comes from the input layer's
// range (RowsArgs::in_range): v = (x - mu) sc + be is monotone in x, so its extremes over the batch
// are at x = min and x = max (the ReLU outputs of layers >= 2 have min 0). Every workgroup of the
// launch reads the same ranges, so all use the same S. Threads t < KC own channel t (chan_stage);
// waves 0-3 reduce the bounds, and after the block barrier every thread forms S from the four.
// The dgrad (SRC_DZ) operand is dz = a (g - kD sD - kD xhat sDx) (masked): |dz| <= |a| (max|g| +
// kDmax (|sD| + max|xhat| |sDx|)), max|g| from the producer's epilogue (in_range), max|xhat| from
// y_l's range -- the same bound as the split-f16 weight gradient's (conv_wgrad.hip).
template <int SRC>
__device__ __forceinline__ void range_stage(const RowsArgs& a, const ChanPre& q, int KC, ChanLds& L) {
  const int t = threadIdx.x;
  if (t >= 256) return;  // waves 0-3 (uniform per wave)
  float bnd = 0.f;
  if (SRC == SRC_DZ) {
    if (t < KC && a.in_range) {
      const unsigned kg = q.r[0], ky = q.r[1];
      const float gmax = kg ? ord_value(kg) : 0.f, ym = ky ? fmaxf(ord_value(ky), 0.f) : 0.f;
      const float mu = L.v[0][t], av = L.v[1][t], iv = L.v[2][t];
      const float xhm = fmaxf(fabsf(mu), fabsf(ym - mu)) * iv;
      bnd = fabsf(av) * (gmax + a.kd_max * (fabsf(L.v[3][t]) + xhm * fabsf(L.v[4][t])));
    }
  } else if (t < KC && a.in_range) {
    const unsigned khi = q.r[0], knlo = q.r[1];
    float hi = khi ? ord_value(khi) : 0.f;
    float lo = (SRC == SRC_ACT) ? 0.f : (knlo ? -ord_value(knlo) : 0.f);
    if (SRC == SRC_ACT) hi = fmaxf(hi, 0.f);
    const float mu = L.v[0][t], sc = L.v[1][t], be = L.v[2][t];
    bnd = fmaxf(fabsf((lo - mu) * sc + be), fabsf((hi - mu) * sc + be));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) bnd = fmaxf(bnd, __shfl_xor(bnd, off, 64));
  if ((t & 63) == 0) L.wmax[t >> 6] = bnd;
}

struct SplitScale {
  float s, inv;
};
__device__ __forceinline__ SplitScale split_scale(const ChanLds& L, int KC) {
  float m = L.wmax[0];
  for (int w = 1; w < (KC + 63) / 64; ++w) m = fmaxf(m, L.wmax[w]);
  SplitScale r = {1.f, 1.f};
  if (m > 0.f && m < INFINITY) {  // else (all zero, or a non-finite input that propagates anyway) 1
    int e;
    (void)frexpf(m, &e);  // m in [2^(e-1), 2^e)
    const int k = min(max(15 - e, -120), 120);
    r.s = ldexpf(1.f, k);
    r.inv = ldexpf(1.f, -k);
  }
  return r;
}

template <int SRC>
__device__ __forceinline__ void chan_stage(const ChanPre& q, int KC, ChanLds& L) {
  const int t = threadIdx.x;
  if (t >= KC) return;
  if constexpr (SRC != SRC_DZ) {
    if (q.train) {  // train: the input BN's batch statistics, finalized here
      const BnChan st = bn_chan_sums(acc128_words(q.w[0], q.w[1]), acc128_words(q.w[2], q.w[3]), q.count,
                                     q.inv_count);
      L.v[0][t] = st.mean;
      L.v[1][t] = q.f[0] * st.invstd;
    } else {
      L.v[0][t] = q.f[0];
      L.v[1][t] = q.f[1];
    }
    L.v[2][t] = q.f[2];
  } else {
    L.v[0][t] = q.f[0];
    L.v[1][t] = q.f[1];
    L.v[2][t] = q.f[2];
    L.v[3][t] = (float)acc128_words(q.w[0], q.w[1]);
    L.v[4][t] = (float)acc128_words(q.w[2], q.w[3]);
  }
}

template <int SRC>
__device__ __forceinline__ ChanOps chan_ops(const ChanLds& L, int c) {
  auto q = [&](int i) { return *reinterpret_cast<const float4*>(&L.v[i][c]); };
  ChanOps k;
  k.mu = q(0);
  k.sc = q(1);
  if constexpr (SRC != SRC_DZ) {
    k.be = q(2);
  } else {
    k.inv = q(2);
    k.sd = q(3);
    k.sdx = q(4);
  }
  return k;
}

struct Raw {
  float4 a, b;
  uint32_t id;
  float cnt;
};

template <int SRC, int KC, int LIN, int LPL, int POOLL>
__device__ __forceinline__ Raw slab_load(const RowsArgs& a, long i, int p, int c, long trk) {
  Raw r;
  if constexpr (SRC == SRC_TRACK_F16) {
    const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.src) +
                                                      ((trk * kFrames + p) * kMels + c));
    r.a.x = __uint_as_float(raw.x);
    r.a.y = __uint_as_float(raw.y);
  } else if constexpr (SRC == SRC_TRACK_F32) {
    r.a = ld4(reinterpret_cast<const float*>(a.src) + ((trk * kFrames + p) * kMels + c));
  } else if constexpr (SRC == SRC_ACT) {
    r.a = ld4(reinterpret_cast<const float*>(a.src) + ((i * LIN + p) * KC + c));
  } else {
    const int w = p / POOLL;
    const long base = (i * LPL + w) * KC + c;
    r.a = ld4(reinterpret_cast<const float*>(a.src) + base);
    r.b = ld4(a.y_l + base);
    r.id = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
    r.cnt = a.counts ? a.counts[i] : 1.f;
  }
  return r;
}

template <int SRC, int POOLL>
__device__ __forceinline__ float4 slab_finish(const RowsArgs& a, const ChanOps& k, int p, const Raw& r) {
  if constexpr (SRC != SRC_DZ) {
    float x[4];
    if constexpr (SRC == SRC_TRACK_F16) {
      const uint32_t lo = __float_as_uint(r.a.x), hi = __float_as_uint(r.a.y);
      const __half2 h0 = *reinterpret_cast<const __half2*>(&lo);
      const __half2 h1 = *reinterpret_cast<const __half2*>(&hi);
      x[0] = __low2float(h0); x[1] = __high2float(h0); x[2] = __low2float(h1); x[3] = __high2float(h1);
    } else {
      x[0] = r.a.x; x[1] = r.a.y; x[2] = r.a.z; x[3] = r.a.w;
    }
    return make_float4((x[0] - k.mu.x) * k.sc.x + k.be.x, (x[1] - k.mu.y) * k.sc.y + k.be.y,
                       (x[2] - k.mu.z) * k.sc.z + k.be.z, (x[3] - k.mu.w) * k.sc.w + k.be.w);
  } else {
    // conv position p of layer l -> pool window w, offset j; gradient reaches p only if it was the
    // window's argmax and the window's ReLU was active (threshold_backward on the ReLU output).
    const int j = p % POOLL;
    const float kD = r.cnt * a.invN;
    const float gv[4] = {r.a.x, r.a.y, r.a.z, r.a.w}, yv[4] = {r.b.x, r.b.y, r.b.z, r.b.w};
    const float mu[4] = {k.mu.x, k.mu.y, k.mu.z, k.mu.w}, iv[4] = {k.inv.x, k.inv.y, k.inv.z, k.inv.w};
    const float av[4] = {k.sc.x, k.sc.y, k.sc.z, k.sc.w}, sd[4] = {k.sd.x, k.sd.y, k.sd.z, k.sd.w};
    const float sdx[4] = {k.sdx.x, k.sdx.y, k.sdx.z, k.sdx.w};
    float o[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float xh = (yv[s] - mu[s]) * iv[s];
      const float dx = av[s] * (gv[s] - kD * sd[s] - kD * xh * sdx[s]);
      const int arg = (r.id >> (8 * s)) & 0xff;
      o[s] = (arg == j && yv[s] > 0.f) ? dx : 0.f;
    }
    return make_float4(o[0], o[1], o[2], o[3]);
  }
}

// MODE 0 = forward (pool+relu+stats epilogue), 1 = dgrad (plain store).
// Slab position p of item i is valid for 0 <= p < LIN; rows are (i, t), t < R; tap k of row t reads
// slab position t + k - PADL.
// Eight waves per workgroup, two per SIMD: wave w owns output columns [16 (w mod 8), +16) of the
// block for all TW row tiles, so while one wave of a SIMD waits on its weight loads the other
// issues MFMAs (with four waves of 32 columns the loads' latency was exposed: ~40% of wave cycles
// parked on s_waitcnt).
constexpr int kRowsWaves = 8, kRowsThreads = 64 * kRowsWaves, kRowsCT = 128 / (16 * kRowsWaves);

// Split-f16 forward (F16): the slab holds every input value v as v = hi + lo, hi = fp16(v), lo =
// fp16(v - hi); a row is [hi x KC][lo x KC] halves (channel c's hi at dword c/2, its lo KC/2 dwords
// further; the pitch is unchanged, KC + 8 dwords). A lane's 8 channels of a 32-channel chunk are
// then 4 dwords at 4g, as in the f32 slab, so the ds_read_b128 lane groups stay conflict-free (an
// interleaved [hi x 8][lo x 8] octet layout put them 8g apart: 2-way on every read, measured 53 % of
// the LDS cycles). |v| must stay below the fp16 range (65504), which the fp16 track table bounds
// for layer 1; BatchNorm keeps the others O(1).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <int KC>
__device__ __forceinline__ void st_split(float* row, int c, float4 v) {
  const f16x4 h = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
  const f16x4 l = {(_Float16)(v.x - (float)h[0]), (_Float16)(v.y - (float)h[1]),
                   (_Float16)(v.z - (float)h[2]), (_Float16)(v.w - (float)h[3])};
  *reinterpret_cast<f16x4*>(row + c / 2) = h;
  *reinterpret_cast<f16x4*>(row + KC / 2 + c / 2) = l;
}
// B k-steps (float4 per lane per 16-column tile) requested ahead of the MFMAs by one-tile workgroups
// (the small layers at in-batch M): a layer's whole K at H = 128 (32 steps), so they wait on the
// weights once, not once every two steps
#ifndef DCUE_ROWS_PD
#define DCUE_ROWS_PD 32
#endif
constexpr int kRowsPD = DCUE_ROWS_PD;

// The workgroup (bx, by) of a k_conv_rows launch, as a device function (k_conv_rows runs it on its grid)
template <int MODE, int SRC, int KC, int KS, int PADL, int LIN, int R, int POOL, int TW, int LPL,
          int POOLL, bool DEEP, bool F16>
__device__ __forceinline__ void conv_rows_body(const RowsArgs& a, const int bx, const int by) {
  critical_path_priority();
  // (DCUE_KTRACE: kernels 2-6 the forwards by input length (layers 1-5), 7-11 the dgrads)
  [[maybe_unused]] constexpr int KID = 2 + MODE * 5 + (LIN >= 131 ? 0 : LIN >= 32 ? 1 : LIN >= 8 ? 2 : LIN >= 2 ? 3 : 4);
  DCUE_KTW(KID, 6);
  DCUE_KT(KID, 0);
  const ChanPre cpre = chan_preload<SRC, F16>(a, KC);
  // (plans, conv 2: the previous step's late Adam on the user stream wrote its weights -- read below,
  // after the loads above, which read only this stream's data)
  if (MODE == 0) dev_wait(a.wait);
  if (MODE == 0 && a.rp_src) {  // conv 2's deferred input-gradient operands (RowsArgs::rp)
    const long n = (long)a.rp.cout * a.rp.cin * a.rp.ks;
    const long nt = (long)gridDim.x * gridDim.y * blockDim.x;
    for (long e = ((long)by * gridDim.x + bx) * blockDim.x + threadIdx.x; e < n; e += nt)
      pack_store(a.rp, e, a.rp_src[e], a.rp_wpack);
  }
  constexpr int RX = R + KS - 1;
  constexpr int ROWS = TW * 16;
  constexpr int MAXI = (ROWS + R - 1) / R + 1;
  constexpr int PITCH = KC + 8;  // == 8 (mod 64) dwords: conflict-free ds_read_b128 over 16 rows
  constexpr int C4 = KC / 4;
  constexpr int NSTEP = KS * (KC / 16);
  extern __shared__ __attribute__((aligned(16))) float slab[];

  const int M = a.M;
  const long total = (long)M * R;
  const long gr0 = (long)bx * ROWS;
  const long gr1 = min(gr0 + ROWS, total);
  const long i0 = gr0 / R, i1 = (gr1 - 1) / R;
  const long elo = i0 * RX + (gr0 - i0 * R);
  const int nslab = (int)(i1 * RX + (gr1 - 1 - i1 * R) + KS - elo);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int nout = a.nout;
  constexpr int CT = kRowsCT;  // 16-column MFMA tiles per wave
  const int ocol0 = by * 128 + wave * 16 * CT;
  const bool colok = ocol0 < nout;

  // B operand (packed weights, L2-resident): the first PD k-steps are requested before anything
  // else -- they land while the slab is filled -- and each consumed slot is refilled PD steps ahead
  // (DEEP: launches of at most one workgroup per CU; the larger ones keep two steps ahead -- deep
  // prefetch there costs occupancy, and their other workgroups cover the load latency)
  constexpr int PDW = DEEP ? kRowsPD / CT : 2;
  constexpr int PD = NSTEP < PDW ? NSTEP : PDW;
  const float* wp = a.wpack + ((size_t)g * nout + (colok ? ocol0 : 0) + l16) * 4;
  const size_t wstep = (size_t)16 * nout;
  float4 bq[F16 ? 1 : PD][CT];
  // split-f16 path: 32-channel K chunks, a lane's (hi, lo) octets of its column per chunk
  constexpr int NCH = KS * (KC / 32);
  constexpr int PDW16 = DEEP ? kRowsPD / (2 * CT) : 3;  // 3 chunks: keeps <= 128 VGPRs (2 WGs per CU)
  constexpr int PD16 = NCH < PDW16 ? NCH : PDW16;
  const f16x8* wp16 = reinterpret_cast<const f16x8*>(a.wpack16) +
                      (((size_t)(colok ? ocol0 : 0) + l16) * 4 + g) * 2;
  const size_t wstep16 = (size_t)8 * nout;
  f16x8 bh[F16 ? PD16 : 1][CT][2];
  if constexpr (F16) {
#pragma unroll
    for (int st = 0; st < PD16; ++st)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bh[st][ct][0] = wp16[st * wstep16 + 128 * ct];
        bh[st][ct][1] = wp16[st * wstep16 + 128 * ct + 1];
      }
  } else {
#pragma unroll
    for (int st = 0; st < PD; ++st)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) bq[st][ct] = ld4(wp + st * wstep + 64 * ct);
  }

  SplitScale sscale = {1.f, 1.f};  // split-f16 operand scale (range_stage)
  {
    static_assert(kRowsThreads % C4 == 0, "a thread's slab slots share one channel quad");
    // slab slots (float4) in flight per thread: at most what the workgroup's slab can hold (its rows
    // plus a KS-1 halo per item spanned) -- every slot of a batch is loaded, masked or not, so the
    // one-tile launches of in-batch steps (<= 2 slots per thread) issued 6 of 8 loads for nothing
    constexpr int FB0 = SRC == SRC_DZ ? 4 : 8;
    constexpr int FB_NEED = ((ROWS + MAXI * (KS - 1)) * C4 + kRowsThreads - 1) / kRowsThreads;
    constexpr int FB = FB_NEED < FB0 ? FB_NEED : FB0;
    const int nfill = nslab * C4;
    const int c = 4 * (threadIdx.x % C4);
    __shared__ ChanLds chl;
    // the track ids of the workgroup's items (uniform: scalar loads issued before anything else), so
    // the slab's row loads do not wait on a per-slot item_track load first; rows of one workgroup
    // span at most two items whenever ROWS <= R (MAXI == 2)
    constexpr bool kTrack = SRC == SRC_TRACK_F16 || SRC == SRC_TRACK_F32;
    constexpr bool trk_pre = kTrack && MAXI <= 2;  // compile-time: no second fill path (VGPRs)
    int trk_lo = 0, trk_hi = 0;                    // uniform: SGPRs
    if constexpr (trk_pre) {
      trk_lo = __builtin_amdgcn_readfirstlane(a.item_track[i0]);
      trk_hi = __builtin_amdgcn_readfirstlane(a.item_track[min(i1, (long)M - 1)]);
    }
    int pp[FB];
    bool ok[FB];
    Raw raw[FB];
    // raw global reads of one batch of slab slots, branch-free (clamped addresses, masked later)
    auto load_batch = [&](int base) {
      long ii[FB];
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int e = base + kRowsThreads * j;
        const long E = elo + e / C4;
        const long i = E / RX;
        const int p = (int)(E - i * RX) - PADL;
        ok[j] = e < nfill && i < M && p >= 0 && p < LIN;
        ii[j] = ok[j] ? i : 0;  // masked slots load a real element and store zero
        pp[j] = ok[j] ? p : 0;
      }
      long trk[FB];
#pragma unroll
      for (int j = 0; j < FB; ++j) trk[j] = 0;
      if constexpr (trk_pre) {
#pragma unroll
        for (int j = 0; j < FB; ++j) trk[j] = ii[j] == i0 ? trk_lo : trk_hi;
      } else if constexpr (kTrack) {
#pragma unroll
        for (int j = 0; j < FB; ++j) trk[j] = a.item_track[ii[j]];
      }
#pragma unroll
      for (int j = 0; j < FB; ++j) raw[j] = slab_load<SRC, KC, LIN, LPL, POOLL>(a, ii[j], pp[j], c, trk[j]);
    };
    auto store_batch = [&](int base, const ChanOps& kop) {
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int e = base + kRowsThreads * j;
        if (e < nfill) {
          const float4 v = slab_finish<SRC, POOLL>(a, kop, pp[j], raw[j]);
          if constexpr (F16)
            st_split<KC>(&slab[(e / C4) * PITCH], c,
                         ok[j] ? make_float4(v.x * sscale.s, v.y * sscale.s, v.z * sscale.s, v.w * sscale.s)
                               : make_float4(0.f, 0.f, 0.f, 0.f));
          else
            st4(&slab[(e / C4) * PITCH + c], ok[j] ? v : make_float4(0.f, 0.f, 0.f, 0.f));
        }
      }
    };
    // the first batch's reads are in flight while the per-channel constants are finalized
    load_batch(threadIdx.x);
    chan_stage<SRC>(cpre, KC, chl);
    if constexpr (F16) range_stage<SRC>(a, cpre, KC, chl);
    if constexpr (SRC != SRC_DZ)
      if (bx == 0 && by == 0) bn_publish(a.in_bn, threadIdx.x);
    DCUE_KT(KID, 5);
    __syncthreads();
    if constexpr (F16) sscale = split_scale(chl, KC);
    const ChanOps kop = chan_ops<SRC>(chl, c);
    store_batch(threadIdx.x, kop);
    for (int base = threadIdx.x + kRowsThreads * FB; base < nfill; base += kRowsThreads * FB) {
      load_batch(base);
      store_batch(base, kop);
    }
  }
  DCUE_KT(KID, 1);
  __syncthreads();
  DCUE_KT(KID, 2);
  if (!colok) return;  // no barrier follows

  int sbase[TW];
#pragma unroll
  for (int r = 0; r < TW; ++r) {
    long gr = gr0 + 16 * r + l16;
    if (gr >= total) gr = gr0;
    const long i = gr / R;
    sbase[r] = (int)(i * RX + (gr - i * R) - elo) * PITCH + 4 * g;
  }

  f32x4 acc[TW][CT];
#pragma unroll
  for (int r = 0; r < TW; ++r)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[r][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (F16) {
    // x*w = (xh + xl)(wh + wl) ~ xl*wh + xh*wl + xh*wh: three v_mfma_f32_16x16x32_f16 per 32-channel
    // chunk (fp16 products are exact in f32; the dropped xl*wl and the lo roundings are ~2^-22 of
    // |x*w|), the small terms first
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      f16x8 b[CT][2];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        b[ct][0] = bh[ch % PD16][ct][0];
        b[ct][1] = bh[ch % PD16][ct][1];
        if (ch + PD16 < NCH) {
          bh[ch % PD16][ct][0] = wp16[(ch + PD16) * wstep16 + 128 * ct];
          bh[ch % PD16][ct][1] = wp16[(ch + PD16) * wstep16 + 128 * ct + 1];
        }
      }
      // one chunk's operands live at a time: without the barrier hipcc hoists every chunk's LDS reads
      // (223 VGPRs, one workgroup per CU, no fill/MFMA overlap between workgroups)
      __builtin_amdgcn_sched_barrier(0);
      const int k = ch / (KC / 32);
      const int aoff = k * PITCH + 16 * (ch - k * (KC / 32));  // + sbase's 4g: the lane's 8 channels
      f16x8 ah[TW], al[TW];
#pragma unroll
      for (int r = 0; r < TW; ++r) {
        ah[r] = *reinterpret_cast<const f16x8*>(&slab[sbase[r] + aoff]);
        al[r] = *reinterpret_cast<const f16x8*>(&slab[sbase[r] + aoff + KC / 2]);
      }
#pragma unroll
      for (int r = 0; r < TW; ++r)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          acc[r][ct] = mfma16(al[r], b[ct][0], acc[r][ct]);
          acc[r][ct] = mfma16(ah[r], b[ct][1], acc[r][ct]);
          acc[r][ct] = mfma16(ah[r], b[ct][0], acc[r][ct]);
        }
    }
  }
  // fully unrolled: straight-line code lets the wait counters track the in-flight B loads exactly
#pragma unroll
  for (int st = 0; st < (F16 ? 0 : NSTEP); ++st) {
    float4 b[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      b[ct] = bq[st % PD][ct];
      if (st + PD < NSTEP) bq[st % PD][ct] = ld4(wp + (st + PD) * wstep + 64 * ct);
    }
    const int k = st / (KC / 16);
    const int c0 = (st - k * (KC / 16)) * 16;
    const int aoff = k * PITCH + c0;
    float4 av[TW];
#pragma unroll
    for (int r = 0; r < TW; ++r) av[r] = *reinterpret_cast<const float4*>(&slab[sbase[r] + aoff]);
#pragma unroll
    for (int r = 0; r < TW; ++r)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[r][ct] = mfma4(av[r].x, b[ct].x, acc[r][ct]);
#pragma unroll
    for (int r = 0; r < TW; ++r)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[r][ct] = mfma4(av[r].y, b[ct].y, acc[r][ct]);
#pragma unroll
    for (int r = 0; r < TW; ++r)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[r][ct] = mfma4(av[r].z, b[ct].z, acc[r][ct]);
#pragma unroll
    for (int r = 0; r < TW; ++r)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[r][ct] = mfma4(av[r].w, b[ct].w, acc[r][ct]);
  }

  DCUE_KT(KID, 3);
  if constexpr (MODE == 1) {
    // g_{l-1} rows, plus this tile's share of BN_{l-1}'s backward sums (sum g, sum g*xhat)
    float sg[CT] = {}, sgx[CT] = {}, gmx[CT] = {};
    // the workgroup's partial sums into the exact accumulators
    auto flush_g = [&](int ct) {
      float s = sg[ct], q = sgx[ct];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (g == 0) {
        const int o = ocol0 + 16 * ct + l16;
        acc128_add(acc_at(a.out_acc, nout, 0, o), s);
        acc128_add(acc_at(a.out_acc, nout, 1, o), q);
      }
      sg[ct] = 0.f;
      sgx[ct] = 0.f;
    };
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int o = ocol0 + 16 * ct + l16;
      const float mu = a.out_acc ? a.omean[o] : 0.f, is = a.out_acc ? a.oinvstd[o] : 0.f;
#pragma unroll
      for (int r = 0; r < TW; ++r) {
        const long grb = gr0 + 16 * r + 4 * g;
        float yv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long row = grb + j < total ? grb + j : gr0;
          yv[j] = a.out_acc ? a.oy[row * nout + o] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (grb + j < total) {
            float gv = acc[r][ct][j] * sscale.inv;  // 1 on the f32 path; exact power of two on the split path
            if (a.skip && o < a.skip_n) gv += a.skip[((grb + j) / R) * a.skip_ld + o] * a.skip_scale;
            a.out[(grb + j) * nout + o] = gv;
            gmx[ct] = fmaxf(gmx[ct], fabsf(gv));
            sg[ct] += gv;
            sgx[ct] += gv * ((yv[j] - mu) * is);
          }
      }
    }
    if (a.out_acc) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) flush_g(ct);
    }
    if (a.out_grange) {  // max |g_{l-1}| per channel: the split-f16 weight gradient's dz bound
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        float m = gmx[ct];
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (g == 0) atomicMax(a.out_grange + ocol0 + 16 * ct + l16, ord_key(m));
      }
    }
  } else {
    constexpr int LP = R / POOL;
    float ssum[CT] = {}, ssq[CT] = {}, ymax[CT] = {};
    const float inv_s = sscale.inv;  // 1 on the f32 path; exact power of two on the split path
    auto flush_y = [&](int ct) {  // (as flush_g)
      float s = ssum[ct], q = ssq[ct];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (g == 0) {
        const int o = ocol0 + 16 * ct + l16;
        acc128_add(acc_at(a.out_acc, nout, 0, o), s);
        acc128_add(acc_at(a.out_acc, nout, 1, o), q);
      }
      ssum[ct] = 0.f;
      ssq[ct] = 0.f;
    };
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int o = ocol0 + 16 * ct + l16;
      const float bias = a.bias[o];
#pragma unroll
      for (int r = 0; r < TW; ++r) {
        const long grb = gr0 + 16 * r + 4 * g;
#pragma unroll
        for (int win = 0; win < 4 / POOL; ++win) {
          const long row = grb + win * POOL;  // first conv row of this pool window
          if (row < total) {
            const long i = row / R;
            const int w = (int)(row - i * R) / POOL;
            float best = acc[r][ct][win * POOL] * inv_s + bias;
            int arg = 0;
#pragma unroll
            for (int j = 1; j < POOL; ++j) {
              const float v = acc[r][ct][win * POOL + j] * inv_s + bias;
              if (v > best) { best = v; arg = j; }  // first maximum wins (max_pool1d)
            }
            const float y = best > 0.f ? best : 0.f;
            ymax[ct] = fmaxf(ymax[ct], y);
            const long oidx = (i * LP + w) * nout + o;
            a.out[oidx] = y;
            a.out_idx[oidx] = (uint8_t)arg;
            const float cnt = a.counts ? a.counts[i] : 1.f;
            ssum[ct] += cnt * y;
            ssq[ct] += cnt * y * y;
          }
        }
      }
    }
    if (a.out_acc) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) flush_y(ct);
    }
    if (a.out_range) {  // the output's per-channel maximum: the next layer's split scale
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        float m = ymax[ct];
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (g == 0) atomicMax(a.out_range + ocol0 + 16 * ct + l16, ord_key(m));
      }
    }
  }
  DCUE_KT(KID, 4);
  DCUE_KTW(KID, 7);
}

template <int MODE, int SRC, int KC, int KS, int PADL, int LIN, int R, int POOL, int TW, int LPL,
          int POOLL, bool DEEP, bool F16>
__global__ __launch_bounds__(kRowsThreads) void k_conv_rows(RowsArgs a) {
  conv_rows_body<MODE, SRC, KC, KS, PADL, LIN, R, POOL, TW, LPL, POOLL, DEEP, F16>(a, blockIdx.x, blockIdx.y);
}

template <int MODE, int SRC, int KC, int KS, int PADL, int LIN, int R, int POOL, int TW, int LPL,
          int POOLL, bool DEEP, bool F16>
static int run_rows_pd(const RowsArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  auto kern = k_conv_rows<MODE, SRC, KC, KS, PADL, LIN, R, POOL, TW, LPL, POOLL, DEEP, F16>;
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
    attr = true;
  }
  DCUE_LAUNCH(kern, grid, dim3(kRowsThreads), lds, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

template <int MODE, int SRC, int KC, int KS, int PADL, int LIN, int R, int POOL, int TW, int LPL,
          int POOLL, bool F16 = false>
static int run_rows(const RowsArgs& a, hipStream_t s) {
  constexpr int ROWS = TW * 16;
  constexpr int MAXI = (ROWS + R - 1) / R + 1;
  constexpr int SLAB = ROWS + MAXI * (KS - 1);
  constexpr size_t LDS = (size_t)SLAB * (KC + 8) * sizeof(float);
  static_assert(LDS + sizeof(ChanLds) <= 160 * 1024, "slab exceeds LDS");
  const long total = (long)a.M * R;
  dim3 grid((unsigned)((total + ROWS - 1) / ROWS), (unsigned)((a.nout + 127) / 128));
  if (TW == 1 && (long)grid.x * grid.y <= 256)  // one-tile workgroups, one per CU: weights run ahead
    return run_rows_pd<MODE, SRC, KC, KS, PADL, LIN, R, POOL, TW, LPL, POOLL, true, F16>(a, grid, LDS, s);
  return run_rows_pd<MODE, SRC, KC, KS, PADL, LIN, R, POOL, TW, LPL, POOLL, false, F16>(a, grid, LDS, s);
}

// Row tiles per workgroup. Each wave runs TW 16-row tiles of its 32 columns back to back, and a
// CU given k workgroups runs their waves on the same four SIMDs, so the launch takes about
// TW * ceil(workgroups / 256) tile times: 528 tiles (layer 1 at B = 64) cost 4 at TW = 2 (264
// workgroups, eight CUs doubled up) but 3 at TW = 3 (176). Ties go to the larger TW (fewer
// re-reads of the weights, which every workgroup streams whole).
static int choose_tw(long rows, int twmax) {
  // tuning diagnostic: DCUE_ROWS_TW=n forces n tiles per workgroup where the slab fits (A/B runs)
  static const int forced = [] {
    const char* e = getenv("DCUE_ROWS_TW");
    return e ? atoi(e) : 0;
  }();
  if (forced == 1 || forced == 2 || forced == 3 || forced == 4 || forced == 8)
    if (forced <= twmax) return forced;
  constexpr long kCUs = 256;
  const long tiles = (rows + 15) / 16;
  // Many tiles (catalogue M): four tiles per workgroup once that still leaves two workgroups per
  // CU. Every workgroup streams the layer's whole packed weights from L2, so one-tile workgroups
  // re-read them 4x as often; measured at M = 1,344 (tw_sweep.sh): layer-2 dgrad 179 -> 105 us,
  // layer-2 forward 86 -> 65 us against the pass-count model's TW = 1.
  // Every workgroup also streams the layer's whole packed weights (256 KB of split-f16 B operand
  // for conv 1) from L2, so the largest launches take eight tiles per workgroup once that still
  // leaves two workgroups per CU: catalogue conv-1 forward (M = 1,344: 11k tiles), forced-TW A/B
  // 0.578 -> 0.556 ms per catalogue step; TW = 2 0.748 ms.
  if (twmax >= 8 && tiles >= 8 * 2 * kCUs) return 8;
  if (twmax >= 4 && tiles >= 4 * 2 * kCUs) return 4;
  int best = 1;
  long best_cost = -1;
  for (int tw : {1, 2, 3, 4, 8}) {
    if (tw > twmax) break;
    const long wgs = (tiles + tw - 1) / tw;
    const long cost = tw * ((wgs + kCUs - 1) / kCUs);
    if (best_cost < 0 || cost <= best_cost) {
      best = tw;
      best_cost = cost;
    }
  }
  return best;
}


// Split-f16 forward (three f16 MFMAs per 32-channel chunk, ~2^-22 relative per product, at 3/16 of
// the f32 MFMA time) unless DCUE_CONV_F16=0 selects the exact-f32 path
static bool conv_f16_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_CONV_F16");
    return !(e && e[0] == '0');
  }();
  return on;
}

// LDS bytes of a slab for R rows per item, KS taps, KC channels and TW row tiles
constexpr size_t slab_bytes(int R, int KS, int KC, int TW) {
  return (size_t)(TW * 16 + ((TW * 16 + R - 1) / R + 1) * (KS - 1)) * (KC + 8) * sizeof(float);
}
constexpr size_t kSlabMax = 160 * 1024 - sizeof(ChanLds);
constexpr int max_tw(int R, int KS, int KC) {
  return slab_bytes(R, KS, KC, 8) <= kSlabMax ? 8
       : slab_bytes(R, KS, KC, 4) <= kSlabMax ? 4
       : slab_bytes(R, KS, KC, 2) <= kSlabMax ? 2 : 1;
}

}  // namespace dcue
