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

// BN_l backward sums of channel c from its accumulators: sum g (sD) and sum g*xhat (sDx)
__device__ __forceinline__ float2 bwd_sums(const unsigned long long* acc, int C, int c) {
  return make_float2((float)acc_sum(acc, C, 0, c), (float)acc_sum(acc, C, 1, c));
}

// Per-channel constants of the fused op, finalized once per channel per workgroup (thread t owns
// channel t) into LDS, then read by quad: the fp64 finalize is one short chain per thread.
struct ChanLds {
  float v[5][256];
  float wmax[4];  // split-f16 forward: the per-wave maxima of the channels' value bounds
};

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
template <int SRC>
__device__ __forceinline__ void range_stage(const RowsArgs& a, int KC, ChanLds& L) {
  const int t = threadIdx.x;
  if (t >= 256) return;  // waves 0-3 (uniform per wave)
  float bnd = 0.f;
  if (t < KC && a.in_range) {
    const unsigned khi = a.in_range[t], knlo = a.in_range[kRngC + t];
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
__device__ __forceinline__ void chan_stage(const RowsArgs& a, int KC, ChanLds& L) {
  const int t = threadIdx.x;
  if (t >= KC) return;
  if constexpr (SRC != SRC_DZ) {
    if (a.in_bn.acc) {  // train: the input BN's batch statistics, finalized here
      const BnChan st = bn_chan_train(a.in_bn.acc, KC, t, a.in_bn.count, a.in_bn.inv_count);
      L.v[0][t] = st.mean;
      L.v[1][t] = a.in_bn.gamma[t] * st.invstd;
    } else {
      L.v[0][t] = a.in_mean[t];
      L.v[1][t] = a.in_a[t];
    }
    L.v[2][t] = a.in_beta ? a.in_beta[t] : 0.f;
  } else {
    L.v[0][t] = a.mean_l[t];
    L.v[1][t] = a.a_l[t];
    L.v[2][t] = a.invstd_l[t];
    const float2 sd = bwd_sums(a.dz_acc, KC, t);
    L.v[3][t] = sd.x;
    L.v[4][t] = sd.y;
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

template <int MODE, int SRC, int KC, int KS, int PADL, int LIN, int R, int POOL, int TW, int LPL,
          int POOLL, bool DEEP, bool F16>
__global__ __launch_bounds__(kRowsThreads) void k_conv_rows(RowsArgs a) {
  critical_path_priority();
  constexpr int RX = R + KS - 1;
  constexpr int ROWS = TW * 16;
  constexpr int MAXI = (ROWS + R - 1) / R + 1;
  constexpr int PITCH = KC + 8;  // == 8 (mod 64) dwords: conflict-free ds_read_b128 over 16 rows
  constexpr int C4 = KC / 4;
  constexpr int NSTEP = KS * (KC / 16);
  extern __shared__ __attribute__((aligned(16))) float slab[];

  const int M = a.M;
  const long total = (long)M * R;
  const long gr0 = (long)blockIdx.x * ROWS;
  const long gr1 = min(gr0 + ROWS, total);
  const long i0 = gr0 / R, i1 = (gr1 - 1) / R;
  const long elo = i0 * RX + (gr0 - i0 * R);
  const int nslab = (int)(i1 * RX + (gr1 - 1 - i1 * R) + KS - elo);
  (void)MAXI;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int nout = a.nout;
  constexpr int CT = kRowsCT;  // 16-column MFMA tiles per wave
  const int ocol0 = blockIdx.y * 128 + wave * 16 * CT;
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
    constexpr int FB = SRC == SRC_DZ ? 4 : 8;  // slab slots (float4) in flight per thread
    const int nfill = nslab * C4;
    const int c = 4 * (threadIdx.x % C4);
    __shared__ ChanLds chl;
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
      if constexpr (SRC == SRC_TRACK_F16 || SRC == SRC_TRACK_F32) {
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
    chan_stage<SRC>(a, KC, chl);
    if constexpr (F16) range_stage<SRC>(a, KC, chl);
    if constexpr (SRC != SRC_DZ)
      if (blockIdx.x == 0 && blockIdx.y == 0) bn_publish(a.in_bn, threadIdx.x);
    __syncthreads();
    if constexpr (F16) sscale = split_scale(chl, KC);
    const ChanOps kop = chan_ops<SRC>(chl, c);
    store_batch(threadIdx.x, kop);
    for (int base = threadIdx.x + kRowsThreads * FB; base < nfill; base += kRowsThreads * FB) {
      load_batch(base);
      store_batch(base, kop);
    }
  }
  __syncthreads();
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

  if constexpr (MODE == 1) {
    // g_{l-1} rows, plus this tile's share of BN_{l-1}'s backward sums (sum g, sum g*xhat)
    float sg[CT] = {}, sgx[CT] = {};
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
            float gv = acc[r][ct][j];
            if (a.skip && o < a.skip_n) gv += a.skip[((grb + j) / R) * a.skip_ld + o] * a.skip_scale;
            a.out[(grb + j) * nout + o] = gv;
            sg[ct] += gv;
            sgx[ct] += gv * ((yv[j] - mu) * is);
          }
      }
    }
    if (a.out_acc) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        float s = sg[ct], q = sgx[ct];
        s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
        if (g == 0) {
          const int o = ocol0 + 16 * ct + l16;
          acc128_add(acc_at(a.out_acc, nout, 0, o), s);
          acc128_add(acc_at(a.out_acc, nout, 1, o), q);
        }
      }
    }
  } else {
    constexpr int LP = R / POOL;
    float ssum[CT] = {}, ssq[CT] = {}, ymax[CT] = {};
    const float inv_s = sscale.inv;  // 1 on the f32 path; exact power of two on the split path
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
      for (int ct = 0; ct < CT; ++ct) {
        float s = ssum[ct], q = ssq[ct];
        s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
        if (g == 0) {
          const int o = ocol0 + 16 * ct + l16;
          acc128_add(acc_at(a.out_acc, nout, 0, o), s);
          acc128_add(acc_at(a.out_acc, nout, 1, o), q);
        }
      }
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

template <int L, int KC, int SRC, int TW>
static int fwd_layer_tw(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  static_assert(KC % 32 == 0, "split-f16 chunks are 32 channels");
  if (a.wpack16 && conv_f16_on())
    return run_rows<0, SRC, KC, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, TW, 1, 1, true>(a, s);
  return run_rows<0, SRC, KC, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, TW, 1, 1>(a, s);
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


template <int L, int KC, int SRC>
static int fwd_layer(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int TWMAX = max_tw(gm.lp * gm.pool, gm.ks, KC);
  const int tw = choose_tw((long)a.M * gm.lp * gm.pool, TWMAX);
  if constexpr (TWMAX >= 8) if (tw == 8) return fwd_layer_tw<L, KC, SRC, 8>(a, s);
  if constexpr (TWMAX >= 4) if (tw == 4) return fwd_layer_tw<L, KC, SRC, 4>(a, s);
  if constexpr (TWMAX >= 3) if (tw == 3) return fwd_layer_tw<L, KC, SRC, 3>(a, s);
  if constexpr (TWMAX >= 2) if (tw == 2) return fwd_layer_tw<L, KC, SRC, 2>(a, s);
  return fwd_layer_tw<L, KC, SRC, 1>(a, s);
}

template <int L>
static int fwd_kc(int kc, int src, const RowsArgs& a, hipStream_t s) {
  if constexpr (L == 1) {
    if (kc != kMels) return DCUE_ERR_INVALID;
    return src == SRC_TRACK_F16 ? fwd_layer<1, 128, SRC_TRACK_F16>(a, s)
                                : fwd_layer<1, 128, SRC_TRACK_F32>(a, s);
  } else {
    switch (kc) {
      case 32: return fwd_layer<L, 32, SRC_ACT>(a, s);
      case 64: return fwd_layer<L, 64, SRC_ACT>(a, s);
      case 128: return fwd_layer<L, 128, SRC_ACT>(a, s);
      case 256: return fwd_layer<L, 256, SRC_ACT>(a, s);
      default: return DCUE_ERR_UNSUPPORTED;
    }
  }
}

int launch_conv_fwd(int layer, int kc, int src, const RowsArgs& a, hipStream_t s) {
  switch (layer) {
    case 1: return fwd_kc<1>(kc, src, a, s);
    case 2: return fwd_kc<2>(kc, src, a, s);
    case 3: return fwd_kc<3>(kc, src, a, s);
    case 4: return fwd_kc<4>(kc, src, a, s);
    case 5: return fwd_kc<5>(kc, src, a, s);
    default: return DCUE_ERR_INVALID;
  }
}

// dgrad of layer L: rows = (item, input position t' < Lin_L), slab = layer-L conv positions
// [0, Lp*pool) carrying dz, taps reversed (PADL = ks-1-pad).
template <int L, int KC, int TW>
static int dgrad_layer_tw(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  return run_rows<1, SRC_DZ, KC, gm.ks, gm.ks - 1 - gm.pad, gm.lp * gm.pool, gm.lin, 1, TW, gm.lp,
                  gm.pool>(a, s);
}

template <int L, int KC>
static int dgrad_layer(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int TWMAX = max_tw(gm.lin, gm.ks, KC);
  const int tw = choose_tw((long)a.M * gm.lin, TWMAX);
  if constexpr (TWMAX >= 8) if (tw == 8) return dgrad_layer_tw<L, KC, 8>(a, s);
  if constexpr (TWMAX >= 4) if (tw == 4) return dgrad_layer_tw<L, KC, 4>(a, s);
  if constexpr (TWMAX >= 3) if (tw == 3) return dgrad_layer_tw<L, KC, 3>(a, s);
  if constexpr (TWMAX >= 2) if (tw == 2) return dgrad_layer_tw<L, KC, 2>(a, s);
  return dgrad_layer_tw<L, KC, 1>(a, s);
}

template <int L>
static int dgrad_kc(int kc, const RowsArgs& a, hipStream_t s) {
  switch (kc) {
    case 32: return dgrad_layer<L, 32>(a, s);
    case 64: return dgrad_layer<L, 64>(a, s);
    case 128: return dgrad_layer<L, 128>(a, s);
    case 256: return dgrad_layer<L, 256>(a, s);
    default: return DCUE_ERR_UNSUPPORTED;
  }
}

int launch_conv_dgrad(int layer, int kc, const RowsArgs& a, hipStream_t s) {
  switch (layer) {
    case 2: return dgrad_kc<2>(kc, a, s);
    case 3: return dgrad_kc<3>(kc, a, s);
    case 4: return dgrad_kc<4>(kc, a, s);
    case 5: return dgrad_kc<5>(kc, a, s);
    default: return DCUE_ERR_INVALID;
  }
}

// ------------------------------------------------------------------------------------ wgrad
static constexpr int kWgradRch = 72;  // rows per chunk step (9 per thread)

// dW[o][k*cin+c] = sum over conv rows (i,t) of dz[i][t][o] * x[i][t+k-pad][c]: a GEMM whose K is
// the row dimension. Workgroup = 128 (o) x 128 (kc) output block x one chunk of rows; the chunk is
// streamed through LDS RCH rows at a time (dz and x tiles, both built by fused elementwise loads);
// each wave owns a 64x64 block (4x4 MFMA tiles). Partial blocks per chunk are summed by
// k_wgrad_reduce in a fixed order (deterministic). EDGES (layer 1) also accumulates the per-output
// sums of dz at the first/last two positions: with them the reduce recovers, per tap, the sum of dz
// over positions whose input is not zero padding -- what bn0's beta gradient and the bn0 affine
// split of dW1 need ("bn0 without conv1 dgrad").
// The body takes its block coordinates (kc tile bx, o tile by, chunk bz) as arguments: k_conv_wgrad
// runs one layer per launch, k_conv_wgrad_multi the weight gradients of layers 2-5 in one launch.
template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP, int RCH, bool EDGES>
__device__ __forceinline__ void wgrad_body(const WgradArgs& a, int bx, int by, int bz, float* lds) {
  constexpr int PW = 128 + 16;  // == 16 (mod 32): ds_read_b32 rows r and r+1 on disjoint banks
  constexpr int NB = EDGES ? 5 : 1;
  constexpr int FR = RCH / 8;   // rows per thread per chunk step (8 row slots x 32 channel quads)
  constexpr bool TRACK = SRCX == SRC_TRACK_F16 || SRCX == SRC_TRACK_F32;
  float* dzs = lds;
  float* xs = lds + RCH * PW;
  float (*bsum)[NB][128] = reinterpret_cast<float (*)[NB][128]>(lds + 2 * RCH * PW);  // [8][NB][128]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int wo = wave >> 1, wk = wave & 1;
  const int cout = a.cout, cin = a.cin, kcn = KS * cin;
  const int obase = by * 128, kcbase = bx * 128;
  const long total = (long)a.M * R;
  const long r_begin = (long)bz * a.rows_per_chunk;
  const long r_end = min(r_begin + a.rows_per_chunk, total);
  const bool do_bias = bx == 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bacc[NB];
#pragma unroll
  for (int e = 0; e < NB; ++e) bacc[e] = make_float4(0.f, 0.f, 0.f, 0.f);

  // this thread fills channel quad q (dz outputs o..o+3, x columns kc..kc+3) of row slots
  // slot, slot+8, ...; everything per channel is loaded once, out of the row loop
  const int q = tid & 31, slot = tid >> 5;
  const int o = obase + 4 * q, kc = kcbase + 4 * q;
  const bool o_ok = o < cout, kc_ok = kc < kcn;
  const int oc = o_ok ? o : 0, kcc = kc_ok ? kc : 0;
  const int kx = kcc / cin, cx = kcc - kx * cin;
  const float4 mean4 = ld4(a.mean_l + oc), inv4 = ld4(a.invstd_l + oc), a4 = ld4(a.a_l + oc);
  float4 sD4, sDx4;
  {
    float sd[4], sdx[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sd[s] = (float)acc_sum(a.dz_acc, cout, 0, oc + s);
      sdx[s] = (float)acc_sum(a.dz_acc, cout, 1, oc + s);
    }
    sD4 = make_float4(sd[0], sd[1], sd[2], sd[3]);
    sDx4 = make_float4(sdx[0], sdx[1], sdx[2], sdx[3]);
  }
  if (bx == 0 && by == 0 && bz == 0 && tid < cout) {
    // BN_l = gamma * xhat + beta: dbeta = sum g, dgamma = sum g * xhat
    a.dbeta[tid] = (float)acc_sum(a.dz_acc, cout, 0, tid);
    a.dgamma[tid] = (float)acc_sum(a.dz_acc, cout, 1, tid);
  }
  const float4 xmu = ld4(a.x_mean + cx), xsc = ld4(a.x_a + cx);
  const float4 xbe = a.x_beta ? ld4(a.x_beta + cx) : make_float4(0.f, 0.f, 0.f, 0.f);

  // raw operands of one chunk step, loaded branch-free (clamped addresses, masks applied later)
  float4 rg[FR], ry[FR], rx[FR];
  uint32_t rid[FR];
  float rcnt[FR];
  auto issue = [&](long rb) {
    long ii[FR];
    int tt[FR], pc[FR];
    int trk[FR];
#pragma unroll
    for (int j = 0; j < FR; ++j) {
      long row = rb + slot + 8 * j;
      row = row < r_end ? row : r_begin;
      ii[j] = row / R;
      tt[j] = (int)(row - ii[j] * R);
      const int p = tt[j] + kx - PAD;
      pc[j] = p < 0 ? 0 : (p >= LIN ? LIN - 1 : p);
    }
    if constexpr (TRACK) {
#pragma unroll
      for (int j = 0; j < FR; ++j) trk[j] = a.item_track[ii[j]];
    }
#pragma unroll
    for (int j = 0; j < FR; ++j) {
      const long base = (ii[j] * LP + tt[j] / POOL) * cout + oc;
      rg[j] = ld4(a.g_l + base);
      ry[j] = ld4(a.y_l + base);
      rid[j] = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
      rcnt[j] = a.counts ? a.counts[ii[j]] : 1.f;
      if constexpr (SRCX == SRC_TRACK_F16) {
        const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.xsrc) +
                                                          (((long)trk[j] * kFrames + pc[j]) * kMels + cx));
        rx[j] = make_float4(__uint_as_float(raw.x), __uint_as_float(raw.y), 0.f, 0.f);
      } else if constexpr (SRCX == SRC_TRACK_F32) {
        rx[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + (((long)trk[j] * kFrames + pc[j]) * kMels + cx));
      } else {
        rx[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + ((ii[j] * LIN + pc[j]) * cin + cx));
      }
    }
  };

  issue(r_begin);
  for (long rb = r_begin; rb < r_end; rb += RCH) {
    // dz (BN_l backward through relu + max-pool, as RowsArgs) and x (BN_{l-1} affine) -> LDS
#pragma unroll
    for (int j = 0; j < FR; ++j) {
      const long row = rb + slot + 8 * j;
      const bool valid = row < r_end;
      const long rowc = valid ? row : r_begin;
      const long ii = rowc / R;
      const int t = (int)(rowc - ii * R), jp = t % POOL;
      const int p = t + kx - PAD;
      float4 dz = make_float4(0.f, 0.f, 0.f, 0.f), xv = dz;
      if (valid && o_ok) {
        const float kD = rcnt[j] * a.invN;
        const float gv[4] = {rg[j].x, rg[j].y, rg[j].z, rg[j].w};
        const float yv[4] = {ry[j].x, ry[j].y, ry[j].z, ry[j].w};
        const float mu[4] = {mean4.x, mean4.y, mean4.z, mean4.w}, iv[4] = {inv4.x, inv4.y, inv4.z, inv4.w};
        const float av[4] = {a4.x, a4.y, a4.z, a4.w}, sd[4] = {sD4.x, sD4.y, sD4.z, sD4.w};
        const float sdx[4] = {sDx4.x, sDx4.y, sDx4.z, sDx4.w};
        float r4[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float xh = (yv[s] - mu[s]) * iv[s];
          const float dx = av[s] * (gv[s] - kD * sd[s] - kD * xh * sdx[s]);
          r4[s] = (((rid[j] >> (8 * s)) & 0xff) == (uint32_t)jp && yv[s] > 0.f) ? dx : 0.f;
        }
        dz = make_float4(r4[0], r4[1], r4[2], r4[3]);
        if (do_bias) {
          bacc[0].x += dz.x; bacc[0].y += dz.y; bacc[0].z += dz.z; bacc[0].w += dz.w;
          if constexpr (EDGES) {  // static indices only: keeps bacc[] in registers
            const int e = t == 0 ? 1 : t == 1 ? 2 : t == R - 2 ? 3 : t == R - 1 ? 4 : 0;
#pragma unroll
            for (int k = 1; k < NB; ++k) {
              const float f = e == k ? 1.f : 0.f;
              bacc[k].x += f * dz.x; bacc[k].y += f * dz.y; bacc[k].z += f * dz.z; bacc[k].w += f * dz.w;
            }
          }
        }
      }
      if (valid && kc_ok && p >= 0 && p < LIN) {
        float x[4];
        if constexpr (SRCX == SRC_TRACK_F16) {
          const uint32_t lo = __float_as_uint(rx[j].x), hi = __float_as_uint(rx[j].y);
          const __half2 h0 = *reinterpret_cast<const __half2*>(&lo);
          const __half2 h1 = *reinterpret_cast<const __half2*>(&hi);
          x[0] = __low2float(h0); x[1] = __high2float(h0); x[2] = __low2float(h1); x[3] = __high2float(h1);
        } else {
          x[0] = rx[j].x; x[1] = rx[j].y; x[2] = rx[j].z; x[3] = rx[j].w;
        }
        xv = make_float4((x[0] - xmu.x) * xsc.x + xbe.x, (x[1] - xmu.y) * xsc.y + xbe.y,
                         (x[2] - xmu.z) * xsc.z + xbe.z, (x[3] - xmu.w) * xsc.w + xbe.w);
      }
      const int rr = slot + 8 * j;
      st4(&dzs[rr * PW + 4 * q], dz);
      st4(&xs[rr * PW + 4 * q], xv);
    }
    __syncthreads();
    if (rb + RCH < r_end) issue(rb + RCH);  // next step's loads fly while the MFMAs run
    const int nr = (int)min((long)RCH, (r_end - rb + 3) & ~3L);  // rows of this step, padded to 4
    for (int r0 = 0; r0 < nr; r0 += 4) {
      float av[4], bv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) av[m] = dzs[(r0 + g) * PW + 64 * wo + 16 * m + l16];
#pragma unroll
      for (int n = 0; n < 4; ++n) bv[n] = xs[(r0 + g) * PW + 64 * wk + 16 * n + l16];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma4(av[m], bv[n], acc[m][n]);
    }
    __syncthreads();
  }

  // partial block -> wpart[z][o][kc]; D lane map: o = 4g + reg, kc = l16
  float* wp = a.wpart + (size_t)bz * cout * kcn;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int kc = kcbase + 64 * wk + 16 * n + l16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = obase + 64 * wo + 16 * m + 4 * g + j;
        if (o < cout && kc < kcn) wp[(size_t)o * kcn + kc] = acc[m][n][j];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < NB; ++e) st4(&bsum[slot][e][4 * q], bacc[e]);
    __syncthreads();
    if (tid < 128 && obase + tid < cout) {
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < 8; ++sl) v += bsum[sl][e][tid];
        a.bpart[((size_t)bz * NB + e) * cout + obase + tid] = v;
      }
    }
  }
}

// LDS floats of the weight-gradient body: the dz and x tiles, then the bias partial sums
constexpr size_t wgrad_lds_floats(int nb) { return (size_t)2 * kWgradRch * (128 + 16) + 8 * nb * 128; }

template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP, int RCH, bool EDGES>
__global__ __launch_bounds__(256) void k_conv_wgrad(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  wgrad_body<SRCX, KS, PAD, LIN, R, POOL, LP, RCH, EDGES>(a, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

// Weight gradients of several conv layers (of 2..5) in one launch: a 1-D grid of the layers'
// (kc tile, o tile, chunk) blocks in slot order; each layer keeps its own partial buffers, summed by
// k_wgrad_reduce_multi.
template <int L>
__device__ __forceinline__ void wgrad_multi_layer(const WgradMulti& w, int j, int b, float* lds) {
  constexpr LayerGeom gm = layer_geom(L);
  const int kt = w.kt[j], ot = w.ot[j];
  wgrad_body<SRC_ACT, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, gm.lp, kWgradRch, false>(
      w.a[j], b % kt, (b / kt) % ot, b / (kt * ot), lds);
}

__global__ __launch_bounds__(256) void k_conv_wgrad_multi(WgradMulti w) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < w.n && b >= w.start[j + 1]) ++j;
  switch (w.layer[j]) {
    case 2: wgrad_multi_layer<2>(w, j, b - w.start[j], lds); break;
    case 3: wgrad_multi_layer<3>(w, j, b - w.start[j], lds); break;
    case 4: wgrad_multi_layer<4>(w, j, b - w.start[j], lds); break;
    default: wgrad_multi_layer<5>(w, j, b - w.start[j], lds); break;
  }
}


// Layer-1 weight gradient (the step's largest MFMA kernel). The GEMM is
// dW1[o][kc] = sum over conv-1 rows (item, t) of dz1[row][o] * xhat0[item][t + kx - 2][c], K = M*132
// rows, kc = kx*128 + c. dz1 is BN1's backward through relu + max-pool: of each pool window's four
// rows only the argmax row carries the window's gradient dx1[window][o]. The operands therefore stay
// compact in HBM -- xhat0 (k_xhat0, zero-padded so every tap row exists) and the pooled dx1
// (k_conv1_dx) plus the pool argmax bytes -- and the dz1 fragment is expanded at MFMA time:
// a = (argmax[window][o] == row & 3) ? dx1[window][o] : 0.
// Workgroup = a 64 (o) x 64 (kc) output tile x one chunk of pool windows, 8 waves: wave w owns the
// (w>>1 & 1, w & 1) 32x32 quarter over half of each step's 32 windows (w >> 2), two
// v_mfma_f32_32x32x2_f32 per window. The LDS stages are filled by global_load_lds_dwordx4
// (no register staging): step s+PD's loads are issued behind step s's first MFMAs and retired by a
// counted vmcnt before the raw barrier that ends step s+1; a window's LDS operands are read one
// window ahead of its MFMAs. In the bias workgroups (kc tile 0) the waves also sum dx1 per channel
// -- all rows and the four edge positions t = 0, 1, 130, 131.
constexpr int kW1Tile = 64;                      // 64 (o) x 64 (kc) output tile
constexpr int kW1Win = 16;                       // pool windows (64 conv rows) per step
constexpr int kW1Half = kW1Win / 2;              // windows per wave per step (two k halves)
constexpr int kW1XPW = kW1Win / 8;               // x pieces (4 rows, 1 KB) per wave per step
constexpr int kW1DW = kW1Win / 4;                // waves loading a dx1 piece (4 windows)
constexpr int kW1AW = kW1Win / 16;               // waves loading an argmax piece (16 windows)
constexpr int kW1XF = kW1Win * 4 * kW1Tile;      // x stage: [128 rows][64 kc] floats, quad-swizzled
constexpr int kW1DF = kW1Win * kW1Tile;          // dx1 stage: [32 windows][64 o]
constexpr int kW1AF = kW1Win * kW1Tile / 4;      // argmax stage: [32 windows][64 o] bytes
constexpr int kW1StageF = kW1XF + kW1DF + kW1AF; // 5376 floats = 21 KB: two workgroups per CU
#ifndef DCUE_W1_STAGES
#define DCUE_W1_STAGES 2
#endif
#ifndef DCUE_W1_WGS
#define DCUE_W1_WGS 2
#endif
// LDS stages; loads run kW1Stages - 1 steps ahead. Measured at two workgroups per CU, two stages
// (42 KB) match three (catalogue 271 vs 277 us, in-batch 22.6 vs 25.1 us) and leave LDS to the
// kernels that run beside it; workgroup counts of 768 or 1024 gain nothing over 512.
constexpr int kW1Stages = DCUE_W1_STAGES;
constexpr int kW1PD = kW1Stages - 1;
static_assert(kW1PD >= 1 && kW1PD <= 2, "wait_stage counts one or two steps in flight");

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void glds16(const void* g, float* l) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)l, 16, 0, 0);
}

__global__ __launch_bounds__(512, DCUE_W1_WGS) void k_conv1_wgrad(WgradArgs a) {
  critical_path_priority();
  constexpr int R = 132, LP = 33, NB = 5;
  static_assert(kW1Win % 16 == 0 && kW1DW + kW1AW <= 8, "load assignment");
  extern __shared__ __attribute__((aligned(16))) float lds[];  // the only LDS object: a second
                                                                // one makes hipcc drain the loads
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cout = a.cout, kcn = 4 * kMels;
  // grid (chunk, kc tile, o tile): consecutive workgroup ids -- dispatched round-robin over the 8
  // XCDs -- are different chunks, so all tiles of one chunk share an XCD and its L2 serves their
  // re-reads of the chunk's rows (8 kc tiles read the same dx1, 2 o tiles the same xhat0 rows)
  const int chunk = blockIdx.x, ktile = blockIdx.y, otile = blockIdx.z;
  const int obase = otile * kW1Tile, kbase = ktile * kW1Tile;
  const int kx = kbase / kMels, cbase = kbase - kx * kMels;
  const int nwin = a.M * LP;
  const int w_begin = min(chunk * (a.rows_per_chunk / 4), nwin);
  const int w_end = min(w_begin + a.rows_per_chunk / 4, nwin);
  const int nsteps = (w_end - w_begin + kW1Win - 1) / kW1Win;
  const bool do_bias = ktile == 0;
  const float* xp = reinterpret_cast<const float*>(a.xsrc);  // [M + 1][kXp][128], zero pads
  const float* dx1 = a.g_l;                                   // [M*33][cout]
  const uint8_t* arg = a.idx_l;                               // [M*33][cout]

  // ---- stage loads (1 KB pieces): per step every wave issues kW1XPW x pieces (rows
  // 4 kW1XPW w + 4h .. +3), waves 0 .. kW1DW-1 one dx1 piece (windows 4w .. 4w+3) and the next
  // kW1AW waves one argmax piece (16 windows)
  const bool dxw = w < kW1DW, agw = w >= kW1DW && w < kW1DW + kW1AW;
  const int nload = kW1XPW + (dxw ? 1 : 0) + (agw ? 1 : 0);
  int xi[kW1XPW], xt[kW1XPW];  // row cursors (item, frame) of the lane's x pieces; rows past the
                               // end read the next chunk's rows or the zero item M (unused)
#pragma unroll
  for (int h = 0; h < kW1XPW; ++h) {
    const int r = 4 * w_begin + 4 * kW1XPW * w + 4 * h + (lane >> 4);
    xi[h] = r / R;
    xt[h] = r - xi[h] * R;
  }
  const int xq = (lane & 15) ^ ((lane >> 4 & 1) << 3);  // row-parity quad swizzle (32-lane reads)
  auto issue = [&](int step) {
    float* st = lds + (step % kW1Stages) * kW1StageF;
    const int win0 = w_begin + step * kW1Win;
#pragma unroll
    for (int h = 0; h < kW1XPW; ++h) {
      glds16(xp + ((size_t)(xi[h] * kXp + xt[h] + kx) * kMels + cbase + 4 * xq), st + (kW1XPW * w + h) * 256);
      xt[h] += 4 * kW1Win;
      if (xt[h] >= R) { xt[h] -= R; ++xi[h]; }
    }
    if (dxw) {
      const int wl = win0 + 4 * w + (lane >> 4), o = obase + 4 * (lane & 15);
      const bool ok = wl < w_end && o < cout;  // else xhat0's zero pad row
      glds16(ok ? (const void*)(dx1 + (size_t)wl * cout + o) : (const void*)(xp + 4 * (lane & 15)),
             st + kW1XF + w * 256);
    }
    if (agw) {
      const int wa = w - kW1DW;
      const int wl = min(win0 + 16 * wa + (lane >> 2), nwin - 1);
      const int ob = min(obase + 16 * (lane & 3), cout - 16);
      glds16(arg + (size_t)wl * cout + ob, st + kW1XF + kW1DF + wa * 256);
    }
  };
  auto wait_stage = [&](bool one_in_flight) {  // retire all but the newest step's loads
    if (!one_in_flight) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (nload == kW1XPW + 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kW1XPW + 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kW1XPW) : "memory");
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  if (chunk == 0 && ktile == 0 && otile == 0 && tid < cout) {  // BN1's gamma/beta gradients
    a.dbeta[tid] = (float)acc_sum(a.dz_acc, cout, 0, tid);
    a.dgamma[tid] = (float)acc_sum(a.dz_acc, cout, 1, tid);
  }

  // ---- MFMA: lane (hl = lane >> 5, l32) holds A[o = l32][row 2h + hl] and B[row 2h + hl][kc = l32]
  const int hl = lane >> 5, l32 = lane & 31;
  const int wo = (w >> 1) & 1, wk = w & 1, hk = w >> 2;
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  float bacc[NB] = {0.f, 0.f, 0.f, 0.f, 0.f};
  const int ao = 32 * wo + l32;                                    // A element's channel in the tile
  const int bx0 = hl * kW1Tile + 4 * ((8 * wk + (l32 >> 2)) ^ (hl << 3)) + (l32 & 3);  // row 2h + hl
  struct Ops { float d, b0, b1; int g; };
  auto ops = [&](const float* st, int kk) {
    const float* dxs = st + kW1XF;
    const uint8_t* ags = reinterpret_cast<const uint8_t*>(st + kW1XF + kW1DF);
    const float* xr = st + 4 * kk * kW1Tile + bx0;
    return Ops{dxs[kk * kW1Tile + ao], xr[0], xr[2 * kW1Tile], (int)ags[kk * kW1Tile + ao]};
  };
  auto mma2 = [&](const Ops& p) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(p.g == hl ? p.d : 0.f, p.b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(p.g == 2 + hl ? p.d : 0.f, p.b1, acc, 0, 0, 0);
  };
  auto bias = [&](const float* st, int win0, int nw) {  // channel tid & 63 of windows w + 8u
    const float* dxs = st + kW1XF;
    const uint8_t* ags = reinterpret_cast<const uint8_t*>(st + kW1XF + kW1DF);
    const int ch = tid & 63;
#pragma unroll
    for (int u = 0; u < kW1Win / 8; ++u) {
      const int kk = w + 8 * u;
      if (kk >= nw) break;
      const float v = dxs[kk * kW1Tile + ch];
      const int t = 4 * ((win0 + kk) % LP) + ags[kk * kW1Tile + ch];
      bacc[0] += v;
      bacc[1] += t == 0 ? v : 0.f;
      bacc[2] += t == 1 ? v : 0.f;
      bacc[3] += t == R - 2 ? v : 0.f;
      bacc[4] += t == R - 1 ? v : 0.f;
    }
  };

  // Pipeline over stages step % kW1Stages, PD = kW1Stages - 1 steps ahead: step s+PD goes into the
  // stage step s-1 read (every wave's reads of it retired before the barrier that ended step s-1);
  // the wait ending step s retires step s+1's loads (each wave its own, the barrier then publishes
  // them to all).
  for (int q = 0; q < kW1PD && q < nsteps; ++q) issue(q);
  wait_stage(kW1PD > 1 && nsteps > 1);
  barrier();
  for (int s = 0; s < nsteps; ++s) {
    const float* st = lds + (s % kW1Stages) * kW1StageF;
    const bool more = s + kW1PD < nsteps;
    const int win0 = w_begin + s * kW1Win;
    const int nw = min(kW1Win, w_end - win0);
    const int kn = min(max(nw - kW1Half * hk, 0), kW1Half);  // this wave's windows
    if (kn == kW1Half) {  // every step but a chunk's last: unrolled, operands read ahead freely
      // two windows of read-ahead, pinned: a window's LDS reads are issued two MFMA pairs
      // (256 pipe cycles) before their use
      Ops q0 = ops(st, kW1Half * hk), q1 = ops(st, kW1Half * hk + 1);
#pragma unroll
      for (int k = 0; k < kW1Half; ++k) {
        const Ops q2 = ops(st, kW1Half * hk + (k < kW1Half - 2 ? k + 2 : kW1Half - 1));
        __builtin_amdgcn_sched_barrier(0);
        mma2(q0);
        __builtin_amdgcn_sched_barrier(0);
        if (k == 0 && more) issue(s + kW1PD);  // behind the first MFMAs: the pipe stays fed
        q0 = q1;
        q1 = q2;
      }
    } else {  // a chunk's last step (never followed by loads)
      for (int k = 0; k < kn; ++k) mma2(ops(st, kW1Half * hk + k));
    }
    if (do_bias) bias(st, win0, nw);
    wait_stage(kW1PD > 1 && more);
    barrier();
  }

  // ---- epilogue: k-halves summed through LDS (the stages are free: no load in flight)
  float* red = lds;                          // [64 o][64 kc] of waves 4-7
  float* bsum = lds + kW1Tile * kW1Tile;     // [8 waves][NB][64]
  // D lane map (32x32): o = (j & 3) + 8 (j >> 2) + 4 hl, kc = l32
  if (hk == 1) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      red[(32 * wo + (j & 3) + 8 * (j >> 2) + 4 * hl) * kW1Tile + 32 * wk + l32] = acc[j];
  }
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < NB; ++e) bsum[(w * NB + e) * kW1Tile + (tid & 63)] = bacc[e];
  }
  __syncthreads();
  if (hk == 0) {
    float* wp = a.wpart + (size_t)chunk * cout * kcn;
    const int kl = 32 * wk + l32;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int ol = 32 * wo + (j & 3) + 8 * (j >> 2) + 4 * hl;
      if (obase + ol < cout) wp[(size_t)(obase + ol) * kcn + kbase + kl] = acc[j] + red[ol * kW1Tile + kl];
    }
  }
  if (do_bias && tid < NB * kW1Tile) {  // one (sum, channel) per thread, its 8 wave slots
    const int e = tid / kW1Tile, c = tid - e * kW1Tile;
    float v[8];
#pragma unroll
    for (int sl = 0; sl < 8; ++sl) v[sl] = bsum[(sl * NB + e) * kW1Tile + c];
    const float sum = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    if (obase + c < cout) a.bpart[((size_t)chunk * NB + e) * cout + obase + c] = sum;
  }
}

static int conv1_wgrad(const WgradArgs& a0, int nchunk, hipStream_t s) {
  constexpr size_t LDS = (size_t)kW1Stages * kW1StageF * sizeof(float);
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv1_wgrad, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)LDS));
    attr = true;
  }
  if (a0.cout % 16 != 0) return DCUE_ERR_UNSUPPORTED;  // argmax rows are loaded 16 channels at a time
  WgradArgs a = a0;
  const long wins = (long)a.M * 33;
  a.rows_per_chunk = (int)(4L * ((wins + nchunk - 1) / nchunk));  // whole pool windows
  dim3 grid((unsigned)nchunk, (unsigned)(4 * kMels / kW1Tile), (unsigned)((a.cout + kW1Tile - 1) / kW1Tile));
  DCUE_LAUNCH(k_conv1_wgrad, grid, dim3(512), LDS, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// BN1's backward through relu at the pooled positions: dx1[window][o] = a_o (g - kD sum_g - kD xhat
// sum_gxhat), zero where the pooled activation is not positive; kD = copies(item) / N. Grid-stride
// over channel quads of windows; each block finalizes the per-channel sums once, into LDS.
__global__ __launch_bounds__(256) void k_conv1_dx(WgradArgs a, float* __restrict__ dx1) {
  critical_path_priority();
  constexpr int LP = 33;
  __shared__ float s_sd[256], s_sdx[256];
  for (int c = threadIdx.x; c < a.cout; c += blockDim.x) {
    s_sd[c] = (float)acc_sum(a.dz_acc, a.cout, 0, c);
    s_sdx[c] = (float)acc_sum(a.dz_acc, a.cout, 1, c);
  }
  __syncthreads();
  const int cq = a.cout / 4;
  const long n = (long)a.M * LP * cq;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int o = 4 * (int)(e % cq);
    const long win = e / cq;
    const int item = (int)(win / LP);
    const float kD = (a.counts ? a.counts[item] : 1.f) * a.invN;
    const float4 g = ld4(a.g_l + win * a.cout + o), y = ld4(a.y_l + win * a.cout + o);
    const float4 mu = ld4(a.mean_l + o), iv = ld4(a.invstd_l + o), av = ld4(a.a_l + o);
    const float gv[4] = {g.x, g.y, g.z, g.w}, yv[4] = {y.x, y.y, y.z, y.w};
    const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, i4[4] = {iv.x, iv.y, iv.z, iv.w};
    const float a4[4] = {av.x, av.y, av.z, av.w};
    float d[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float xh = (yv[s] - m4[s]) * i4[s];
      const float dx = a4[s] * (gv[s] - kD * s_sd[o + s] - kD * xh * s_sdx[o + s]);
      d[s] = yv[s] > 0.f ? dx : 0.f;
    }
    st4(dx1 + win * a.cout + o, make_float4(d[0], d[1], d[2], d[3]));
  }
}

int launch_conv1_dx(const WgradArgs& a, float* dx1, hipStream_t s) {
  if (a.cout > 256 || a.cout % 4) return DCUE_ERR_UNSUPPORTED;
  const long n = (long)a.M * 33 * (a.cout / 4);
  const long blocks = (n + 255) / 256;
  DCUE_LAUNCH(k_conv1_dx, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, s, a, dx1);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// bn0(x) without its affine, zero-padded for the conv-1 taps: xhat0[i][p][c] for p = t + 2 (t the
// frame), rows p < 2 and p > 132 zero. One thread per channel quad of a padded row.
template <int SRC>
__global__ __launch_bounds__(256) void k_xhat0(const void* __restrict__ tracks, const int32_t* __restrict__ item_track,
                                               int M, const unsigned long long* acc0, double count,
                                               double inv_count, float* __restrict__ xhat0) {
  __shared__ float s_mu[kMels], s_is[kMels];
  if (threadIdx.x < kMels) {
    if (acc0) {
      const BnChan st = bn_chan_train(acc0, kMels, threadIdx.x, count, inv_count);
      s_mu[threadIdx.x] = st.mean;
      s_is[threadIdx.x] = st.invstd;
    } else {  // towers without bn0: the raw input
      s_mu[threadIdx.x] = 0.f;
      s_is[threadIdx.x] = 1.f;
    }
  }
  __syncthreads();
  const long n4 = (long)(M + 1) * kXp * (kMels / 4);  // item M: zeros
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += (long)gridDim.x * blockDim.x) {
    const int c = 4 * (int)(e % (kMels / 4));
    const long row = e / (kMels / 4);  // item * kXp + p
    const long i = row / kXp;
    const int t = (int)(row - i * kXp) - 2;
    float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t >= 0 && t < kFrames && i < M) {
      const long src = ((long)item_track[i] * kFrames + t) * kMels + c;
      float x[4];
      if constexpr (SRC == SRC_TRACK_F16) {
        const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(tracks) + src);
        const __half2 h0 = *reinterpret_cast<const __half2*>(&raw.x);
        const __half2 h1 = *reinterpret_cast<const __half2*>(&raw.y);
        x[0] = __low2float(h0); x[1] = __high2float(h0); x[2] = __low2float(h1); x[3] = __high2float(h1);
      } else {
        const float4 v = ld4(reinterpret_cast<const float*>(tracks) + src);
        x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
      }
      out = make_float4((x[0] - s_mu[c]) * s_is[c], (x[1] - s_mu[c + 1]) * s_is[c + 1],
                        (x[2] - s_mu[c + 2]) * s_is[c + 2], (x[3] - s_mu[c + 3]) * s_is[c + 3]);
    }
    st4(xhat0 + 4 * e, out);
  }
}

int launch_xhat0(int src, const void* tracks, const int32_t* item_track, int M, const unsigned long long* acc0,
                 double count, float* xhat0, hipStream_t s) {
  const long n4 = (long)(M + 1) * kXp * (kMels / 4);
  const long blocks = (n4 + 255) / 256;
  const dim3 grid((unsigned)(blocks < 2048 ? blocks : 2048));
  if (src == SRC_TRACK_F16)
    DCUE_LAUNCH(k_xhat0<SRC_TRACK_F16>, grid, dim3(256), 0, s, tracks, item_track, M, acc0, count, 1.0 / count, xhat0);
  else
    DCUE_LAUNCH(k_xhat0<SRC_TRACK_F32>, grid, dim3(256), 0, s, tracks, item_track, M, acc0, count, 1.0 / count, xhat0);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int wgrad_nchunk(int layer, int M, int cout, int cin) {
  // one workgroup per CU (LDS-bound): at most 256 / tiles chunks, each of >= 64 rows; partial
  // blocks cost a write + a read of cout*ks*cin floats per chunk
  const LayerGeom gm = layer_geom(layer);
  const long rows = (long)M * gm.lp * gm.pool;
  if (layer == 1) {  // k_conv1_wgrad: 64x64 tiles, >= 4 steps per chunk, <= ~512 workgroups (2 per CU)
    // tuning diagnostic: DCUE_W1_CHUNKS=n caps the split-K chunk count (A/B runs; the workspace is
    // sized through this same function, so it follows)
    static const long forced = [] {
      const char* e = getenv("DCUE_W1_CHUNKS");
      const long v = e ? atol(e) : 0;
      return v >= 1 && v <= 64 ? v : 0L;
    }();
    const long tiles1 = (4L * kMels / kW1Tile) * ((cout + kW1Tile - 1) / kW1Tile);
    long n = forced ? forced : 512 / tiles1;
    const long wins = (long)M * gm.lp;
    if (n > (wins + 4 * kW1Win - 1) / (4 * kW1Win)) n = (wins + 4 * kW1Win - 1) / (4 * kW1Win);
    return (int)(n < 1 ? 1 : n);
  }
  const long tiles = ((gm.ks * cin + 127) / 128) * ((cout + 127) / 128);
  long n = 256 / tiles;
  if (n > (rows + 63) / 64) n = (rows + 63) / 64;
  const long cap = (8L << 20) / ((long)cout * gm.ks * cin);
  if (n > cap) n = cap;
  return (int)(n < 1 ? 1 : n);
}

template <int L, int SRCX>
static int wgrad_layer(const WgradArgs& a0, int nchunk, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int R = gm.lp * gm.pool;
  constexpr bool EDGES = L == 1;
  constexpr size_t LDS = wgrad_lds_floats(EDGES ? 5 : 1) * sizeof(float);
  auto kern = k_conv_wgrad<SRCX, gm.ks, gm.pad, gm.lin, R, gm.pool, gm.lp, kWgradRch, EDGES>;
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)LDS));
    attr = true;
  }
  WgradArgs a = a0;
  const long rows = (long)a.M * R;
  const long rpc = (rows + nchunk - 1) / nchunk;  // the last chunk may be short; rows past it are masked
  a.rows_per_chunk = (int)rpc;
  dim3 grid((unsigned)((gm.ks * a.cin + 127) / 128), (unsigned)((a.cout + 127) / 128), (unsigned)nchunk);
  DCUE_LAUNCH(kern, grid, dim3(256), LDS, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_conv_wgrad(int layer, int src, const WgradArgs& a, int nchunk, hipStream_t s) {
  switch (layer) {
    case 1: (void)src; return conv1_wgrad(a, nchunk, s);  // X = xhat0 (k_xhat0), whatever the table dtype
    case 2: return wgrad_layer<2, SRC_ACT>(a, nchunk, s);
    case 3: return wgrad_layer<3, SRC_ACT>(a, nchunk, s);
    case 4: return wgrad_layer<4, SRC_ACT>(a, nchunk, s);
    case 5: return wgrad_layer<5, SRC_ACT>(a, nchunk, s);
    default: return DCUE_ERR_INVALID;
  }
}

// Sum partial blocks over chunks and write reference layout dW[o][c][k], db[o]. A workgroup owns
// 32 float4 columns (128 outputs) x 8 chunk groups; each thread sums its group's chunks with every
// load of a batch of 8 in flight (the chunk count is small, so this is one or two load rounds), and
// the eight group sums are combined in a fixed order (deterministic). The bias (+ layer-1 edge)
// sums use the same shape over the [chunk][nb][cout] bias partials. Layer 1 writes
// G[o][k*cin+c] (the xhat0 contraction) and the five bias sums E[5][o] instead of dW1 and db1
// (k_bn0_grads finishes them).
constexpr int kRedGroups = 8, kRedBatch = 8;

__device__ __forceinline__ float4 sum_chunks(const float* __restrict__ base, size_t stride, int nchunk,
                                             int grp) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z0 = grp; z0 < nchunk; z0 += kRedGroups * kRedBatch) {
    float4 v[kRedBatch];
#pragma unroll
    for (int i = 0; i < kRedBatch; ++i) {
      const int z = z0 + kRedGroups * i;
      v[i] = z < nchunk ? ld4(base + (size_t)z * stride) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < kRedBatch; ++i) {
      acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w;
    }
  }
  return acc;
}

__device__ __forceinline__ float4 combine_groups(float4 (*red)[32], int col) {
  float4 r = red[0][col];
#pragma unroll
  for (int g = 1; g < kRedGroups; ++g) {
    r.x += red[g][col].x; r.y += red[g][col].y; r.z += red[g][col].z; r.w += red[g][col].w;
  }
  return r;
}

__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ wpart, const float* __restrict__ bpart,
                                                  int nchunk, int cout, int cin, int ks, int nb, float* dW,
                                                  float* db, float* G, float* S, long blk) {
  __shared__ float4 red[kRedGroups][32];
  const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long kcn = (long)ks * cin;
  const long nw = (long)cout * kcn;  // multiple of 4 (cin % 32 == 0)
  const long nwblk = (nw + 127) / 128;
  if (blk < nwblk) {
    const long e4 = blk * 128 + 4 * col;
    red[grp][col] = e4 < nw ? sum_chunks(wpart + e4, (size_t)nw, nchunk, grp) : make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (grp == 0 && e4 < nw) {
      const float4 r = combine_groups(red, col);
      if (G) {
        st4(G + e4, r);
      } else {
        const float v[4] = {r.x, r.y, r.z, r.w};
        const long o = e4 / kcn, kc = e4 - o * kcn;
        const long k = kc / cin, c0 = kc - k * cin;
#pragma unroll
        for (int j = 0; j < 4; ++j) dW[(o * cin + c0 + j) * ks + k] = v[j];
      }
    }
    return;
  }
  // bias (+ layer-1 edge) sums: bpart[z][j][o]; a workgroup owns 128 consecutive (j, o) entries
  const long nbo = (long)nb * cout;  // multiple of 4
  const long e4 = (blk - nwblk) * 128 + 4 * col;
  red[grp][col] = e4 < nbo ? sum_chunks(bpart + e4, (size_t)nbo, nchunk, grp) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (grp == 0 && e4 < nbo) st4(G ? S + e4 : db + e4, combine_groups(red, col));
}

__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ wpart,
                                                      const float* __restrict__ bpart, int nchunk,
                                                      int cout, int cin, int ks, int nb, float* dW,
                                                      float* db, float* G, float* S) {
  critical_path_priority();
  wgrad_reduce_body(wpart, bpart, nchunk, cout, cin, ks, nb, dW, db, G, S, blockIdx.x);
}

// the partial sums of k_conv_wgrad_multi, layers 2..5 in one launch (block ranges rstart[])
__global__ __launch_bounds__(256) void k_wgrad_reduce_multi(WgradMulti w) {
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < w.n && b >= w.rstart[j + 1]) ++j;
  const WgradArgs& a = w.a[j];
  wgrad_reduce_body(a.wpart, a.bpart, w.nchunk[j], a.cout, a.cin, layer_geom(w.layer[j]).ks, 1, w.dW[j],
                    w.db[j], nullptr, nullptr, b - w.rstart[j]);
}

int launch_conv_wgrad_multi(WgradMulti w, hipStream_t s) {
  constexpr size_t LDS = wgrad_lds_floats(1) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_wgrad_multi, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)LDS));
    attr = true;
  }
  w.start[0] = 0;
  w.rstart[0] = 0;
  if (w.n < 1 || w.n > 4) return DCUE_ERR_INVALID;
  for (int j = 0; j < w.n; ++j) {
    if (w.layer[j] < 2 || w.layer[j] > 5) return DCUE_ERR_INVALID;
    WgradArgs& a = w.a[j];
    const LayerGeom gm = layer_geom(w.layer[j]);
    if (a.cin % 32 || a.cout % 4) return DCUE_ERR_UNSUPPORTED;
    const long rows = (long)a.M * gm.lp * gm.pool;
    a.rows_per_chunk = (int)((rows + w.nchunk[j] - 1) / w.nchunk[j]);
    w.kt[j] = (gm.ks * a.cin + 127) / 128;
    w.ot[j] = (a.cout + 127) / 128;
    w.start[j + 1] = w.start[j] + w.kt[j] * w.ot[j] * w.nchunk[j];
    w.rstart[j + 1] = w.rstart[j] + (int)(((long)a.cout * gm.ks * a.cin + 127) / 128 + (a.cout + 127) / 128);
  }
  DCUE_LAUNCH(k_conv_wgrad_multi, dim3((unsigned)w.start[w.n]), dim3(256), LDS, s, w);
  DCUE_LAUNCH_CHECK();
  DCUE_LAUNCH(k_wgrad_reduce_multi, dim3((unsigned)w.rstart[w.n]), dim3(256), 0, s, w);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_wgrad_reduce(int layer, const float* wpart, const float* bpart, int nchunk, int cout,
                        int cin, float* dW, float* db, float* G_tmp, float* E_tmp, hipStream_t s) {
  const LayerGeom gm = layer_geom(layer);
  const int nb = layer == 1 ? 5 : 1;
  const long nblk = ((long)cout * gm.ks * cin + 127) / 128 + ((long)nb * cout + 127) / 128;
  // layer 1: the five bias partial sums land in E_tmp[5][cout]; k_bn0_grads derives db1 and S
  DCUE_LAUNCH(k_wgrad_reduce, dim3((unsigned)nblk), dim3(256), 0, s, wpart, bpart, nchunk, cout, cin,
                     gm.ks, nb, dW, db, layer == 1 ? G_tmp : nullptr, layer == 1 ? E_tmp : nullptr);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// bn0 gradients without conv1's input gradient: with xhat0 the normalised input and
// G[o][k*128+c] = sum dz1 * xhat0_pad, S[k][o] = sum of dz1 over rows whose tap-k input is real,
//   dW1[o][c][k] = gamma0[c] G + beta0[c] S,   dgamma0[c] = sum_{o,k} W1 G,   dbeta0[c] = sum_{o,k} W1 S.
__global__ __launch_bounds__(256) void k_bn0_grads(const float* __restrict__ G, const float* __restrict__ E,
                                                   const float* __restrict__ W1, const float* gamma0,
                                                   const float* beta0, int H, float* dW1,
                                                   float* dgamma0, float* dbeta0, float* db1) {
  critical_path_priority();
  // E = the five layer-1 bias-partial sums [5][H]: sum dz1 and its parts at t = 0, 1, R-2, R-1.
  // Tap k of conv row t reads input t+k-2 (zero padding at t+k-2 < 0 or > 130), so
  //   S[0] = e0-e1-e2, S[1] = e0-e1, S[2] = e0-e4, S[3] = e0-e3-e4;  db1 = e0.
  __shared__ float rg[256], rb[256];
  const int c = blockIdx.x, t = threadIdx.x;
  const float ga = gamma0[c], be = beta0[c];
  float dg = 0.f, db = 0.f;
  for (int e = t; e < 4 * H; e += blockDim.x) {  // e = o*4 + k: dW1[o][c][k] layout
    const int o = e >> 2, k = e & 3;
    const float gv = G[(size_t)o * 4 * kMels + k * kMels + c];
    const float e0 = E[o], e1 = E[H + o], e2 = E[2 * H + o], e3 = E[3 * H + o], e4 = E[4 * H + o];
    const float sv = k == 0 ? e0 - e1 - e2 : k == 1 ? e0 - e1 : k == 2 ? e0 - e4 : e0 - e3 - e4;
    const float w = W1[((size_t)o * kMels + c) * 4 + k];
    dg += w * gv;
    db += w * sv;
    dW1[((size_t)o * kMels + c) * 4 + k] = ga * gv + be * sv;
  }
  if (c == 0)
    for (int o = t; o < H; o += blockDim.x) db1[o] = E[o];
  rg[t] = dg;
  rb[t] = db;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) {
      rg[t] += rg[t + off];
      rb[t] += rb[t + off];
    }
    __syncthreads();
  }
  if (t == 0) {
    dgamma0[c] = rg[0];
    dbeta0[c] = rb[0];
  }
}

int launch_bn0_grads(const float* G, const float* E, const float* W1, const float* gamma0,
                     const float* beta0, int H, float* dW1, float* dgamma0, float* dbeta0, float* db1,
                     hipStream_t s) {
  DCUE_LAUNCH(k_bn0_grads, dim3(kMels), dim3(256), 0, s, G, E, W1, gamma0, beta0, H, dW1, dgamma0,
                     dbeta0, db1);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
