// Conv weight gradients (layers 1..5 and the fc), their split-K reduction, the conv-1 operands
// (xhat0, pooled BN1 backward) and bn0's gradients -- gfx950.
// Reference: autograd of the Conv1d / BatchNorm1d layers of truedcuemel1dbn.py:24-101 (nn/dcue.py:208).
#include "dcue_internal.h"
#include "bn0adam.h"

namespace dcue {

// ------------------------------------------------------------------------------------ wgrad
DCUE_KTRACE_READER(wgrad)  // diagnostic builds only (dcue_common.h): kernel 0 = conv-1 wgrad16t, 1 = layer 2, 2 = reduce
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
// RAW: dz is g_l itself (no BatchNorm / ReLU / pool between): the fc layer's weight gradient,
// dW[n][k] = sum over items of df[i][n] bn5(y5)[i][k], run as a 1x1 "conv" (k_conv_wgrad_multi slot
// with layer 6) -- split-K over the items like the convs, where a row-serial small GEMM walked all
// M rows in 16 workgroups.
template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP, int RCH, bool EDGES, bool RAW = false>
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
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 mean4 = RAW ? zero4 : ld4(a.mean_l + oc), inv4 = RAW ? zero4 : ld4(a.invstd_l + oc),
               a4 = RAW ? zero4 : ld4(a.a_l + oc);
  float4 sD4 = zero4, sDx4 = zero4;
  if constexpr (!RAW) {
    float sd[4], sdx[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sd[s] = (float)acc_sum(a.dz_acc, cout, 0, oc + s);
      sdx[s] = (float)acc_sum(a.dz_acc, cout, 1, oc + s);
    }
    sD4 = make_float4(sd[0], sd[1], sd[2], sd[3]);
    sDx4 = make_float4(sdx[0], sdx[1], sdx[2], sdx[3]);
  }
  if (!RAW && bx == 0 && by == 0 && bz == 0 && tid < cout) {
    // BN_l = gamma * xhat + beta: dbeta = sum g, dgamma = sum g * xhat
    a.dbeta[tid] = (float)(acc_sum(a.dz_acc, cout, 0, tid) * bn_grad_scale(a));
    a.dgamma[tid] = (float)(acc_sum(a.dz_acc, cout, 1, tid) * bn_grad_scale(a));
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
      if constexpr (!RAW) {
        ry[j] = ld4(a.y_l + base);
        rid[j] = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
        rcnt[j] = a.counts ? a.counts[ii[j]] : 1.f;
      }
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
      if (valid && o_ok && RAW) {
        dz = rg[j];
        if (do_bias) {
          bacc[0].x += dz.x; bacc[0].y += dz.y; bacc[0].z += dz.z; bacc[0].w += dz.w;
        }
      } else if (valid && o_ok) {
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
template <int L>  // L = 6: the fc layer (a 1x1 conv over bn5(y5) with dz = df, wgrad_body RAW)
__device__ __forceinline__ void wgrad_multi_layer(const WgradMulti& w, int j, int b, float* lds) {
  constexpr LayerGeom gm = layer_geom(L == 6 ? 5 : L);
  const int kt = w.kt[j], ot = w.ot[j];
  wgrad_body<SRC_ACT, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, gm.lp, kWgradRch, false, L == 6>(
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
    case 5: wgrad_multi_layer<5>(w, j, b - w.start[j], lds); break;
    default: wgrad_multi_layer<6>(w, j, b - w.start[j], lds); break;
  }
}


// ------------------------------------------------------------ split-f16 weight gradient
// The same GEMM as wgrad_body, dW[o][kc] = sum over rows of dz[row][o] x[row][kc], on f16 MFMA
// (v_mfma_f32_16x16x32_f16, 16x the f32 MFMA rate): both operands are split into fp16 pairs,
// v = hi + lo (hi = fp16(v), lo = fp16(v - hi)), and each product is hi*hi + lo*hi + hi*lo (the
// dropped lo*lo and the lo roundings are ~2^-22 of the product; f32 accumulation), i.e. three f16
// MFMAs per product at 3/16 of the f32 MFMA time. Every dz column (output channel o) and every x
// column (input channel c) is scaled by its own power of two, 2^e_o and 2^e_c, from a bound of
// the column's largest magnitude -- so the largest value lands in [2^14, 2^15): no fp16 overflow,
// and small gradients (~1e-6) stay clear of fp16's subnormals -- and the epilogue multiplies each
// output by 2^-(e_o + e_c): exact, so the scaling changes no rounding. The bounds (WgradArgs
// x_range, y_range, g_range, kd_max):
//   x = (src - mu) sc + be is monotone in src: its extremes are at the source's min and max (the
//       forward's per-channel value ranges; a ReLU output's min is 0);
//   dz = a (g - kD sD - kD xhat sDx) (masked): |dz| <= |a| (max|g| + kDmax (|sD| + max|xhat| |sDx|)),
//       max|g| from the producing dgrad / item-gradient epilogue, max|xhat| from y_l's range;
//   RAW (fc): |dz| = |df| <= max|df|.
// A loose bound only lowers the scaled maximum: values down to 2^-17 of the bound keep all 22 bits.
// LDS: the four operand images (dz hi/lo, x hi/lo) are [64 rows][128 channels] fp16, 256-byte rows
// with the 16-byte chunks XOR-swizzled (guide T10, layout (b)); the fill writes a thread's four
// channels as one 8-byte store per image, and the MFMA fragments (8 consecutive rows of one
// column: K = rows) come out of ds_read_b64_tr_b16 transposed reads, two per fragment.
typedef short w16_s16x4 __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) w16_s16x4 w16_lds_s16x4;
typedef _Float16 w16_h4 __attribute__((ext_vector_type(4)));
typedef _Float16 w16_h8 __attribute__((ext_vector_type(8)));

constexpr int kW16Rows = 64;                    // rows per LDS stage: two 32-row MFMA k-steps
constexpr int kW16ImgB = kW16Rows * 256;        // bytes per operand image
constexpr size_t kW16LdsB = 4 * kW16ImgB + 2 * 128 * sizeof(int);  // + the column exponents

__device__ __forceinline__ int w16_off(int r, int ch) {  // byte offset of 16-byte chunk ch of row r
  return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}
__device__ __forceinline__ w16_h4 w16_tr(const char* lds, int off) {
  const w16_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (w16_lds_s16x4*)((__attribute__((address_space(3))) char*)lds + off));
  return __builtin_bit_cast(w16_h4, v);
}
__device__ __forceinline__ void w16_split_store(char* hi_img, char* lo_img, int off, float4 v) {
  const w16_h4 h = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
  const w16_h4 l = {(_Float16)(v.x - (float)h[0]), (_Float16)(v.y - (float)h[1]),
                    (_Float16)(v.z - (float)h[2]), (_Float16)(v.w - (float)h[3])};
  *reinterpret_cast<w16_h4*>(hi_img + off) = h;
  *reinterpret_cast<w16_h4*>(lo_img + off) = l;
}
// e with bound * 2^e in [2^14, 2^15); 0 for a zero or non-finite bound
__device__ __forceinline__ int w16_exp(float bound) {
  if (!(bound > 0.f) || !(bound < INFINITY)) return 0;
  int ex;
  (void)frexpf(bound, &ex);
  return min(max(15 - ex, -120), 120);
}
__device__ __forceinline__ float w16_key(const unsigned* keys, int i) {
  const unsigned k = keys ? keys[i] : 0u;
  return k ? ord_value(k) : 0.f;
}

template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP, bool EDGES, bool RAW = false>
__device__ __forceinline__ void wgrad16_body(const WgradArgs& a, int bx, int by, int bz, char* lds) {
  constexpr int RCH = kW16Rows;
  constexpr int NB = EDGES ? 5 : 1;
  constexpr int FR = RCH / 8;          // x rows per thread per stage (8 row slots x 32 channel quads)
  constexpr int FW = RCH / POOL / 8;   // dz pool windows per thread per stage
  static_assert(RCH % (8 * POOL) == 0 && R % POOL == 0, "a stage holds whole pool windows");
  constexpr bool TRACK = SRCX == SRC_TRACK_F16 || SRCX == SRC_TRACK_F32;
  // an fp16 track table is its own exact fp16 operand: one image, no split, one MFMA fewer per
  // product, and bn0's affine (x - mu0) * invstd0 is applied to the reduced sums (k_bn0_grads)
  constexpr bool XRAW = SRCX == SRC_TRACK_F16;
  char* dzh = lds;
  char* dzl = lds + kW16ImgB;
  char* xh = lds + 2 * kW16ImgB;
  char* xl = lds + 3 * kW16ImgB;
  int* exp_o = reinterpret_cast<int*>(lds + 4 * kW16ImgB);
  int* exp_c = exp_o + 128;
  float (*bsum)[NB][128] = reinterpret_cast<float (*)[NB][128]>(lds);  // after the last stage

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int wo = wave >> 1, wk = wave & 1;
  const int cout = a.cout, cin = a.cin, kcn = KS * cin;
  const int obase = by * 128, kcbase = bx * 128;
  const int total = a.M * R;  // rows (the host keeps M * R below 2^31)
  const int r_begin = bz * a.rows_per_chunk;  // a multiple of RCH: stages hold whole windows
  const int r_end = min(r_begin + a.rows_per_chunk, total);
  const bool do_bias = bx == 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bacc[NB];
#pragma unroll
  for (int e = 0; e < NB; ++e) bacc[e] = make_float4(0.f, 0.f, 0.f, 0.f);

  // this thread fills channel quad q (dz outputs o..o+3, x columns kc..kc+3): dz of pool windows
  // slot, slot+8, ... and x of row slots slot, slot+8, ...; everything per channel is set up once
  const int q = tid & 31, slot = tid >> 5;
  const int o = obase + 4 * q, kc = kcbase + 4 * q;
  const bool o_ok = o < cout, kc_ok = kc < kcn;
  const int oc = o_ok ? o : 0, kcc = kc_ok ? kc : 0;
  const int kx = kcc / cin, cx = kcc - kx * cin;
  float mu[4] = {}, iv[4] = {}, av[4] = {}, sd[4] = {}, sdx[4] = {};
  if constexpr (!RAW) {
    const float4 m4 = ld4(a.mean_l + oc), i4 = ld4(a.invstd_l + oc), a4 = ld4(a.a_l + oc);
    mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
    iv[0] = i4.x; iv[1] = i4.y; iv[2] = i4.z; iv[3] = i4.w;
    av[0] = a4.x; av[1] = a4.y; av[2] = a4.z; av[3] = a4.w;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sd[s] = (float)acc_sum(a.dz_acc, cout, 0, oc + s);
      sdx[s] = (float)acc_sum(a.dz_acc, cout, 1, oc + s);
    }
  }
  if (!RAW && bx == 0 && by == 0 && bz == 0 && tid < cout) {
    // BN_l = gamma * xhat + beta: dbeta = sum g, dgamma = sum g * xhat
    a.dbeta[tid] = (float)(acc_sum(a.dz_acc, cout, 0, tid) * bn_grad_scale(a));
    a.dgamma[tid] = (float)(acc_sum(a.dz_acc, cout, 1, tid) * bn_grad_scale(a));
  }
  const float4 xmu = ld4(a.x_mean + cx), xsc = ld4(a.x_a + cx);
  const float4 xbe = a.x_beta ? ld4(a.x_beta + cx) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float xm[4] = {xmu.x, xmu.y, xmu.z, xmu.w}, xs_[4] = {xsc.x, xsc.y, xsc.z, xsc.w};
  const float xb[4] = {xbe.x, xbe.y, xbe.z, xbe.w};

  // the column scales (exponents also to LDS for the epilogue), folded into the per-channel
  // coefficients: scaled dz = cas g - count (cA + xhat cB), scaled x = (src - xm) xas + xbs
  float cas[4], cA[4], cB[4], xas[4], xbs[4];
  {
    int eo[4], ec[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float gmax = w16_key(a.g_range, oc + s);
      float bo;
      if constexpr (RAW) {
        bo = gmax;
      } else {
        const float ym = fmaxf(w16_key(a.y_range, oc + s), 0.f);
        const float xhm = fmaxf(fabsf(mu[s]), fabsf(ym - mu[s])) * iv[s];
        bo = fabsf(av[s]) * (gmax + a.kd_max * (fabsf(sd[s]) + xhm * fabsf(sdx[s])));
      }
      eo[s] = o_ok ? w16_exp(bo) : 0;
      float lo, hi;
      if constexpr (TRACK) {
        lo = -w16_key(a.x_range + kRngC, cx + s);
        hi = w16_key(a.x_range, cx + s);
      } else {
        lo = 0.f;
        hi = fmaxf(w16_key(a.x_range, cx + s), 0.f);
      }
      const float bx_ = fmaxf(fabsf((lo - xm[s]) * xs_[s] + xb[s]), fabsf((hi - xm[s]) * xs_[s] + xb[s]));
      ec[s] = (kc_ok && !XRAW) ? w16_exp(bx_) : 0;
      const float so = ldexpf(1.f, eo[s]), sx = ldexpf(1.f, ec[s]);
      if constexpr (RAW) {
        cas[s] = so; cA[s] = 0.f; cB[s] = 0.f;
      } else {
        cas[s] = av[s] * so;
        cA[s] = av[s] * a.invN * sd[s] * so;
        cB[s] = av[s] * a.invN * sdx[s] * so;
      }
      xas[s] = xs_[s] * sx;
      xbs[s] = xb[s] * sx;
    }
    if (slot == 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        exp_o[4 * q + s] = eo[s];
        exp_c[4 * q + s] = ec[s];
      }
    }
  }
  __syncthreads();  // the exponents are read by other waves' epilogues (even with no stage to run)

  // raw operands of one stage, loaded branch-free (clamped addresses, masks applied at the fill):
  // per pool window g, y, the argmax bytes and the item's count; per x row its four channels
  float4 wg[FW], wy[FW];
  uint32_t wid[FW];
  float wcnt[FW];
  float4 xr[XRAW ? 1 : FR];
  uint2 xr16[XRAW ? FR : 1];
  uint32_t xvalid = 0;
  auto issue = [&](int rb) {
    if constexpr (R >= RCH && TRACK) {
      // layer 1: a stage's rows span at most two items, ia = rb / R and ia + 1 -- one division, two
      // item-id loads and two row bases per stage instead of one of each per row (32-bit offsets
      // for the pooled operands; the table's needs 64 bits)
      const int ia = rb / R, ra = (ia + 1) * R;  // ra: the first row of item ia + 1
      const int ib = min(ia + 1, a.M - 1);
      const float ca = (!RAW && a.counts) ? a.counts[ia] : 1.f, cb = (!RAW && a.counts) ? a.counts[ib] : 1.f;
#pragma unroll
      for (int j = 0; j < FW; ++j) {
        int rw = rb + (slot + 8 * j) * POOL;
        rw = rw < r_end ? rw : rb;
        const bool nb = rw >= ra;
        const int t0 = rw - (nb ? ra : ra - R);
        const int base = ((nb ? ib : ia) * LP + t0 / POOL) * cout + oc;
        wg[j] = ld4(a.g_l + base);
        if constexpr (!RAW) {
          wy[j] = ld4(a.y_l + base);
          wid[j] = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
          wcnt[j] = nb ? cb : ca;
        }
      }
      const long ta = a.item_track[ia], tb = a.item_track[ib];
      uint32_t vm = 0;
#pragma unroll
      for (int j = 0; j < FR; ++j) {
        const int row = rb + slot + 8 * j;
        const int rowc = row < r_end ? row : rb;
        const bool nb = rowc >= ra;
        const int p = rowc - (nb ? ra : ra - R) + kx - PAD;
        vm |= (row < r_end && kc_ok && p >= 0 && p < LIN) ? (1u << j) : 0u;
        const int pc = p < 0 ? 0 : (p >= LIN ? LIN - 1 : p);
        const long e = ((nb ? tb : ta) * kFrames + pc) * kMels + cx;
        if constexpr (XRAW)
          xr16[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.xsrc) + e);
        else
          xr[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + e);
      }
      xvalid = vm;
      return;
    }
#pragma unroll
    for (int j = 0; j < FW; ++j) {
      int rw = rb + (slot + 8 * j) * POOL;
      rw = rw < r_end ? rw : r_begin;
      const int ii = rw / R, t0 = rw - ii * R;
      const long base = ((long)ii * LP + t0 / POOL) * cout + oc;
      wg[j] = ld4(a.g_l + base);
      if constexpr (!RAW) {
        wy[j] = ld4(a.y_l + base);
        wid[j] = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
        wcnt[j] = a.counts ? a.counts[ii] : 1.f;
      }
    }
    int ii[FR], pc[FR];
    uint32_t vm = 0;
#pragma unroll
    for (int j = 0; j < FR; ++j) {
      const int row = rb + slot + 8 * j;
      const int rowc = row < r_end ? row : r_begin;
      ii[j] = rowc / R;
      const int p = rowc - ii[j] * R + kx - PAD;
      vm |= (row < r_end && kc_ok && p >= 0 && p < LIN) ? (1u << j) : 0u;
      pc[j] = p < 0 ? 0 : (p >= LIN ? LIN - 1 : p);
    }
    xvalid = vm;
    if constexpr (TRACK) {
      int trk[FR];
#pragma unroll
      for (int j = 0; j < FR; ++j) trk[j] = a.item_track[ii[j]];
#pragma unroll
      for (int j = 0; j < FR; ++j) {
        const long e = ((long)trk[j] * kFrames + pc[j]) * kMels + cx;
        if constexpr (XRAW)
          xr16[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.xsrc) + e);
        else
          xr[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + e);
      }
    } else {
#pragma unroll
      for (int j = 0; j < FR; ++j)
        xr[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + (((long)ii[j] * LIN + pc[j]) * cin + cx));
    }
  };

  // fragment read offsets: lane 4q'+p of its 16-lane group g supplies row (8g + 4h + q') of the
  // k-step, columns 4p..4p+3 of the 16-column tile (chunk = tile/8 + p/2, +8 B for odd p)
  const int fq = l16 >> 2, fp = l16 & 3;
  const int qoff = 8 * (q & 1);
  if (r_begin < r_end) issue(r_begin);
  for (int rb = r_begin; rb < r_end; rb += RCH) {
    // dz: BN_l's backward once per pool window, scaled and split, then written to the window's
    // rows -- the argmax row of each channel carries it, the others are zero (relu + max-pool)
#pragma unroll
    for (int j = 0; j < FW; ++j) {
      const int wl = slot + 8 * j;
      const int rw = rb + wl * POOL;
      const bool wv = rw < r_end && o_ok;
      const float gv[4] = {wg[j].x, wg[j].y, wg[j].z, wg[j].w};
      float d[4];
      if constexpr (RAW) {
#pragma unroll
        for (int s = 0; s < 4; ++s) d[s] = wv ? gv[s] * cas[s] : 0.f;
      } else {
        const float yv[4] = {wy[j].x, wy[j].y, wy[j].z, wy[j].w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float xh_ = (yv[s] - mu[s]) * iv[s];
          const float v = cas[s] * gv[s] - wcnt[j] * (cA[s] + xh_ * cB[s]);
          d[s] = (wv && yv[s] > 0.f) ? v : 0.f;
        }
      }
      if (do_bias) {
        bacc[0].x += d[0]; bacc[0].y += d[1]; bacc[0].z += d[2]; bacc[0].w += d[3];
        if constexpr (EDGES) {  // t = 0, 1 (first window), R-2, R-1 (last): static indices only
          int t0;
          if constexpr (R >= RCH) {  // as in issue(): at most two items per stage
            const int ra = (rb / R + 1) * R;
            t0 = rw - (rw >= ra ? ra : ra - R);
          } else {
            t0 = rw - (rw / R) * R;
          }
          const bool first = t0 == 0, last = t0 == R - POOL;
          float e1[4], e2[4], e3[4], e4[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const uint32_t r = (wid[j] >> (8 * s)) & 0xffu;
            e1[s] = (first && r == 0u) ? d[s] : 0.f;
            e2[s] = (first && r == 1u) ? d[s] : 0.f;
            e3[s] = (last && r == (uint32_t)(POOL - 2)) ? d[s] : 0.f;
            e4[s] = (last && r == (uint32_t)(POOL - 1)) ? d[s] : 0.f;
          }
          bacc[1].x += e1[0]; bacc[1].y += e1[1]; bacc[1].z += e1[2]; bacc[1].w += e1[3];
          bacc[2 % NB].x += e2[0]; bacc[2 % NB].y += e2[1]; bacc[2 % NB].z += e2[2]; bacc[2 % NB].w += e2[3];
          bacc[3 % NB].x += e3[0]; bacc[3 % NB].y += e3[1]; bacc[3 % NB].z += e3[2]; bacc[3 % NB].w += e3[3];
          bacc[4 % NB].x += e4[0]; bacc[4 % NB].y += e4[1]; bacc[4 % NB].z += e4[2]; bacc[4 % NB].w += e4[3];
        }
      }
      const w16_h4 h = {(_Float16)d[0], (_Float16)d[1], (_Float16)d[2], (_Float16)d[3]};
      const w16_h4 l = {(_Float16)(d[0] - (float)h[0]), (_Float16)(d[1] - (float)h[1]),
                        (_Float16)(d[2] - (float)h[2]), (_Float16)(d[3] - (float)h[3])};
      const uint2 hb = __builtin_bit_cast(uint2, h), lb = __builtin_bit_cast(uint2, l);
#pragma unroll
      for (int jp = 0; jp < POOL; ++jp) {
        uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
        if constexpr (POOL > 1) {
          const uint32_t id = wid[j];
          m0 = ((id & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
               (((id >> 8) & 0xffu) == (uint32_t)jp ? 0xffff0000u : 0u);
          m1 = (((id >> 16) & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
               ((id >> 24) == (uint32_t)jp ? 0xffff0000u : 0u);
        }
        const int off = w16_off(wl * POOL + jp, q >> 1) + qoff;
        *reinterpret_cast<uint2*>(dzh + off) = make_uint2(hb.x & m0, hb.y & m1);
        *reinterpret_cast<uint2*>(dzl + off) = make_uint2(lb.x & m0, lb.y & m1);
      }
    }
    // x: the layer input at tap kx (zero padding outside [0, LIN)), scaled and split
#pragma unroll
    for (int j = 0; j < FR; ++j) {
      const bool ok = (xvalid >> j) & 1u;
      const int off = w16_off(slot + 8 * j, q >> 1) + qoff;
      if constexpr (XRAW) {
        *reinterpret_cast<uint2*>(xh + off) = ok ? xr16[j] : make_uint2(0u, 0u);
      } else {
        const float x[4] = {xr[j].x, xr[j].y, xr[j].z, xr[j].w};
        float v[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = ok ? (x[s] - xm[s]) * xas[s] + xbs[s] : 0.f;
        w16_split_store(xh, xl, off, make_float4(v[0], v[1], v[2], v[3]));
      }
    }
    __syncthreads();
    if (rb + RCH < r_end) issue(rb + RCH);  // next stage's loads fly while the MFMAs run
#pragma unroll
    for (int ks = 0; ks < RCH / 32; ++ks) {
      w16_h8 ah[4], al[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int ch = (64 * wo + 16 * m) / 8 + (fp >> 1);
        const int r0 = 32 * ks + 8 * g + fq;
        const int o0 = w16_off(r0, ch) + 8 * (fp & 1), o1 = w16_off(r0 + 4, ch) + 8 * (fp & 1);
        const w16_h4 h0 = w16_tr(dzh, o0), h1 = w16_tr(dzh, o1), l0 = w16_tr(dzl, o0), l1 = w16_tr(dzl, o1);
        ah[m] = w16_h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        al[m] = w16_h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int ch = (64 * wk + 16 * n) / 8 + (fp >> 1);
        const int r0 = 32 * ks + 8 * g + fq;
        const int o0 = w16_off(r0, ch) + 8 * (fp & 1), o1 = w16_off(r0 + 4, ch) + 8 * (fp & 1);
        const w16_h4 h0 = w16_tr(xh, o0), h1 = w16_tr(xh, o1);
        const w16_h8 bh = w16_h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        if constexpr (XRAW) {
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[m], bh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bh, acc[m][n], 0, 0, 0);
          }
        } else {
          const w16_h4 l0 = w16_tr(xl, o0), l1 = w16_tr(xl, o1);
          const w16_h8 bl = w16_h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[m], bh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bl, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bh, acc[m][n], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }

  // partial block -> wpart[z][o][kc], unscaled; D lane map: o = 4g + reg, kc = l16
  float* wp = a.wpart + (size_t)bz * cout * kcn;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int kcl = 64 * wk + 16 * n + l16;
    const int kcg = kcbase + kcl;
    const int ecn = exp_c[kcl];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ol = 64 * wo + 16 * m + 4 * g + j;
        if (obase + ol < cout && kcg < kcn)
          wp[(size_t)(obase + ol) * kcn + kcg] = ldexpf(acc[m][n][j], -(exp_o[ol] + ecn));
      }
  }
  if (do_bias) {  // (the operand images are free: the last stage ended with a barrier)
#pragma unroll
    for (int e = 0; e < NB; ++e) st4(&bsum[slot][e][4 * q], bacc[e]);
    __syncthreads();
    if (tid < 128 && obase + tid < cout) {
      const int eo = exp_o[tid];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < 8; ++sl) v += bsum[sl][e][tid];
        a.bpart[((size_t)bz * NB + e) * cout + obase + tid] = ldexpf(v, -eo);
      }
    }
  }
}

template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP, bool EDGES>
__global__ __launch_bounds__(256, 2) void k_conv_wgrad16(WgradArgs a) {
  // the conv-1 weight gradient is the step's tail on the caller's stream: its waves take the issue
  // slots the side-stream weight gradients (priority 0) share with it
  critical_path_priority();
  extern __shared__ __attribute__((aligned(16))) char lds16[];
  // the kc tiles of one chunk read the same x rows and dz windows: consecutive logical blocks
  // (kc tile fastest) on one XCD share its L2 instead of fetching them once per tile from HBM
  const int gx = gridDim.x, gy = gridDim.y;
  const int L = xcd_swizzle(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  wgrad16_body<SRCX, KS, PAD, LIN, R, POOL, LP, EDGES>(a, L % gx, (L / gx) % gy, L / (gx * gy), lds16);
  if constexpr (SRCX != SRC_ACT) dev_wait_order(a.wait);  // (as k_conv_wgrad16t, layer 1)
}

template <int L>
__device__ __forceinline__ void wgrad16_multi_layer(const WgradMulti& w, int j, int b, char* lds) {
  constexpr LayerGeom gm = layer_geom(L == 6 ? 5 : L);
  const int kt = w.kt[j], ot = w.ot[j];
  wgrad16_body<SRC_ACT, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, gm.lp, false, L == 6>(
      w.a[j], b % kt, (b / kt) % ot, b / (kt * ot), lds);
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_conv_wgrad16_multi(WgradMulti w) {
  extern __shared__ __attribute__((aligned(16))) char lds16[];
  const int b = xcd_swizzle(blockIdx.x, gridDim.x);  // a chunk's tiles on one XCD (k_conv_wgrad16)
  int j = 0;
  while (j + 1 < w.n && b >= w.start[j + 1]) ++j;
  switch (w.layer[j]) {
    case 2: wgrad16_multi_layer<2>(w, j, b - w.start[j], lds16); break;
    case 3: wgrad16_multi_layer<3>(w, j, b - w.start[j], lds16); break;
    case 4: wgrad16_multi_layer<4>(w, j, b - w.start[j], lds16); break;
    case 5: wgrad16_multi_layer<5>(w, j, b - w.start[j], lds16); break;
    default: wgrad16_multi_layer<6>(w, j, b - w.start[j], lds16); break;
  }
}

// ------------------------------------------------ tap-fused split-f16 weight gradient (layers 1, 2)
// dW[o][k*128 + c] for one 64-channel o tile and ALL four taps in one workgroup of 8 waves: wave w
// owns tap k = w & 3 and o half w >> 2 (32 o x 128 c, 2 x 8 MFMA tiles). The kc-tiled kernel above
// builds a stage's dz windows once per kc tile (four times, one per tap) and its x rows once per
// tap; here the dz windows are built once per o tile and the x rows once: the x image holds, item
// by item, the input positions the stage's conv rows read -- each item's rows plus KS - 1 halo
// positions -- so tap k's B fragment of conv row r is image row r + k + (KS - 1) * (items of the
// stage before r's), a per-lane row address in the transposed read. dz rows are 128 B (64 o);
// x rows 256 B (cin = 128: the mels, or layer 2's input at H = 128).
constexpr int kW16tO = 64;   // o per workgroup
constexpr int kW16tThreads = 512;
// conv 1 (the track table): a chunk's items' track ids (+ the next item's, for the halo) are staged in
// LDS, at most this many -- wgrad_nchunk keeps rows_per_chunk <= (kWgItems - 3) R
constexpr int kWgItems = 128;
template <int R, int KS>
constexpr int w16t_img_rows() { return kW16Rows + (KS - 1) * (R >= kW16Rows ? 2 : kW16Rows / R + 2); }
template <int R, int KS>
constexpr size_t w16t_lds_bytes(bool xraw) {
  // the stage images, or (epilogue) the partial tile: 64 o rows of KS * 128 + 4 floats
  const size_t st = (size_t)2 * kW16Rows * 128 + (size_t)(xraw ? 1 : 2) * w16t_img_rows<R, KS>() * 256 +
                    (size_t)(kW16tO + 128 + 2 * kWgItems) * sizeof(int);
  const size_t ep = (size_t)kW16tO * (KS * 128 + 4) * sizeof(float);
  return st > ep ? st : ep;
}
// 16-byte chunk ch (of 8) of 128-byte dz row r: a transposed read's 32-lane half touches rows
// r0 + {0..3} + {0, 8}, two chunks each -- row bits 1 and 3 spread them over all 64 banks
__device__ __forceinline__ int w16_off128(int r, int ch) { return 128 * r + 16 * (ch ^ ((r & 2) | ((r >> 1) & 4))); }

template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP>
__device__ __forceinline__ void wgrad16t_body(const WgradArgs& a, int by, int bz, char* lds) {
  constexpr int RCH = kW16Rows;
  constexpr bool TRACK = SRCX == SRC_TRACK_F16 || SRCX == SRC_TRACK_F32;
  constexpr bool EDGES = TRACK;  // layer 1
  constexpr int NB = EDGES ? 5 : 1;  // bias (+ the four edge sums)
  constexpr int HALO = KS - 1;
  constexpr int IMG = w16t_img_rows<R, KS>();
  constexpr int FX = (IMG + 15) / 16;  // x image rows per thread (16 row slots x 32 channel quads)
  static_assert(KS == 4 && POOL == 4 && R % POOL == 0, "8 waves = 4 taps x 2 o halves; 16 windows per stage");
  constexpr bool TWO = R >= RCH;  // a stage spans at most two items
  constexpr bool XRAW = SRCX == SRC_TRACK_F16;
  static_assert(TRACK || SRCX == SRC_ACT, "x: the track table (layer 1) or y_{l-1}");
  char* dzh = lds;
  char* dzl = dzh + RCH * 128;
  char* xh = dzl + RCH * 128;
  char* xl = xh + IMG * 256;
  int* exp_o = reinterpret_cast<int*>(xh + (XRAW ? 1 : 2) * IMG * 256);
  int* exp_c = exp_o + kW16tO;
  [[maybe_unused]] int* trk_s = exp_c + 128;  // (conv 1) the chunk's items' track ids and counts
  [[maybe_unused]] float* cnt_s = reinterpret_cast<float*>(trk_s + kWgItems);
  float (*bsum)[NB][kW16tO] = reinterpret_cast<float (*)[NB][kW16tO]>(lds);  // after the last stage

  [[maybe_unused]] constexpr int KID = TRACK ? 0 : 1;
  DCUE_KTW(KID, 6);
  DCUE_KT(KID, 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int kx = wave & 3, oh = wave >> 2;  // this wave's tap and o half
  const int cout = a.cout, cin = a.cin;
  const int obase = by * kW16tO;
  const int total = a.M * R;  // rows (the host keeps M * R below 2^30)
  const int r_begin = bz * a.rows_per_chunk;  // a multiple of RCH
  const int r_end = min(r_begin + a.rows_per_chunk, total);
  [[maybe_unused]] const int item0 = r_begin / R;

  f32x4 acc[2][8];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bacc[NB];
#pragma unroll
  for (int e = 0; e < NB; ++e) bacc[e] = make_float4(0.f, 0.f, 0.f, 0.f);

  // dz: threads 0..255, window slot ws (16 per stage) x o quad q (16); x: every thread, row slot
  // xs (16) x mel quad cq (32)
  const bool dzt = tid < 256;
  const int q = tid & 15, ws = (tid >> 4) & 15;
  const int o = obase + 4 * q;
  const bool o_ok = o < cout;
  const int oc = o_ok ? o : 0;
  const int cq = tid & 31, xs = tid >> 5;
  const int cx = 4 * cq;
  // raw operands of one stage, loaded branch-free: the thread's dz window (g, y, argmax bytes, the
  // item's count) and its x image rows xs, xs + 16, ...
  // (a register set per stage in flight: one -- a second, two stages ahead, measured no faster: the
  // stages are MFMA + LDS bound, not load-latency bound; profiles/r06_ktrace_wgrad.txt)
  struct StageRegs {
    float4 wg, wy;
    uint32_t wid;
    float wcnt;
    float4 xr[XRAW ? 1 : FX];
    uint2 xr16[XRAW ? FX : 1];
    uint32_t xvalid;
  };
  StageRegs s0 = {};
  // (every thread issues the same loads on every path -- threads 256..511 a copy of 0..255's dz
  // window, counts through LDS or a select: the compiler's wait counts merge paths conservatively,
  // and a load skipped on one path made a stage wait for every load in flight)
  auto issue = [&](StageRegs& S, int rb) {
    const int i0 = rb / R, D = rb - i0 * R;  // the stage starts D rows into item i0
    {
      int rw = rb + ws * POOL;
      rw = rw < r_end ? rw : rb;
      const int ii = rw / R, t0 = rw - ii * R;
      const int base = (ii * LP + t0 / POOL) * cout + oc;
      S.wg = ld4(a.g_l + base);
      S.wy = ld4(a.y_l + base);
      S.wid = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
      if constexpr (TRACK && TWO) {
        S.wcnt = cnt_s[ii - item0];
      } else {
        const float c = *(a.counts ? a.counts + ii : a.mean_l);
        S.wcnt = a.counts ? c : 1.f;
      }
    }
    long t_a = 0, t_b = 0;
    if constexpr (TRACK && TWO) {  // (from LDS: a global load here would hold the x loads -- and so
      t_a = trk_s[i0 - item0];      // the stage's MFMAs behind them -- for an L2 round trip a stage)
      t_b = trk_s[min(i0 + 1, a.M - 1) - item0];
    }
    uint32_t vm = 0;
#pragma unroll
    for (int j = 0; j < FX; ++j) {
      const int jr = xs + 16 * j;  // image row
      int k;                       // items after i0
      if constexpr (TWO)
        k = jr + D >= R + HALO ? 1 : 0;
      else
        k = (jr + D) / (R + HALO);
      const int i = i0 + k;
      const int p = jr + D - k * (R + HALO) - PAD;  // input position in item i
      const bool ok = jr < IMG && i < a.M && p >= 0 && p < LIN;
      vm |= ok ? (1u << j) : 0u;
      if constexpr (TRACK) {
        long trk;
        if constexpr (TWO)
          trk = k ? t_b : t_a;
        else
          trk = a.item_track[ok ? i : i0];
        const long e = (trk * kFrames + (ok ? p : 0)) * kMels + cx;
        if constexpr (XRAW)
          S.xr16[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.xsrc) + e);
        else
          S.xr[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + e);
      } else {
        S.xr[j] = ld4(reinterpret_cast<const float*>(a.xsrc) + (((long)(ok ? i : i0) * LIN + (ok ? p : 0)) * cin + cx));
      }
    }
    S.xvalid = vm;
  };
  // The column constants' loads (independent of each other) go out first, then the first stage's:
  // loads return in issue order, so the constants' math overlaps the stage's flight. (Round 6, per-WG
  // phase trace: prologue + first fill 4.5 us either way -- the kernel's first loads after its
  // producer cost ~3 us however they are ordered; profiles/r06_ktrace_wgrad.txt)
  float mu[4] = {}, iv[4] = {}, av[4] = {}, sd[4] = {}, sdx[4] = {};
  float gmx[4], ymx[4], xlo[4], xhi[4];
  {
    const float4 m4 = ld4(a.mean_l + oc), i4 = ld4(a.invstd_l + oc), a4 = ld4(a.a_l + oc);
    mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
    iv[0] = i4.x; iv[1] = i4.y; iv[2] = i4.z; iv[3] = i4.w;
    av[0] = a4.x; av[1] = a4.y; av[2] = a4.z; av[3] = a4.w;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sd[s] = (float)acc_sum(a.dz_acc, cout, 0, oc + s);
      sdx[s] = (float)acc_sum(a.dz_acc, cout, 1, oc + s);
      gmx[s] = w16_key(a.g_range, oc + s);
      ymx[s] = w16_key(a.y_range, oc + s);
      if constexpr (TRACK) {
        xlo[s] = -w16_key(a.x_range + kRngC, cx + s);
        xhi[s] = w16_key(a.x_range, cx + s);
      } else {  // a ReLU output
        xlo[s] = 0.f;
        xhi[s] = fmaxf(w16_key(a.x_range, cx + s), 0.f);
      }
    }
  }
  const float4 xmu = ld4(a.x_mean + cx), xsc = ld4(a.x_a + cx);
  const float4 xbe = a.x_beta ? ld4(a.x_beta + cx) : make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (TRACK && TWO) {
    const int nitem = min(a.M - item0, (r_end - 1) / R - item0 + 2);
    for (int k = tid; k < nitem; k += kW16tThreads) {
      trk_s[k] = a.item_track[item0 + k];
      cnt_s[k] = a.counts ? a.counts[item0 + k] : 1.f;
    }
    __syncthreads();
  }
  if (r_begin < r_end) issue(s0, r_begin);
  if (by == 0 && bz == 0 && tid < cout) {  // BN_l = gamma * xhat + beta: dbeta = sum g, dgamma = sum g * xhat
    a.dbeta[tid] = (float)(acc_sum(a.dz_acc, cout, 0, tid) * bn_grad_scale(a));
    a.dgamma[tid] = (float)(acc_sum(a.dz_acc, cout, 1, tid) * bn_grad_scale(a));
  }
  const float xm[4] = {xmu.x, xmu.y, xmu.z, xmu.w}, xs_[4] = {xsc.x, xsc.y, xsc.z, xsc.w};
  const float xb[4] = {xbe.x, xbe.y, xbe.z, xbe.w};
  // column scales as wgrad16_body: scaled dz = cas g - count (cA + xhat cB), scaled x = (src - xm) xas + xbs
  float cas[4], cA[4], cB[4], xas[4], xbs[4];
  {
    int eo[4], ec[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float gmax = gmx[s];
      const float ym = fmaxf(ymx[s], 0.f);
      const float xhm = fmaxf(fabsf(mu[s]), fabsf(ym - mu[s])) * iv[s];
      const float bo = fabsf(av[s]) * (gmax + a.kd_max * (fabsf(sd[s]) + xhm * fabsf(sdx[s])));
      eo[s] = o_ok ? w16_exp(bo) : 0;
      const float lo = xlo[s], hi = xhi[s];
      const float bx_ = fmaxf(fabsf((lo - xm[s]) * xs_[s] + xb[s]), fabsf((hi - xm[s]) * xs_[s] + xb[s]));
      ec[s] = XRAW ? 0 : w16_exp(bx_);
      const float so = ldexpf(1.f, eo[s]), sx = ldexpf(1.f, ec[s]);
      cas[s] = av[s] * so;
      cA[s] = av[s] * a.invN * sd[s] * so;
      cB[s] = av[s] * a.invN * sdx[s] * so;
      xas[s] = xs_[s] * sx;
      xbs[s] = xb[s] * sx;
    }
    if (tid < 16)
#pragma unroll
      for (int s = 0; s < 4; ++s) exp_o[4 * q + s] = eo[s];
    if (xs == 0)
#pragma unroll
      for (int s = 0; s < 4; ++s) exp_c[4 * cq + s] = ec[s];
  }
  __syncthreads();
  DCUE_KT(KID, 1);


  // fragment read offsets: lane 4q'+p of its 16-lane group g supplies row (8g + 4h + q') of the
  // k-step, columns 4p..4p+3 of the 16-column tile
  const int fq = l16 >> 2, fp = l16 & 3;
  auto stage = [&](StageRegs& S, int rb) {
    if (dzt) {  // dz: BN_1's backward for the thread's window, scaled, split, written to its rows
      const int rw = rb + ws * POOL;
      const bool wv = rw < r_end && o_ok;
      const float gv[4] = {S.wg.x, S.wg.y, S.wg.z, S.wg.w}, yv[4] = {S.wy.x, S.wy.y, S.wy.z, S.wy.w};
      float d[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float xh_ = (yv[s] - mu[s]) * iv[s];
        const float v = cas[s] * gv[s] - S.wcnt * (cA[s] + xh_ * cB[s]);
        d[s] = (wv && yv[s] > 0.f) ? v : 0.f;
      }
      bacc[0].x += d[0]; bacc[0].y += d[1]; bacc[0].z += d[2]; bacc[0].w += d[3];
      if constexpr (EDGES) {  // t = 0, 1 (first window), R-2, R-1 (last window)
        const int t0 = rw - (rw / R) * R;
        const bool first = t0 == 0, last = t0 == R - POOL;
        float e1[4], e2[4], e3[4], e4[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint32_t r = (S.wid >> (8 * s)) & 0xffu;
          e1[s] = (first && r == 0u) ? d[s] : 0.f;
          e2[s] = (first && r == 1u) ? d[s] : 0.f;
          e3[s] = (last && r == (uint32_t)(POOL - 2)) ? d[s] : 0.f;
          e4[s] = (last && r == (uint32_t)(POOL - 1)) ? d[s] : 0.f;
        }
        bacc[1].x += e1[0]; bacc[1].y += e1[1]; bacc[1].z += e1[2]; bacc[1].w += e1[3];
        bacc[2 % NB].x += e2[0]; bacc[2 % NB].y += e2[1]; bacc[2 % NB].z += e2[2]; bacc[2 % NB].w += e2[3];
        bacc[3 % NB].x += e3[0]; bacc[3 % NB].y += e3[1]; bacc[3 % NB].z += e3[2]; bacc[3 % NB].w += e3[3];
        bacc[4 % NB].x += e4[0]; bacc[4 % NB].y += e4[1]; bacc[4 % NB].z += e4[2]; bacc[4 % NB].w += e4[3];
      }
      const w16_h4 h = {(_Float16)d[0], (_Float16)d[1], (_Float16)d[2], (_Float16)d[3]};
      const w16_h4 l = {(_Float16)(d[0] - (float)h[0]), (_Float16)(d[1] - (float)h[1]),
                        (_Float16)(d[2] - (float)h[2]), (_Float16)(d[3] - (float)h[3])};
      const uint2 hb = __builtin_bit_cast(uint2, h), lb = __builtin_bit_cast(uint2, l);
#pragma unroll
      for (int jp = 0; jp < POOL; ++jp) {
        const uint32_t m0 = ((S.wid & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
                            (((S.wid >> 8) & 0xffu) == (uint32_t)jp ? 0xffff0000u : 0u);
        const uint32_t m1 = (((S.wid >> 16) & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
                            ((S.wid >> 24) == (uint32_t)jp ? 0xffff0000u : 0u);
        const int off = w16_off128(ws * POOL + jp, q >> 1) + 8 * (q & 1);
        *reinterpret_cast<uint2*>(dzh + off) = make_uint2(hb.x & m0, hb.y & m1);
        *reinterpret_cast<uint2*>(dzl + off) = make_uint2(lb.x & m0, lb.y & m1);
      }
    }
#pragma unroll
    for (int j = 0; j < FX; ++j) {  // x image (zero padding and past-the-batch rows are zeros)
      const int jr = xs + 16 * j;
      if (jr < IMG) {
        const bool ok = (S.xvalid >> j) & 1u;
        const int off = w16_off(jr, cq >> 1) + 8 * (cq & 1);
        if constexpr (XRAW) {
          *reinterpret_cast<uint2*>(xh + off) = ok ? S.xr16[j] : make_uint2(0u, 0u);
        } else {
          const float x[4] = {S.xr[j].x, S.xr[j].y, S.xr[j].z, S.xr[j].w};
          float v[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) v[s] = ok ? (x[s] - xm[s]) * xas[s] + xbs[s] : 0.f;
          w16_split_store(xh, xl, off, make_float4(v[0], v[1], v[2], v[3]));
        }
      }
    }
    __syncthreads();
    if (rb == r_begin) DCUE_KT(KID, 2);
    const int i0 = rb / R;
    const int lb = (i0 + 1) * R - rb;  // the stage row where item i0 + 1 starts (TWO)
    if (rb + RCH < r_end) issue(S, rb + RCH);  // next stage's loads fly while the MFMAs run
#pragma unroll
    for (int ks = 0; ks < RCH / 32; ++ks) {
      const int r0 = 32 * ks + 8 * g + fq;  // this lane's conv rows: r0 (first read), r0 + 4 (second)
      w16_h8 ah[2], al[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int ch = 4 * oh + 2 * m + (fp >> 1);
        const int o0 = w16_off128(r0, ch) + 8 * (fp & 1), o1 = w16_off128(r0 + 4, ch) + 8 * (fp & 1);
        const w16_h4 h0 = w16_tr(dzh, o0), h1 = w16_tr(dzh, o1), l0 = w16_tr(dzl, o0), l1 = w16_tr(dzl, o1);
        ah[m] = w16_h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        al[m] = w16_h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      }
      int img0, img1;  // the image rows tap kx reads for conv rows r0, r0 + 4
      if constexpr (TWO) {
        img0 = r0 + kx + (r0 >= lb ? HALO : 0);
        img1 = r0 + 4 + kx + (r0 + 4 >= lb ? HALO : 0);
      } else {
        img0 = r0 + kx + HALO * ((rb + r0) / R - i0);
        img1 = r0 + 4 + kx + HALO * ((rb + r0 + 4) / R - i0);
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const int ch = 2 * n + (fp >> 1);
        const int ob0 = w16_off(img0, ch) + 8 * (fp & 1), ob1 = w16_off(img1, ch) + 8 * (fp & 1);
        const w16_h4 h0 = w16_tr(xh, ob0), h1 = w16_tr(xh, ob1);
        const w16_h8 bh = w16_h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        if constexpr (XRAW) {
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[m], bh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bh, acc[m][n], 0, 0, 0);
          }
        } else {
          const w16_h4 l0 = w16_tr(xl, ob0), l1 = w16_tr(xl, ob1);
          const w16_h8 bl = w16_h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[m], bh, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bl, acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[m], bh, acc[m][n], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  };
  for (int rb = r_begin; rb < r_end; rb += RCH) stage(s0, rb);

  DCUE_KT(KID, 3);
  int eo_bias;  // (the bias partials' exponent, read before the tile staging overwrites exp_o)
  // partial block -> wpart[z][o][kx * cin + c], unscaled; D lane map: o = 4g + reg, c = l16. The
  // workgroup's 64 o x KS*128 kc block is contiguous in wpart: it is staged through LDS (row pitch
  // KC + 4 floats: the four g rows of a store land on disjoint banks) and written with linear float4
  // stores -- the accumulators' per-lane dword stores took 3.7 of the workgroup's 16 us (round 6)
  {
    constexpr int KC = KS * 128, PITCH = KC + 4;  // (cin == 128: the launch checks it)
    int eo_r[2][4], ec_r[8];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) eo_r[m][j] = exp_o[32 * oh + 16 * m + 4 * g + j];
#pragma unroll
    for (int n = 0; n < 8; ++n) ec_r[n] = exp_c[16 * n + l16];
    eo_bias = tid < kW16tO ? exp_o[tid] : 0;
    __syncthreads();  // (the exponents are read: the tile overwrites them)
    float* tl = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          tl[(32 * oh + 16 * m + 4 * g + j) * PITCH + kx * 128 + 16 * n + l16] =
              ldexpf(acc[m][n][j], -(eo_r[m][j] + ec_r[n]));
    __syncthreads();
    const int nrow = min(kW16tO, cout - obase);
    float* wp = a.wpart + ((size_t)bz * cout + obase) * KC;
    constexpr int Q = KC / 4;  // float4 per row
    for (int i = tid; i < nrow * Q; i += kW16tThreads) {
      const int r = i / Q, k4 = i - r * Q;
      st4(wp + (size_t)r * KC + 4 * k4, *reinterpret_cast<const float4*>(tl + r * PITCH + 4 * k4));
    }
    __syncthreads();  // (bsum below reuses the tile's LDS)
  }
  // bias (+ edge) partials of the tile's 64 channels: the 16 window slots, summed in order (the
  // operand images are free: the last stage ended with a barrier)
  if (dzt)
#pragma unroll
    for (int e = 0; e < NB; ++e) st4(&bsum[ws][e][4 * q], bacc[e]);
  __syncthreads();
  if (tid < kW16tO && obase + tid < cout) {
#pragma unroll
    for (int e = 0; e < NB; ++e) {
      float v = 0.f;
#pragma unroll
      for (int sl = 0; sl < 16; ++sl) v += bsum[sl][e][tid];
      a.bpart[((size_t)bz * NB + e) * cout + obase + tid] = ldexpf(v, -eo_bias);
    }
  }
  DCUE_KT(KID, 4);
  DCUE_KTW(KID, 7);
}

template <int SRCX, int KS, int PAD, int LIN, int R, int POOL, int LP>
__global__ __launch_bounds__(kW16tThreads, 1) void k_conv_wgrad16t(WgradArgs a) {
  // layer 1 is the step's tail on the caller's stream (as k_conv_wgrad16); layer 2 a side stream's
  if constexpr (SRCX != SRC_ACT) critical_path_priority();
  extern __shared__ __attribute__((aligned(16))) char lds16t[];
  // a chunk's o tiles read the same x rows: consecutive logical blocks (o tile fastest) on one XCD
  const int ot = (a.cout + kW16tO - 1) / kW16tO;
  const int L = xcd_swizzle(blockIdx.x, gridDim.x);
  wgrad16t_body<SRCX, KS, PAD, LIN, R, POOL, LP>(a, L % ot, L / ot, lds16t);
  // (plans, layer 1: the next step's prepared inputs -- only an order for the kernels after this one)
  if constexpr (SRCX != SRC_ACT) dev_wait_order(a.wait);
}

// ---------------------------------------------------------------------------------------------------
// Conv-1 weight gradient, one tap per workgroup (round 6). wgrad16t_body gives
// a workgroup a 64 o x 512 kc tile, so the chip fills only through split-K: 33 chunks x 2 tiles at
// the in-batch shape, 8.7 MB of partial blocks for a 0.26 MB dW, and a workgroup's 4 stages run at
// one per CU. Here the dW is cut into 32 o x 128 c tiles (4 o tiles x 4 taps = 16 per chunk) of 256
// threads, so ~16 chunks fill the chip: half the partial bytes, and the x and dz operands a chunk's
// 16 tiles share are re-read from L2 (the tiles of a chunk are consecutive logical blocks: one XCD).
// Operands, column scaling and the hi + lo split of dz are wgrad16t_body's (XRAW: x is the raw fp16
// table, exact in f16); the partial layout is the same, so launch_wgrad_reduce and bn0's gradient
// kernels read it unchanged. Two stages' loads are in flight (the stage work is a quarter of
// wgrad16t's, so the L2 round trip is what a stage would otherwise wait on).
constexpr int kW1kO = 32;         // o per workgroup
constexpr int kW1kThreads = 256;  // 4 waves: o block (16) x c half (64)
template <int R, int KS>
constexpr size_t w1k_lds_bytes() {
  // dz hi / lo images (64 rows x 128 B; the tile's 32 o use the first 64 B of a row), the x image
  // (IMG rows x 256 B) and the o exponents; after the stages the same bytes hold the tile (32 rows
  // of 128 + 4 floats), then the bias partials (16 x 5 x 32 floats)
  const size_t st = (size_t)2 * kW16Rows * 128 + (size_t)w16t_img_rows<R, KS>() * 256 + kW1kO * sizeof(int) +
                    (size_t)kWgItems * (sizeof(int) + sizeof(float));
  const size_t ep = (size_t)kW1kO * (128 + 4) * sizeof(float);
  const size_t bs = (size_t)16 * 5 * kW1kO * sizeof(float);
  const size_t m = st > ep ? st : ep;
  return m > bs ? m : bs;
}

template <int KS, int PAD, int LIN, int R, int POOL, int LP>
__device__ __forceinline__ void wgrad1k_body(const WgradArgs& a, int ot, int kx, int bz, char* lds) {
  constexpr int RCH = kW16Rows;
  constexpr int NB = 5;  // bias + the four edge sums (conv 1's zero padding)
  constexpr int HALO = KS - 1;
  constexpr int IMG = w16t_img_rows<R, KS>();
  constexpr int FX = (IMG + 7) / 8;  // x image rows per thread (8 row slots x 32 channel quads)
  static_assert(KS == 4 && POOL == 4 && R % POOL == 0 && R >= RCH, "conv 1: 16 windows a stage, at most two items");
  char* dzh = lds;
  char* dzl = dzh + RCH * 128;
  char* xh = dzl + RCH * 128;
  int* exp_o = reinterpret_cast<int*>(xh + IMG * 256);
  int* trk_s = exp_o + kW1kO;  // the chunk's items' track ids and counts (the host bounds their number)
  float* cnt_s = reinterpret_cast<float*>(trk_s + kWgItems);
  float (*bsum)[NB][kW1kO] = reinterpret_cast<float (*)[NB][kW1kO]>(lds);  // after the tile's stores

  DCUE_KTW(0, 6);
  DCUE_KT(0, 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int ob = wave & 1, chh = wave >> 1;  // this wave's o block (16 o) and c half (64 c)
  const int cout = a.cout;
  const int obase = ot * kW1kO;
  const int total = a.M * R;  // rows (the host keeps M * R below 2^30)
  const int r_begin = bz * a.rows_per_chunk;  // a multiple of RCH
  const int r_end = min(r_begin + a.rows_per_chunk, total);
  const int item0 = r_begin / R;

  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bacc[NB];
#pragma unroll
  for (int e = 0; e < NB; ++e) bacc[e] = make_float4(0.f, 0.f, 0.f, 0.f);

  // dz: threads 0..127, window slot ws (16 a stage) x o quad q (8); x: every thread, row slot xs (8)
  // x channel quad cq (32)
  const bool dzt = tid < 128;
  const int q = tid & 7, ws = (tid >> 3) & 15;
  const int o = obase + 4 * q;
  const bool o_ok = o < cout;
  const int oc = o_ok ? o : 0;
  const int cq = tid & 31, xs = tid >> 5;
  const int cx = 4 * cq;
  struct StageRegs {
    float4 wg, wy;
    uint32_t wid;
    float wcnt;
    uint2 xr[FX];
    uint32_t xvalid;
  };
  StageRegs s0 = {}, s1 = {};
  // One stage's raw operands. Every thread issues the same loads on every path (threads 128..255 load
  // a copy of threads 0..127's windows; a stage past the chunk reloads its first): the compiler's
  // wait counts merge paths conservatively, so a load skipped on one path made every stage wait for
  // all loads in flight -- the other stage's too -- which undid the two-stage pipeline
  auto issue = [&](StageRegs& S, int rb_) {
    const int rb = rb_ < r_end ? rb_ : r_begin;
    const int i0 = rb / R, D = rb - i0 * R;  // the stage starts D rows into item i0
    {
      int rw = rb + ws * POOL;
      rw = rw < r_end ? rw : rb;
      const int ii = rw / R, t0 = rw - ii * R;
      const int base = (ii * LP + t0 / POOL) * cout + oc;
      S.wg = ld4(a.g_l + base);
      S.wy = ld4(a.y_l + base);
      S.wid = *reinterpret_cast<const uint32_t*>(a.idx_l + base);
      S.wcnt = cnt_s[ii - item0];
    }
    // (track ids from LDS: a dependent global load here would make the stage's x loads wait for it,
    // and loads retire in order, so for every load in flight before it -- the other stage's)
    const long t_a = trk_s[i0 - item0], t_b = trk_s[min(i0 + 1, a.M - 1) - item0];
    uint32_t vm = 0;
#pragma unroll
    for (int j = 0; j < FX; ++j) {
      const int jr = xs + 8 * j;                       // image row
      const int k = jr + D >= R + HALO ? 1 : 0;        // items after i0
      const int i = i0 + k;
      const int p = jr + D - k * (R + HALO) - PAD;     // input position in item i
      const bool ok = jr < IMG && i < a.M && p >= 0 && p < LIN;
      vm |= ok ? (1u << j) : 0u;
      const long e = ((k ? t_b : t_a) * kFrames + (ok ? p : 0)) * kMels + cx;
      S.xr[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(a.xsrc) + e);
    }
    S.xvalid = vm;
  };

  // the column constants' loads first, then the first two stages' (loads return in issue order)
  float mu[4], iv[4], av[4], sd[4], sdx[4], gmx[4], ymx[4];
  {
    const float4 m4 = ld4(a.mean_l + oc), i4 = ld4(a.invstd_l + oc), a4 = ld4(a.a_l + oc);
    mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
    iv[0] = i4.x; iv[1] = i4.y; iv[2] = i4.z; iv[3] = i4.w;
    av[0] = a4.x; av[1] = a4.y; av[2] = a4.z; av[3] = a4.w;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sd[s] = (float)acc_sum(a.dz_acc, cout, 0, oc + s);
      sdx[s] = (float)acc_sum(a.dz_acc, cout, 1, oc + s);
      gmx[s] = w16_key(a.g_range, oc + s);
      ymx[s] = w16_key(a.y_range, oc + s);
    }
  }
  {
    const int nitem = min(a.M - item0, (r_end - 1) / R - item0 + 2);
    for (int k = tid; k < nitem; k += kW1kThreads) {
      trk_s[k] = a.item_track[item0 + k];
      cnt_s[k] = a.counts ? a.counts[item0 + k] : 1.f;
    }
  }
  __syncthreads();
  issue(s0, r_begin);
  issue(s1, r_begin + RCH);
  if (ot == 0 && kx == 0 && bz == 0 && tid < cout) {  // BN_1 = gamma * xhat + beta: dbeta = sum g, dgamma = sum g * xhat
    a.dbeta[tid] = (float)(acc_sum(a.dz_acc, cout, 0, tid) * bn_grad_scale(a));
    a.dgamma[tid] = (float)(acc_sum(a.dz_acc, cout, 1, tid) * bn_grad_scale(a));
  }
  // scaled dz = cas g - count (cA + xhat cB), as wgrad16t_body (x: raw fp16, exponent 0)
  float cas[4], cA[4], cB[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float ym = fmaxf(ymx[s], 0.f);
    const float xhm = fmaxf(fabsf(mu[s]), fabsf(ym - mu[s])) * iv[s];
    const float bo = fabsf(av[s]) * (gmx[s] + a.kd_max * (fabsf(sd[s]) + xhm * fabsf(sdx[s])));
    const int eo = o_ok ? w16_exp(bo) : 0;
    const float so = ldexpf(1.f, eo);
    cas[s] = av[s] * so;
    cA[s] = av[s] * a.invN * sd[s] * so;
    cB[s] = av[s] * a.invN * sdx[s] * so;
    if (tid < 8) exp_o[4 * q + s] = eo;
  }
  __syncthreads();
  DCUE_KT(0, 1);

  // fragment read offsets: lane 4q'+p of its 16-lane group g supplies row (8g + 4h + q') of the
  // k-step, columns 4p..4p+3 of the 16-column tile
  const int fq = l16 >> 2, fp = l16 & 3;
  auto stage = [&](StageRegs& S, int rb) {
    if (dzt) {  // dz: BN_1's backward for the thread's window, scaled, split, written to its rows
      const int rw = rb + ws * POOL;
      const bool wv = rw < r_end && o_ok;
      const float gv[4] = {S.wg.x, S.wg.y, S.wg.z, S.wg.w}, yv[4] = {S.wy.x, S.wy.y, S.wy.z, S.wy.w};
      float d[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float xh_ = (yv[s] - mu[s]) * iv[s];
        const float v = cas[s] * gv[s] - S.wcnt * (cA[s] + xh_ * cB[s]);
        d[s] = (wv && yv[s] > 0.f) ? v : 0.f;
      }
      bacc[0].x += d[0]; bacc[0].y += d[1]; bacc[0].z += d[2]; bacc[0].w += d[3];
      {  // t = 0, 1 (first window), R-2, R-1 (last window)
        const int t0 = rw - (rw / R) * R;
        const bool first = t0 == 0, last = t0 == R - POOL;
        float e1[4], e2[4], e3[4], e4[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint32_t r = (S.wid >> (8 * s)) & 0xffu;
          e1[s] = (first && r == 0u) ? d[s] : 0.f;
          e2[s] = (first && r == 1u) ? d[s] : 0.f;
          e3[s] = (last && r == (uint32_t)(POOL - 2)) ? d[s] : 0.f;
          e4[s] = (last && r == (uint32_t)(POOL - 1)) ? d[s] : 0.f;
        }
        bacc[1].x += e1[0]; bacc[1].y += e1[1]; bacc[1].z += e1[2]; bacc[1].w += e1[3];
        bacc[2].x += e2[0]; bacc[2].y += e2[1]; bacc[2].z += e2[2]; bacc[2].w += e2[3];
        bacc[3].x += e3[0]; bacc[3].y += e3[1]; bacc[3].z += e3[2]; bacc[3].w += e3[3];
        bacc[4].x += e4[0]; bacc[4].y += e4[1]; bacc[4].z += e4[2]; bacc[4].w += e4[3];
      }
      const w16_h4 h = {(_Float16)d[0], (_Float16)d[1], (_Float16)d[2], (_Float16)d[3]};
      const w16_h4 l = {(_Float16)(d[0] - (float)h[0]), (_Float16)(d[1] - (float)h[1]),
                        (_Float16)(d[2] - (float)h[2]), (_Float16)(d[3] - (float)h[3])};
      const uint2 hb = __builtin_bit_cast(uint2, h), lb = __builtin_bit_cast(uint2, l);
#pragma unroll
      for (int jp = 0; jp < POOL; ++jp) {  // the window's argmax row carries it, the others zeros
        const uint32_t m0 = ((S.wid & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
                            (((S.wid >> 8) & 0xffu) == (uint32_t)jp ? 0xffff0000u : 0u);
        const uint32_t m1 = (((S.wid >> 16) & 0xffu) == (uint32_t)jp ? 0x0000ffffu : 0u) |
                            ((S.wid >> 24) == (uint32_t)jp ? 0xffff0000u : 0u);
        const int off = w16_off128(ws * POOL + jp, q >> 1) + 8 * (q & 1);
        *reinterpret_cast<uint2*>(dzh + off) = make_uint2(hb.x & m0, hb.y & m1);
        *reinterpret_cast<uint2*>(dzl + off) = make_uint2(lb.x & m0, lb.y & m1);
      }
    }
#pragma unroll
    for (int j = 0; j < FX; ++j) {  // x image (zero padding and past-the-batch rows are zeros)
      const int jr = xs + 8 * j;
      if (jr < IMG) {
        const bool ok = (S.xvalid >> j) & 1u;
        *reinterpret_cast<uint2*>(xh + w16_off(jr, cq >> 1) + 8 * (cq & 1)) = ok ? S.xr[j] : make_uint2(0u, 0u);
      }
    }
    __syncthreads();
    if (rb == r_begin) DCUE_KT(0, 2);
    const int lb = (rb / R + 1) * R - rb;  // the stage row where the next item starts
    issue(S, rb + 2 * RCH);  // (S is in LDS: its registers take stage + 2)
#pragma unroll
    for (int ks = 0; ks < RCH / 32; ++ks) {
      const int r0 = 32 * ks + 8 * g + fq;  // this lane's conv rows: r0 (first read), r0 + 4 (second)
      const int ch = 2 * ob + (fp >> 1);
      const int o0 = w16_off128(r0, ch) + 8 * (fp & 1), o1 = w16_off128(r0 + 4, ch) + 8 * (fp & 1);
      const w16_h4 h0 = w16_tr(dzh, o0), h1 = w16_tr(dzh, o1), l0 = w16_tr(dzl, o0), l1 = w16_tr(dzl, o1);
      const w16_h8 ah = w16_h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      const w16_h8 al = w16_h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      const int img0 = r0 + kx + (r0 >= lb ? HALO : 0), img1 = r0 + 4 + kx + (r0 + 4 >= lb ? HALO : 0);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int cc = 2 * (4 * chh + n) + (fp >> 1);
        const int ob0 = w16_off(img0, cc) + 8 * (fp & 1), ob1 = w16_off(img1, cc) + 8 * (fp & 1);
        const w16_h4 x0 = w16_tr(xh, ob0), x1 = w16_tr(xh, ob1);
        const w16_h8 bh = w16_h8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[n], 0, 0, 0);
      }
    }
    __syncthreads();
  };
  // stages in pairs: a chunk's odd last stage is paired with an empty one (every dz masked: it adds
  // zeros), so the two register sets alternate on every path
  for (int rb = r_begin; rb < r_end; rb += 2 * RCH) {
    stage(s0, rb);
    stage(s1, rb + RCH);
  }

  DCUE_KT(0, 3);
  // partial block -> wpart[z][o][kx * 128 + c], unscaled; D lane map: o = 4g + reg, c = l16. The
  // tile's 32 rows of 128 floats go through LDS (row pitch 132: the four g rows of a store land on
  // disjoint banks) and out as linear float4 stores (512-byte row segments)
  int eo_r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) eo_r[j] = exp_o[16 * ob + 4 * g + j];
  const int eo_bias = tid < kW1kO ? exp_o[tid] : 0;
  __syncthreads();  // (the exponents are read: the tile overwrites them)
  {
    constexpr int PITCH = 128 + 4, KC = KS * 128;
    float* tl = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        tl[(16 * ob + 4 * g + j) * PITCH + 16 * (4 * chh + n) + l16] = ldexpf(acc[n][j], -eo_r[j]);
    __syncthreads();
    const int nrow = min(kW1kO, cout - obase);
    float* wp = a.wpart + ((size_t)bz * cout + obase) * KC + kx * 128;
    for (int i = tid; i < nrow * 32; i += kW1kThreads) {
      const int r = i >> 5, k4 = i & 31;
      st4(wp + (size_t)r * KC + 4 * k4, *reinterpret_cast<const float4*>(tl + r * PITCH + 4 * k4));
    }
  }
  if (kx == 0) {  // bias (+ edge) partials: the tap-0 workgroups (every tap sees the same dz)
    __syncthreads();  // (bsum reuses the tile's LDS)
    if (dzt)
#pragma unroll
      for (int e = 0; e < NB; ++e) st4(&bsum[ws][e][4 * q], bacc[e]);
    __syncthreads();
    if (tid < kW1kO && obase + tid < cout) {
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < 16; ++sl) v += bsum[sl][e][tid];  // the 16 window slots, in order
        a.bpart[((size_t)bz * NB + e) * cout + obase + tid] = ldexpf(v, -eo_bias);
      }
    }
  }
  DCUE_KT(0, 4);
  DCUE_KTW(0, 7);
}

template <int KS, int PAD, int LIN, int R, int POOL, int LP>
__global__ __launch_bounds__(kW1kThreads, 2) void k_conv_wgrad1k(WgradArgs a) {
  critical_path_priority();  // the step's tail on the caller's stream
  extern __shared__ __attribute__((aligned(16))) char lds1k[];
  // a chunk's 16 tiles (o tile fastest, then tap) are consecutive logical blocks: one XCD, one L2
  const int ot = (a.cout + kW1kO - 1) / kW1kO;
  const int L = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tile = L % (ot * KS);
  wgrad1k_body<KS, PAD, LIN, R, POOL, LP>(a, tile % ot, tile / ot, L / (ot * KS), lds1k);
  dev_wait_order(a.wait);  // (plans: the next step's prepared inputs -- an order for later kernels only)
}

// whether the weight gradients run on split-f16 MFMA (DCUE_WGRAD_F16=0: the f32-MFMA kernels)
bool wgrad_f16_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_WGRAD_F16");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the layers whose split-f16 weight gradient runs tap-fused (k_conv_wgrad16t): 1 and 2, whose
// inputs have 128 channels (layer 2 at H = 128). DCUE_W16_TAPFUSED=0: neither, =1: layer 1 only
// (A/B; the kc-tiled k_conv_wgrad16 / multi kernel otherwise)
static bool w16t_layer(int layer, int cin) {
  static const int mode = [] {
    const char* e = getenv("DCUE_W16_TAPFUSED");
    return e ? atoi(e) : 2;
  }();
  if (!wgrad_f16_on() || cin != kMels) return false;
  return layer == 1 ? mode >= 1 : (layer == 2 && mode >= 2);
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
    a.dbeta[tid] = (float)(acc_sum(a.dz_acc, cout, 0, tid) * bn_grad_scale(a));
    a.dgamma[tid] = (float)(acc_sum(a.dz_acc, cout, 1, tid) * bn_grad_scale(a));
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

// split-K chunk length of the split-f16 kernels: whole stages (so whole pool windows), (wgrad_nchunk
// picks counts that leave no chunk empty)
static long w16_rows_per_chunk(long rows, int nchunk) {
  const long rpc = (rows + nchunk - 1) / nchunk;
  return (rpc + kW16Rows - 1) / kW16Rows * kW16Rows;
}

// conv 1's split-f16 weight gradient on k_conv_wgrad1k (one tap per workgroup, round 6; needs
// 128 input channels and cout <= 256) under DCUE_W1K=1. Off by default: at the in-batch shape it
// measured 24.6-34.5 us (2-16 stages a chunk) against k_conv_wgrad16t's 19.9 us, although it writes
// half the partial bytes (profiles/r06_w1k_sweep.txt).
static bool w1k_layer1(int cin, int cout) {
  static const bool on = [] {
    const char* e = getenv("DCUE_W1K");
    return e && e[0] == '1';
  }();
  return on && wgrad_f16_on() && cin == kMels && cout % 4 == 0 && cout <= kW1kThreads;
}

int wgrad_nchunk(int layer, int M, int cout, int cin) {
  // one workgroup per CU (LDS-bound): at most 256 / tiles chunks, each of >= 64 rows; partial
  // blocks cost a write + a read of cout*ks*cin floats per chunk (layer 6: the fc, geometry of 5)
  const LayerGeom gm = layer_geom(layer == 6 ? 5 : layer);
  const long rows = (long)M * gm.lp * gm.pool;
  if (layer == 1 && !wgrad_f16_on()) {  // k_conv1_wgrad: 64x64 tiles, >= 4 steps per chunk, <= ~512 workgroups (2 per CU)
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
  if (layer == 1 && w1k_layer1(cin, cout)) {
    // k_conv_wgrad1k: 16 tiles a chunk (4 o tiles x 4 taps at H = 128), two workgroups per CU, and
    // at least DCUE_W1K_MIN_STAGES (default 8) 64-row stages a chunk: each chunk writes a 0.26 MB
    // partial block, so the split-K depth is held down (in-batch: 15 chunks, 3.9 MB of partials
    // against rounds 3-5's 33 and 8.7 MB)
    static const long min_st = [] {
      const char* e = getenv("DCUE_W1K_MIN_STAGES");
      const long v = e ? atol(e) : 0;
      return v >= 1 && v <= 256 ? v : 8L;
    }();
    const long tiles1 = ((cout + kW1kO - 1) / kW1kO) * gm.ks;
    long n = 512 / tiles1;
    const long per = min_st * kW16Rows;
    if (n > (rows + per - 1) / per) n = (rows + per - 1) / per;
    const long cap = (8L << 20) / ((long)cout * gm.ks * cin);
    if (n > cap) n = cap;
    // a chunk's items fit the kernel's LDS table: rows_per_chunk <= (kWgItems - 3) R
    const long rmax = ((long)(kWgItems - 3) * gm.lp * gm.pool) / kW16Rows * kW16Rows;
    if (n < (rows + rmax - 1) / rmax) n = (rows + rmax - 1) / rmax;
    if (n < 1) n = 1;
    n = (rows + w16_rows_per_chunk(rows, (int)n) - 1) / w16_rows_per_chunk(rows, (int)n);
    return (int)(n < 1 ? 1 : n);
  }
  const long tiles = w16t_layer(layer, cin)
                        ? (cout + kW16tO - 1) / kW16tO  // k_conv_wgrad16t: 64 o x all taps
                        : ((gm.ks * cin + 127) / 128) * ((cout + 127) / 128);
  // split-f16 kernels: two workgroups per CU (one's MFMAs and fill run while the other's stage
  // loads are in flight); DCUE_W16_WGS_PER_CU=1 halves the chunks (A/B diagnostic)
  static const long per_cu = [] {
    const char* e = getenv("DCUE_W16_WGS_PER_CU");
    return e && atoi(e) == 1 ? 1L : 2L;
  }();
  long n = (wgrad_f16_on() ? 256 * per_cu : 256) / tiles;
  if (!wgrad_f16_on()) {
    if (n > (rows + 63) / 64) n = (rows + 63) / 64;
  } else {
    // at least DCUE_W16_MIN_STAGES (default 4) 64-row stages per chunk: each chunk costs a
    // prologue, a partial block written and read back by the reduce, so short ones do not pay
    // (A/B, GPU-only: 1, 2, 4 stages within noise in-batch; 4 the fastest catalogue, -8 us)
    static const long min_stages = [] {
      const char* e = getenv("DCUE_W16_MIN_STAGES");
      const long v = e ? atol(e) : 0;
      return v >= 1 && v <= 64 ? v : 4L;
    }();
    // DCUE_W16T_MIN_STAGES: the same for the tap-fused conv-1 kernel (A/B diagnostic)
    static const long min_stages_t = [] {
      const char* e = getenv("DCUE_W16T_MIN_STAGES");
      const long v = e ? atol(e) : 0;
      return v >= 1 && v <= 64 ? v : 0L;
    }();
    const bool fused = w16t_layer(layer, cin);
    const long per = (fused && min_stages_t ? min_stages_t : min_stages) * kW16Rows;
    if (n > (rows + per - 1) / per) n = (rows + per - 1) / per;
  }
  const long cap = (8L << 20) / ((long)cout * gm.ks * cin);
  if (n > cap) n = cap;
  if (layer == 1 && wgrad_f16_on()) {  // the tap-fused kernel's LDS item table (kWgItems)
    const long rmax = ((long)(kWgItems - 3) * gm.lp * gm.pool) / kW16Rows * kW16Rows;
    if (n < (rows + rmax - 1) / rmax) n = (rows + rmax - 1) / rmax;
  }
  if (n < 1) n = 1;
  if (wgrad_f16_on())  // whole stages per chunk: no chunk left empty by the rounding
    n = (rows + w16_rows_per_chunk(rows, (int)n) - 1) / w16_rows_per_chunk(rows, (int)n);
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

template <int L, int SRCX>
static int wgrad16t_launch(const WgradArgs& a0, int nchunk, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int R = gm.lp * gm.pool;
  constexpr size_t LDS = w16t_lds_bytes<R, gm.ks>(SRCX == SRC_TRACK_F16);
  auto kern = k_conv_wgrad16t<SRCX, gm.ks, gm.pad, gm.lin, R, gm.pool, gm.lp>;
  if (a0.cin != kMels || a0.cout % 4) return DCUE_ERR_INVALID;  // x image rows: 128 channels
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS));
    attr = true;
  }
  WgradArgs a = a0;
  const long rows = (long)a.M * R;
  if (rows >= (1L << 30)) return DCUE_ERR_UNSUPPORTED;  // 32-bit row indices
  a.rows_per_chunk = (int)w16_rows_per_chunk(rows, nchunk);
  if (SRCX != SRC_ACT && R >= kW16Rows && a.rows_per_chunk / R + 3 > kWgItems) return DCUE_ERR_INVALID;
  const unsigned ot = (unsigned)((a.cout + kW16tO - 1) / kW16tO);
  DCUE_LAUNCH(kern, dim3(ot * (unsigned)nchunk), dim3(kW16tThreads), LDS, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

static int wgrad1k_launch(const WgradArgs& a0, int nchunk, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(1);
  constexpr int R = gm.lp * gm.pool;
  constexpr size_t LDS = w1k_lds_bytes<R, gm.ks>();
  auto kern = k_conv_wgrad1k<gm.ks, gm.pad, gm.lin, R, gm.pool, gm.lp>;
  if (a0.cin != kMels || a0.cout % 4 || a0.cout > kW1kThreads) return DCUE_ERR_INVALID;
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS));
    attr = true;
  }
  WgradArgs a = a0;
  const long rows = (long)a.M * R;
  if (rows >= (1L << 30)) return DCUE_ERR_UNSUPPORTED;  // 32-bit row indices
  a.rows_per_chunk = (int)w16_rows_per_chunk(rows, nchunk);
  if (a.rows_per_chunk / R + 3 > kWgItems) return DCUE_ERR_INVALID;  // (wgrad_nchunk keeps it in range)
  const unsigned tiles = (unsigned)(((a.cout + kW1kO - 1) / kW1kO) * gm.ks);
  DCUE_LAUNCH(kern, dim3(tiles * (unsigned)nchunk), dim3(kW1kThreads), LDS, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

template <int L, int SRCX>
static int wgrad16_layer(const WgradArgs& a0, int nchunk, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int R = gm.lp * gm.pool;
  if constexpr (L == 1 && SRCX == SRC_TRACK_F16)
    if (w1k_layer1(a0.cin, a0.cout)) return wgrad1k_launch(a0, nchunk, s);
  if constexpr (L == 1)
    if (w16t_layer(1, a0.cin)) return wgrad16t_launch<1, SRCX>(a0, nchunk, s);
  auto kern = k_conv_wgrad16<SRCX, gm.ks, gm.pad, gm.lin, R, gm.pool, gm.lp, L == 1>;
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kW16LdsB));
    attr = true;
  }
  WgradArgs a = a0;
  const long rows = (long)a.M * R;
  if (rows >= (1L << 30)) return DCUE_ERR_UNSUPPORTED;  // 32-bit row indices
  a.rows_per_chunk = (int)w16_rows_per_chunk(rows, nchunk);
  dim3 grid((unsigned)((gm.ks * a.cin + 127) / 128), (unsigned)((a.cout + 127) / 128), (unsigned)nchunk);
  DCUE_LAUNCH(kern, grid, dim3(256), kW16LdsB, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_conv_wgrad(int layer, int src, const WgradArgs& a, int nchunk, hipStream_t s) {
  if (wgrad_f16_on()) {  // layer 1 reads the track table (bn0 applied at the fill), not xhat0
    switch (layer) {
      case 1: return src == SRC_TRACK_F16 ? wgrad16_layer<1, SRC_TRACK_F16>(a, nchunk, s)
                                          : wgrad16_layer<1, SRC_TRACK_F32>(a, nchunk, s);
      case 2: return wgrad16_layer<2, SRC_ACT>(a, nchunk, s);
      case 3: return wgrad16_layer<3, SRC_ACT>(a, nchunk, s);
      case 4: return wgrad16_layer<4, SRC_ACT>(a, nchunk, s);
      case 5: return wgrad16_layer<5, SRC_ACT>(a, nchunk, s);
      default: return DCUE_ERR_INVALID;
    }
  }
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
  wgrad_reduce_body(a.wpart, a.bpart, w.nchunk[j], a.cout, a.cin, layer_geom(w.layer[j] == 6 ? 5 : w.layer[j]).ks, 1,
                    w.dW[j], w.db[j], nullptr, nullptr, b - w.rstart[j]);
}

int launch_conv_wgrad_multi(WgradMulti w, hipStream_t s) {
  const bool f16 = wgrad_f16_on();
  const size_t LDS = f16 ? kW16LdsB : wgrad_lds_floats(1) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_wgrad_multi, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(wgrad_lds_floats(1) * sizeof(float))));
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_wgrad16_multi<1>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kW16LdsB));
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_conv_wgrad16_multi<2>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kW16LdsB));
    attr = true;
  }
  w.start[0] = 0;
  w.rstart[0] = 0;
  if (w.n < 1 || w.n > kWgradMultiMax) return DCUE_ERR_INVALID;
  if (w.n == 1 && w.layer[0] == 2 && w16t_layer(2, w.a[0].cin)) {  // layer 2 alone: tap-fused + its reduce
    const WgradArgs& a = w.a[0];
    TRY((wgrad16t_launch<2, SRC_ACT>(a, w.nchunk[0], s)));
    w.rstart[1] = (int)(((long)a.cout * 4 * a.cin + 127) / 128 + (a.cout + 127) / 128);
    DCUE_LAUNCH(k_wgrad_reduce_multi, dim3((unsigned)w.rstart[1]), dim3(256), 0, s, w);
    DCUE_LAUNCH_CHECK();
    return DCUE_OK;
  }
  for (int j = 0; j < w.n; ++j) {
    if (w.layer[j] < 2 || w.layer[j] > 6) return DCUE_ERR_INVALID;
    WgradArgs& a = w.a[j];
    const LayerGeom gm = layer_geom(w.layer[j] == 6 ? 5 : w.layer[j]);
    if (a.cin % 32 || a.cout % 4) return DCUE_ERR_UNSUPPORTED;
    const long rows = (long)a.M * gm.lp * gm.pool;
    if (f16 && rows >= (1L << 30)) return DCUE_ERR_UNSUPPORTED;
    a.rows_per_chunk = (int)(f16 ? w16_rows_per_chunk(rows, w.nchunk[j]) : (rows + w.nchunk[j] - 1) / w.nchunk[j]);
    w.kt[j] = (gm.ks * a.cin + 127) / 128;
    w.ot[j] = (a.cout + 127) / 128;
    w.start[j + 1] = w.start[j] + w.kt[j] * w.ot[j] * w.nchunk[j];
    w.rstart[j + 1] = w.rstart[j] + (int)(((long)a.cout * gm.ks * a.cin + 127) / 128 + (a.cout + 127) / 128);
  }
  if (f16)
  {
    // two workgroups per CU (the layer-5 / fc branch spills 148 B per lane at that register budget);
    // DCUE_W16_MULTI_OCC=1: one, no spill (A/B diagnostic)
    static const bool occ1 = [] {
      const char* e = getenv("DCUE_W16_MULTI_OCC");
      return e && e[0] == '1';
    }();
    if (occ1)
      DCUE_LAUNCH(k_conv_wgrad16_multi<1>, dim3((unsigned)w.start[w.n]), dim3(256), LDS, s, w);
    else
      DCUE_LAUNCH(k_conv_wgrad16_multi<2>, dim3((unsigned)w.start[w.n]), dim3(256), LDS, s, w);
  }
  else
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
// With mean0 set, G holds the contraction with the raw fp16 input instead (the split-f16 weight
// gradient's exact operand): sum dz1 * xhat0 = invstd0 (G - mean0 S) over the same rows.
// The per-element arithmetic is bn0_elem (explicit fmaf): k_bn0_grads_adam (adam.hip, built without
// contraction) repeats it bit for bit.
__global__ __launch_bounds__(256) void k_bn0_grads(const float* __restrict__ G, const float* __restrict__ E,
                                                   const float* __restrict__ W1, const float* gamma0,
                                                   const float* beta0, const float* mean0,
                                                   const float* invstd0, int H, float* dW1,
                                                   float* dgamma0, float* dbeta0, float* db1) {
  critical_path_priority();
  __shared__ float rg[256], rb[256];
  bn0_channel<false>(G, E, gamma0, beta0, mean0, invstd0, H, dgamma0, dbeta0, Bn0AdamDev{}, W1, dW1, db1,
                     blockIdx.x, threadIdx.x, rg, rb, true);
}

int launch_bn0_grads(const float* G, const float* E, const float* W1, const float* gamma0,
                     const float* beta0, const float* mean0, const float* invstd0, int H, float* dW1,
                     float* dgamma0, float* dbeta0, float* db1, hipStream_t s) {
  DCUE_LAUNCH(k_bn0_grads, dim3(kMels), dim3(256), 0, s, G, E, W1, gamma0, beta0, mean0, invstd0, H, dW1,
              dgamma0, dbeta0, db1);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue

