// Shared by adam.hip and conv_wgrad.hip: torch.optim.Adam's element arithmetic (adam_replay.h) with
// correctly rounded primitives, the conv-weight repack store, and bn0's gradients + Adam over segments
// [0, DCUE_SEG_LATE) for one input channel (k_bn0_grads_adam; the conv-1 weight-gradient tail kernel
// runs the same function). Every operation here is an explicit rounding primitive or fmaf, so the
// bits do not depend on the including file's contraction flags.
#pragma once

#include "dcue_internal.h"

namespace dcue {

// Every operation rounded on its own unless written as an fma, so that the dense sweep, the deferred
// replay and the touched-row step produce identical bits. sqrt must be __builtin_sqrtf: hipcc lowers
// it to v_sqrt_f32 plus the two-fma correction, while __fsqrt_rn compiles to the bare 1-ulp v_sqrt_f32.
#define DCUE_RHD __device__ __forceinline__
DCUE_RHD float rn_fma(float a, float b, float c) { return __fmaf_rn(a, b, c); }
DCUE_RHD float rn_mul(float a, float b) { return __fmul_rn(a, b); }
DCUE_RHD float rn_add(float a, float b) { return __fadd_rn(a, b); }
DCUE_RHD float rn_sub(float a, float b) { return __fsub_rn(a, b); }
DCUE_RHD float rn_div(float a, float b) { return __fdiv_rn(a, b); }
DCUE_RHD float rn_sqrt(float a) { return __builtin_sqrtf(a); }

}  // namespace dcue

#include "adam_replay.h"

namespace dcue {

// bn0's gradients + Adam over segments [0, DCUE_SEG_LATE) in one launch (dcue_internal.h Bn0Adam):
// the channel owning input channel c -- W1[:, c, :] (gradient, Adam, repack), bn0's gamma/beta[c] --
// and channels 0 / 1 conv 1's bias and bn1's gamma/beta (whose gradients the conv-1 weight gradient
// already wrote). Gradient arithmetic: bn0_elem, as k_bn0_grads; Adam: adam_elem, as the dense sweep --
// the plan's fused step and an eager backward + dcue_adam_step agree bit for bit.
struct Bn0AdamDev {
  float *p, *m, *v, *g;
  long o_w1, o_cb1, o_g0, o_b0, o_g1, o_b1;  // -1: no such segment (towers without BatchNorm)
  AdamScalars sc;
  PackSeg seg1;
  float* wpack;
};

__device__ __forceinline__ void adam_at(const Bn0AdamDev& a, long idx, float gr) {
  float pp = a.p[idx], mm = a.m[idx], vv = a.v[idx];
  adam_elem(pp, gr, mm, vv, a.sc);
  a.p[idx] = pp;
  a.m[idx] = mm;
  a.v[idx] = vv;
}
Bn0AdamDev bn0adam_dev(const Bn0Adam& a);  // (host, adam.hip)

// One input channel c of bn0's backward, by a group of 256 threads t (the caller's 256-float LDS
// arrays rg, rb; every thread of the workgroup calls it -- the reduction's barriers are the
// workgroup's -- with active = false for groups without a channel).
// ADAM: k_bn0_grads_adam (the gradient of W1[:, c, :] into grads, Adam over it with the repack, conv
// 1's bias (c = 0) and bn1's gamma / beta (c = 1), bn0's gamma / beta[c]);
// !ADAM: k_bn0_grads (dW1[:, c, :] from W1, db1 (c = 0), dgamma0 / dbeta0[c]).
template <bool ADAM>
DCUE_RHD void bn0_channel(const float* __restrict__ G, const float* __restrict__ E, const float* gamma0,
                          const float* beta0, const float* mean0, const float* invstd0, int H, float* dgamma0,
                          float* dbeta0, const Bn0AdamDev& a, const float* __restrict__ W1, float* dW1, float* db1,
                          int c, int t, float* rg, float* rb, bool active) {
  // the parameter, gradient and moment buffers never alias G / E (workspace): restrict lets every
  // element's loads issue before the first element's stores (one memory round instead of one per
  // element); the per-element arithmetic and the order of the dg / db sums are unchanged
  float* __restrict__ P = a.p;
  float* __restrict__ Mo = a.m;
  float* __restrict__ V = a.v;
  float* __restrict__ Gd = a.g;
  float dg = 0.f, db = 0.f;
  // bn0's gamma / beta state of this channel, loaded up front (thread 0 steps them last)
  float pg = 0.f, mg = 0.f, vg = 0.f, pb = 0.f, mb = 0.f, vb = 0.f;
  if (active) {
    if (ADAM && t == 0 && a.o_g0 >= 0) {
      pg = P[a.o_g0 + c]; mg = Mo[a.o_g0 + c]; vg = V[a.o_g0 + c];
      pb = P[a.o_b0 + c]; mb = Mo[a.o_b0 + c]; vb = V[a.o_b0 + c];
    }
    const Bn0Chan ch = bn0_chan(gamma0, beta0, mean0, invstd0, c);
    constexpr int kMaxIt = 4;  // 4H <= 1024 = 4 x 256 threads (H <= 256)
#pragma unroll
    for (int it = 0; it < kMaxIt; ++it) {
      const int e = t + 256 * it;
      if (e < 4 * H) {  // e = o*4 + k: the dW1[o][c][k] layout
        const int o = e >> 2, k = e & 3;
        const long wi = ((long)o * kMels + c) * 4 + k;
        if constexpr (ADAM) {
          const long idx = a.o_w1 + wi;
          float pp = P[idx];
          const float gw = bn0_elem(G, E, H, ch, o, k, c, pp, dg, db);  // reads the pre-step weight
          Gd[idx] = gw;
          float mm = Mo[idx], vv = V[idx];
          adam_elem(pp, gw, mm, vv, a.sc);
          P[idx] = pp;
          Mo[idx] = mm;
          V[idx] = vv;
          pack_store(a.seg1, wi, pp, a.wpack);
        } else {
          dW1[wi] = bn0_elem(G, E, H, ch, o, k, c, W1[wi], dg, db);
        }
      }
    }
    if constexpr (ADAM) {
      if (c == 0)
        for (int o = t; o < H; o += 256) {
          a.g[a.o_cb1 + o] = E[o];
          adam_at(a, a.o_cb1 + o, E[o]);
        }
      if (c == 1 && a.o_g1 >= 0)
        for (int o = t; o < H; o += 256) {
          adam_at(a, a.o_g1 + o, a.g[a.o_g1 + o]);
          adam_at(a, a.o_b1 + o, a.g[a.o_b1 + o]);
        }
    } else {
      if (c == 0)
        for (int o = t; o < H; o += 256) db1[o] = E[o];
    }
  }
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
  if (active && t == 0) {
    dgamma0[c] = rg[0];
    dbeta0[c] = rb[0];
    if (ADAM && a.o_g0 >= 0) {
      adam_elem(pg, rg[0], mg, vg, a.sc);
      adam_elem(pb, rb[0], mb, vb, a.sc);
      P[a.o_g0 + c] = pg; Mo[a.o_g0 + c] = mg; V[a.o_g0 + c] = vg;
      P[a.o_b0 + c] = pb; Mo[a.o_b0 + c] = mb; V[a.o_b0 + c] = vb;
    }
  }
}

}  // namespace dcue
