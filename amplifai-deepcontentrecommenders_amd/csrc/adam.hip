// torch.optim.Adam over the flat dense buffer and the user table, plus the weight repack -- gfx950.
// Reference: optim.Adam as built at nn/dcue.py:143-147 and stepped at :209 (CPU single-tensor path).
#include "dcue_internal.h"

namespace dcue {

// torch.optim.Adam, foreach=False/fused=False (the CPU reference path), per element:
//   g += wd*p (wd != 0);  m.lerp_(g, 1-b1);  v = v*b2 + (1-b2)*g*g;
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
struct AdamScalars {
  float lr_bc1, one_m_b1, b2, one_m_b2, bc2_sqrt, eps, wd;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& s) {
  if (s.wd != 0.f) g = g + s.wd * p;
  m = m + s.one_m_b1 * (g - m);
  v = v * s.b2 + s.one_m_b2 * (g * g);
  const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
  p = p - s.lr_bc1 * (m / denom);
}

__global__ __launch_bounds__(256) void k_adam_dense(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    long n, AdamScalars s) {
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = ld4(p + 4 * i), gg = ld4(g + 4 * i), mm = ld4(m + 4 * i), vv = ld4(v + 4 * i);
    adam_elem(pp.x, gg.x, mm.x, vv.x, s);
    adam_elem(pp.y, gg.y, mm.y, vv.y, s);
    adam_elem(pp.z, gg.z, mm.z, vv.z, s);
    adam_elem(pp.w, gg.w, mm.w, vv.w, s);
    st4(p + 4 * i, pp); st4(m + 4 * i, mm); st4(v + 4 * i, vv);
  }
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    adam_elem(p[i], g[i], m[i], v[i], s);
}

// User table: one wave per row; rows without a gradient this step get g = 0 (the reference's dense
// embedding gradient), then the row's slot is cleared for the next step.
__global__ __launch_bounds__(256) void k_adam_embed(float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v,
                                                    const float* __restrict__ gcompact,
                                                    int32_t* slot, long n_rows, int E, AdamScalars s) {
  const int lane = threadIdx.x & 63;
  const long wave0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave0; r < n_rows; r += nwaves) {
    const int sl = slot[r];
    float* pr = p + r * E;
    float* mr = m + r * E;
    float* vr = v + r * E;
    const float* gr = sl >= 0 ? gcompact + (long)sl * E : nullptr;
    if ((E & 3) == 0) {
      for (int k4 = lane; k4 < E / 4; k4 += 64) {
        float4 pp = ld4(pr + 4 * k4), mm = ld4(mr + 4 * k4), vv = ld4(vr + 4 * k4);
        const float4 gg = gr ? ld4(gr + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        adam_elem(pp.x, gg.x, mm.x, vv.x, s);
        adam_elem(pp.y, gg.y, mm.y, vv.y, s);
        adam_elem(pp.z, gg.z, mm.z, vv.z, s);
        adam_elem(pp.w, gg.w, mm.w, vv.w, s);
        st4(pr + 4 * k4, pp); st4(mr + 4 * k4, mm); st4(vr + 4 * k4, vv);
      }
    } else {
      for (int k = lane; k < E; k += 64) adam_elem(pr[k], gr ? gr[k] : 0.f, mr[k], vr[k], s);
    }
    if (lane == 0 && sl >= 0) slot[r] = -1;
  }
}

int launch_adam(const dcue_model* md, const dcue_adam_args* a, const int64_t* poff, hipStream_t s) {
  const double bc1 = 1.0 - pow((double)a->beta1, (double)a->step);
  const double bc2 = 1.0 - pow((double)a->beta2, (double)a->step);
  AdamScalars sc;
  sc.lr_bc1 = (float)((double)a->lr / bc1);
  sc.one_m_b1 = (float)(1.0 - (double)a->beta1);
  sc.b2 = a->beta2;
  sc.one_m_b2 = (float)(1.0 - (double)a->beta2);
  sc.bc2_sqrt = (float)sqrt(bc2);
  sc.eps = a->eps;
  sc.wd = a->weight_decay;
  const int parts = a->parts ? a->parts : (DCUE_ADAM_DENSE | DCUE_ADAM_EMBEDDING);
  const long n = poff[DCUE_N_DENSE_SEGMENTS];
  if (parts & DCUE_ADAM_DENSE) {
    hipLaunchKernelGGL(k_adam_dense, dim3(512), dim3(256), 0, s, md->params, md->grads, md->exp_avg,
                       md->exp_avg_sq, n, sc);
    DCUE_LAUNCH_CHECK();
  }
  if ((parts & DCUE_ADAM_EMBEDDING) && md->dims.n_users > 0) {
    long blocks = (md->dims.n_users + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_adam_embed, dim3((unsigned)blocks), dim3(256), 0, s, md->emb,
                       md->emb_exp_avg, md->emb_exp_avg_sq, md->emb_grad, md->emb_slot,
                       (long)md->dims.n_users, md->dims.user_embdim, sc);
    DCUE_LAUNCH_CHECK();
  }
  return DCUE_OK;
}

// ------------------------------------------------------------------------- weight packing
// conv layer l forward B operand: [k][cin/4][cout][4]; dgrad (l >= 2): [k'][cout/4][cin][4] with
// k' = ks-1-k.
struct PackSeg {
  long src, fwd, bwd;  // floats: W in params; forward pack; dgrad pack (-1: none)
  int cout, cin, ks;
};
struct PackArgs {
  PackSeg seg[5];
};

__global__ void k_pack(const float* __restrict__ params, float* wpack, PackArgs pa) {
  const PackSeg sg = pa.seg[blockIdx.y];
  const long ks = sg.ks;
  const long n = (long)sg.cout * sg.cin * ks;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long o = e / ((long)sg.cin * ks);
    const long rem = e - o * sg.cin * ks;
    const long c = rem / ks, k = rem - c * ks;
    const float w = params[sg.src + e];  // W[o][c][k]
    wpack[sg.fwd + (((k * (sg.cin / 4) + c / 4) * sg.cout + o) * 4 + (c & 3))] = w;
    if (sg.bwd >= 0) {
      const long kr = sg.ks - 1 - k;
      wpack[sg.bwd + (((kr * (sg.cout / 4) + o / 4) * sg.cin + c) * 4 + (o & 3))] = w;
    }
  }
}

int launch_pack(const dcue_model* md, const int64_t* poff, hipStream_t s) {
  const int H = md->dims.conv_hidden, d = md->dims.feature_dim;
  const WpackLayout wl = wpack_layout(&md->dims);
  PackArgs pa;
  for (int l = 1; l <= 5; ++l) {
    PackSeg& sg = pa.seg[l - 1];
    sg.cin = l == 1 ? kMels : H;
    sg.cout = l == 5 ? d : H;
    sg.ks = layer_geom(l).ks;
    sg.src = poff[2 + 4 * (l - 1)];  // conv.layer{l}.weight
    sg.fwd = wl.conv_fwd[l];
    sg.bwd = l >= 2 ? wl.conv_bwd[l] : -1;
  }
  hipLaunchKernelGGL(k_pack, dim3(64, 5), dim3(256), 0, s, md->params, md->wpack, pa);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
