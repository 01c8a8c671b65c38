// torch.optim.Adam over the flat dense buffer and the user table, plus the weight repack -- gfx950.
// Reference: optim.Adam as built at nn/dcue.py:143-147 and stepped at :209 (CPU single-tensor path).
#include "dcue_internal.h"

namespace dcue {

// torch.optim.Adam, foreach=False/fused=False, per element, as torch 2.10's CPU kernels round it
// (torch/optim/adam.py _single_tensor_adam; each form below was matched bit for bit against those
// kernels on random inputs, tests/test_adam_cpu.py):
//   g = fma(p, wd, g)                      grad.add(param, alpha=wd)
//   m = fma(c, g - m, base)                exp_avg.lerp_(grad, 1-b1): c = w, base = m (w < 0.5),
//                                          else c = w - 1, base = g (the vectorised lerp)
//   v = fma((1-b2)*g, g, v*b2)             exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1-b2)
//   d = sqrt(v) / bc2_sqrt + eps           (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
//   p = p + (step * m) / d                 param.addcdiv_(exp_avg, denom, value=-step_size)
// The one place this cannot be bit-identical is sqrt: the CPU kernel's vectorised sqrt is not
// correctly rounded (1 ulp off on ~0.6% of inputs, tests/test_adam_cpu.py); here it is. (It must be
// __builtin_sqrtf: hipcc lowers it to v_sqrt_f32 plus the two-fma correction, while __fsqrt_rn
// compiles to the bare 1-ulp v_sqrt_f32.)
struct AdamScalars {
  float neg_step, lerp_c, b2, one_m_b2, bc2_sqrt, eps, wd;  // neg_step = -(lr / bc1)
  float inv_bc2_sqrt;  // RN(1 / bc2_sqrt): Markstein division by the per-step constant
};
static_assert(sizeof(AdamScalars) == 32, "history entry is [8] floats");

// Every operation rounded on its own unless written as an fma (fp contraction off for this file)
// so that the dense sweep, the deferred replay and the touched-row step produce identical bits.
// lerp_c < 0: the lerp weight is >= 0.5 (beta1 <= 0.5), so the blend base is g.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& s) {
#pragma clang fp contract(off)
  if (s.wd != 0.f) g = __fmaf_rn(p, s.wd, g);
  m = __fmaf_rn(s.lerp_c, __fsub_rn(g, m), s.lerp_c < 0.f ? g : m);
  v = __fmaf_rn(__fmul_rn(s.one_m_b2, g), g, __fmul_rn(v, s.b2));
  const float denom = __fadd_rn(__fdiv_rn(__builtin_sqrtf(v), s.bc2_sqrt), s.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(s.neg_step, m), denom));
}

// The zero-gradient step (a row outside the batch, wd == 0, lerp weight < 0.5), bit-identical to
// adam_elem(p, +0, m, v, s): fma((1-b2)*0, 0, v*b2) == v*b2 (v >= 0), and sqrt(v)/bc2_sqrt by
// Markstein's correction with r = RN(1/bc2_sqrt): q = RN(a r), q' = RN(q + RN?(a - q bc2)*r) is the
// correctly rounded quotient for a >= 2^-100 (below it the plain division runs). This is the
// deferred replay's inner loop (VALU-bound).
__device__ __forceinline__ void adam_zero_elem(float& p, float& m, float& v, const AdamScalars& s) {
  m = __fmaf_rn(s.lerp_c, __fsub_rn(0.f, m), m);
  v = __fmul_rn(v, s.b2);
  const float sq = __builtin_sqrtf(v);
  float t;
  if (sq >= 0x1p-100f) {
    const float q = __fmul_rn(sq, s.inv_bc2_sqrt);
    const float r = __fmaf_rn(-q, s.bc2_sqrt, sq);
    t = __fmaf_rn(r, s.inv_bc2_sqrt, q);
  } else {
    t = __fdiv_rn(sq, s.bc2_sqrt);
  }
  const float denom = __fadd_rn(t, s.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(s.neg_step, m), denom));
}

// replay of a zero-gradient step: the fast form when no weight decay touches g
__device__ __forceinline__ void adam_replay(float& p, float& m, float& v, const AdamScalars& s, float gz) {
  if (s.wd == 0.f && s.lerp_c < 0.5f)
    adam_zero_elem(p, m, v, s);
  else
    adam_elem(p, gz, m, v, s);
}

// (m, v) = (+0, +0) is a fixed point of the zero-gradient step without weight decay (adam_zero_elem:
// m - w*0 = +0, v*b2 = +0, sqrt(0)/bc2 = 0, denom = eps, p + (-lr_bc1)*(0/eps) = p + (-0) = p,
// signed zeros included): a user row never in a batch needs no replay, bit for bit what the dense
// sweep computes. The replay kernels skip such elements (no loads of p, no stores).
__device__ __forceinline__ bool idle_moments(float m, float v) {
  return (__float_as_uint(m) | __float_as_uint(v)) == 0u;
}
__device__ __forceinline__ bool idle_moments4(const float4& m, const float4& v) {
  return (__float_as_uint(m.x) | __float_as_uint(m.y) | __float_as_uint(m.z) | __float_as_uint(m.w) |
          __float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z) | __float_as_uint(v.w)) == 0u;
}
// whether every replayed step of [j0, j1] (history slots j % cap) is free of weight decay
__device__ __forceinline__ bool no_decay(const AdamScalars* hs, int j0, int j1, int cap, float gz) {
  if (gz != 0.f) return false;
  for (int j = j0; j <= j1; ++j)
    if (hs[j % cap].wd != 0.f) return false;
  return true;
}

struct PackSeg {
  long src, fwd, bwd;  // floats: W in params; forward pack; dgrad pack (-1: none)
  int cout, cin, ks;
};
struct PackArgs;
PackArgs pack_args(const dcue_model* md, const int64_t* poff);
struct PackArgs {
  PackSeg seg[5];
};

// Packed position of element e of conv segment sg (W[o][c][k], k fastest): the forward B operand
// [k][cin/4][cout][4] and (layers >= 2) the dgrad one [ks-1-k][cout/4][cin][4].
__device__ __forceinline__ void pack_store(const PackSeg& sg, long e, float w, float* wpack) {
  const long ks = sg.ks;
  const long o = e / ((long)sg.cin * ks);
  const long rem = e - o * sg.cin * ks;
  const long cc = rem / ks, k = rem - cc * ks;
  wpack[sg.fwd + (((k * (sg.cin / 4) + cc / 4) * sg.cout + o) * 4 + (cc & 3))] = w;
  if (sg.bwd >= 0) {
    const long kr = sg.ks - 1 - k;
    wpack[sg.bwd + (((kr * (sg.cout / 4) + o / 4) * sg.cin + cc) * 4 + (o & 3))] = w;
  }
}

// Adam over the flat dense buffer with the conv-weight repack fused in: a float4 that lies in a
// conv weight segment (segments are 4-float aligned) also writes its four packed copies.
// gdiv > 0: the gradient is an all-reduced sum over gdiv ranks; it becomes the mean first (stored
// back, as grad.div_(world) leaves it) -- DDP's averaging fused into the sweep.
__global__ __launch_bounds__(256) void k_adam_dense_pack(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         long n, AdamScalars s, PackArgs pa,
                                                         float* __restrict__ wpack, float gdiv) {
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = ld4(p + 4 * i), gg = ld4(g + 4 * i), mm = ld4(m + 4 * i), vv = ld4(v + 4 * i);
    if (gdiv > 0.f) {
      gg.x = __fdiv_rn(gg.x, gdiv); gg.y = __fdiv_rn(gg.y, gdiv);
      gg.z = __fdiv_rn(gg.z, gdiv); gg.w = __fdiv_rn(gg.w, gdiv);
      st4(g + 4 * i, gg);
    }
    adam_elem(pp.x, gg.x, mm.x, vv.x, s);
    adam_elem(pp.y, gg.y, mm.y, vv.y, s);
    adam_elem(pp.z, gg.z, mm.z, vv.z, s);
    adam_elem(pp.w, gg.w, mm.w, vv.w, s);
    st4(p + 4 * i, pp); st4(m + 4 * i, mm); st4(v + 4 * i, vv);
    const long e0 = 4 * i;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const PackSeg& sg = pa.seg[q];
      const long len = (long)sg.cout * sg.cin * sg.ks;
      if (e0 >= sg.src && e0 < sg.src + len) {
        const long e = e0 - sg.src;
        pack_store(sg, e + 0, pp.x, wpack);
        pack_store(sg, e + 1, pp.y, wpack);
        pack_store(sg, e + 2, pp.z, wpack);
        pack_store(sg, e + 3, pp.w, wpack);
      }
    }
  }
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gi = g[i];  // tail past the last float4: never a conv weight
    if (gdiv > 0.f) g[i] = gi = __fdiv_rn(gi, gdiv);
    adam_elem(p[i], gi, m[i], v[i], s);
  }
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

// ------------------------------------------------------------- deferred user-table Adam
// The dense sweep's zero-gradient steps, replayed late with the recorded scalars of each step.
// adam_elem is the same function (and `gz` a runtime 0.0f), so every replayed element goes through
// the identical fp32 operation sequence as in k_adam_embed: results are bit-identical.
__device__ __forceinline__ AdamScalars* log_hist(dcue_emb_log* hdr) {
  return reinterpret_cast<AdamScalars*>(hdr + 1);
}

// Bring users' rows current to step_done (before a forward reads them). One workgroup per listed
// user; a row listed twice is claimed by one workgroup (CAS on its clock; INT_MIN = in progress).
__global__ __launch_bounds__(1024) void k_emb_sync(float* __restrict__ p, float* __restrict__ m,
                                                  float* __restrict__ v, dcue_emb_log* hdr,
                                                  int32_t* emb_step, const int64_t* users, int E,
                                                  float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ int s_from;
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  const int64_t u = users[blockIdx.x];
  if (threadIdx.x == 0) {
    int from = T;  // nothing to do
    const int old = emb_step[u];
    if (old != INT_MIN && max(old, F) < T && atomicCAS(&emb_step[u], old, INT_MIN) == old) from = max(old, F);
    s_from = from;
  }
  __syncthreads();
  const int from = s_from;
  if (from >= T) return;
  const AdamScalars* hist = log_hist(hdr);
  for (int j = from + 1 + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  __syncthreads();
  const bool nd = no_decay(hs, from + 1, T, cap, gz);
  float* pr = p + u * E;
  float* mr = m + u * E;
  float* vr = v + u * E;
  // one element per thread: each element's replay is a dependent chain of VALU-bound steps, so the
  // row is spread over as many lanes as it has elements (launch: blockDim >= E)
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    float mm = mr[k], vv = vr[k];
    if (nd && idle_moments(mm, vv)) continue;  // fixed point (idle_moments)
    float pp = pr[k];
    for (int j = from + 1; j <= T; ++j) adam_replay(pp, mm, vv, hs[j % cap], gz);
    pr[k] = pp; mr[k] = mm; vr[k] = vv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    emb_step[u] = T;
  }
}

// Every row current to step_done. Lanes walk the outstanding steps in lockstep (LDS broadcast of
// each step's scalars) and skip the steps their row already has.
__global__ __launch_bounds__(256) void k_emb_flush(float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, const dcue_emb_log* hdr,
                                                   const int32_t* __restrict__ emb_step, long n_rows,
                                                   int E, float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  if (T <= F) return;
  const AdamScalars* hist = log_hist(const_cast<dcue_emb_log*>(hdr));
  // Only the ring's live window [lo, T] is staged (slot j % cap): the full flush may come thousands
  // of steps after the previous one, but the rolling slices keep every row within `cap` steps of T,
  // so no row needs an entry older than lo.
  const int lo = max(F + 1, T - cap + 1);
  for (int j = lo + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  __syncthreads();
  const bool nd = no_decay(hs, lo, T, cap, gz);
  const long stride = (long)gridDim.x * blockDim.x;
  if ((E & 3) == 0) {
    const int E4 = E >> 2;
    const long n4 = n_rows * E4;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const int from = max(emb_step[i / E4], F);
      float4 mm = ld4(m + 4 * i), vv = ld4(v + 4 * i);
      if (nd && idle_moments4(mm, vv)) continue;  // fixed point (idle_moments)
      float4 pp = ld4(p + 4 * i);
      for (int j = max(from + 1, lo); j <= T; ++j) {
        const AdamScalars s = hs[j % cap];
        adam_replay(pp.x, mm.x, vv.x, s, gz);
        adam_replay(pp.y, mm.y, vv.y, s, gz);
        adam_replay(pp.z, mm.z, vv.z, s, gz);
        adam_replay(pp.w, mm.w, vv.w, s, gz);
      }
      st4(p + 4 * i, pp); st4(m + 4 * i, mm); st4(v + 4 * i, vv);
    }
  } else {
    const long n = n_rows * E;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const int from = max(emb_step[i / E], F);
      float mm = m[i], vv = v[i];
      if (nd && idle_moments(mm, vv)) continue;
      float pp = p[i];
      for (int j = max(from + 1, lo); j <= T; ++j) adam_replay(pp, mm, vv, hs[j % cap], gz);
      p[i] = pp; m[i] = mm; v[i] = vv;
    }
  }
}

__global__ void k_emb_flush_done(dcue_emb_log* hdr) { hdr->flush_step = hdr->step_done; }

// Rolling flush: at step t the rows of chunk t mod cap (a contiguous 1/cap of the table) are brought
// current, so every row is replayed at least once per `cap` steps -- the replay work spread evenly
// over the steps (it runs on the user-tower stream, beside the item tower) instead of a full-table
// sweep every cap steps. A workgroup owns whole rows: it reads their clocks, replays, then sets them.
__global__ __launch_bounds__(256) void k_emb_flush_rows(float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, const dcue_emb_log* hdr,
                                                        int32_t* emb_step, long r0, long r1, int E,
                                                        int rows_per_block, float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ int from_s[256];
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  const long rb = r0 + (long)blockIdx.x * rows_per_block;
  const int nr = (int)min((long)rows_per_block, r1 - rb);
  if (nr <= 0) return;
  const AdamScalars* hist = reinterpret_cast<const AdamScalars*>(hdr + 1);
  const int lo = max(F + 1, T - cap + 1);
  for (int j = lo + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  for (int i = threadIdx.x; i < nr; i += blockDim.x) from_s[i] = max(emb_step[rb + i], F);
  __syncthreads();
  const bool nd = no_decay(hs, lo, T, cap, gz);
  if ((E & 3) == 0) {
    const int E4 = E >> 2;
    for (int e = threadIdx.x; e < nr * E4; e += blockDim.x) {
      const int i = e / E4;
      const long off = (rb + i) * E + 4 * (e - i * E4);
      float4 mm = ld4(m + off), vv = ld4(v + off);
      if (nd && idle_moments4(mm, vv)) continue;  // fixed point (idle_moments)
      float4 pp = ld4(p + off);
      for (int j = from_s[i] + 1; j <= T; ++j) {
        const AdamScalars s = hs[j % cap];
        adam_replay(pp.x, mm.x, vv.x, s, gz);
        adam_replay(pp.y, mm.y, vv.y, s, gz);
        adam_replay(pp.z, mm.z, vv.z, s, gz);
        adam_replay(pp.w, mm.w, vv.w, s, gz);
      }
      st4(p + off, pp); st4(m + off, mm); st4(v + off, vv);
    }
  } else {
    for (int e = threadIdx.x; e < nr * E; e += blockDim.x) {
      const int i = e / E;
      const long off = (rb + i) * E + (e - i * E);
      float mm = m[off], vv = v[off];
      if (nd && idle_moments(mm, vv)) continue;
      float pp = p[off];
      for (int j = from_s[i] + 1; j <= T; ++j) adam_replay(pp, mm, vv, hs[j % cap], gz);
      p[off] = pp; m[off] = mm; v[off] = vv;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += blockDim.x) emb_step[rb + i] = T;
}

int launch_emb_flush_rows(const dcue_model* md, int step, hipStream_t s) {
  const long n = md->dims.n_users;
  const int cap = md->emb_log_cap, E = md->dims.user_embdim;
  const int k = step % cap;
  const long r0 = n * k / cap, r1 = n * (k + 1) / cap;
  if (r1 <= r0) return DCUE_OK;
  int rpb = 1024 / E;
  if (rpb < 1) rpb = 1;
  if (rpb > 256) rpb = 256;
  const long blocks = (r1 - r0 + rpb - 1) / rpb;
  TimerScope tsc;
  int st = timer_begin(&tsc, DCUE_TIMED_EMB_SLICE, s);
  if (st) return st;
  DCUE_LAUNCH(k_emb_flush_rows, dim3((unsigned)blocks), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, r0, r1, E, rpb, 0.f);
  DCUE_LAUNCH_CHECK();
  return timer_end(&tsc);
}



// Step t for the rows that have a gradient (emb_rows from the backward); records step t's scalars.
__global__ __launch_bounds__(256) void k_adam_touched(float* __restrict__ p, float* __restrict__ m,
                                                      float* __restrict__ v,
                                                      const float* __restrict__ gcompact,
                                                      const int64_t* emb_rows, int32_t* emb_step,
                                                      dcue_emb_log* hdr, int E, int t, AdamScalars s,
                                                      float gz) {
  __shared__ int s_from;
  const int cap = hdr->cap, F = hdr->flush_step;
  const int n = hdr->grad_step == t ? hdr->n_touched : 0;
  const AdamScalars* hist = log_hist(hdr);
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    const int64_t u = emb_rows[b];
    if (u < 0) continue;
    if (threadIdx.x == 0) s_from = max(emb_step[u], F);
    __syncthreads();
    const int from = s_from;
    float* pr = p + u * E;
    float* mr = m + u * E;
    float* vr = v + u * E;
    const float* gr = gcompact + (long)b * E;
    for (int k = threadIdx.x; k < E; k += blockDim.x) {
      float pp = pr[k], mm = mr[k], vv = vr[k];
      for (int j = from + 1; j < t; ++j) adam_replay(pp, mm, vv, hist[j % cap], gz);  // normally none
      adam_elem(pp, gr[k], mm, vv, s);
      pr[k] = pp; mr[k] = mm; vr[k] = vv;
    }
    __syncthreads();
    if (threadIdx.x == 0) emb_step[u] = t;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    log_hist(hdr)[t % cap] = s;
    hdr->step_done = t;
  }
}

__global__ void k_emb_log_init(dcue_emb_log* hdr, int cap, int step) {
  hdr->step_done = step;
  hdr->flush_step = step;
  hdr->n_touched = 0;
  hdr->grad_step = -1;
  hdr->cap = cap;
}

int launch_emb_log_init(const dcue_model* md, int cap, int step, hipStream_t s) {
  DCUE_HIP_CHECK(hipMemsetAsync(md->emb_step, 0, sizeof(int32_t) * md->dims.n_users, s));
  DCUE_LAUNCH(k_emb_log_init, dim3(1), dim3(1), 0, s, md->emb_log, cap, step);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_emb_sync(const dcue_model* md, const int64_t* users, int n, hipStream_t s) {
  if (n <= 0) return DCUE_OK;
  const int E = md->dims.user_embdim;
  const int threads = E <= 64 ? 64 : (E >= 1024 ? 1024 : (E + 63) / 64 * 64);
  DCUE_LAUNCH(k_emb_sync, dim3((unsigned)n), dim3(threads), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, users, md->dims.user_embdim, 0.f);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_emb_flush(const dcue_model* md, hipStream_t s) {
  const long n = md->dims.n_users * (long)md->dims.user_embdim;
  long blocks = (n / 4 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  TimerScope tsc;
  int st = timer_begin(&tsc, DCUE_TIMED_EMB_FLUSH, s);
  if (st) return st;
  DCUE_LAUNCH(k_emb_flush, dim3((unsigned)blocks), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, (long)md->dims.n_users,
                     md->dims.user_embdim, 0.f);
  DCUE_LAUNCH_CHECK();
  if ((st = timer_end(&tsc))) return st;
  DCUE_LAUNCH(k_emb_flush_done, dim3(1), dim3(1), 0, s, md->emb_log);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_adam(const dcue_model* md, const dcue_adam_args* a, const int64_t* poff, hipStream_t s,
                bool flush_slice) {
  // host scalars as torch.optim.Adam forms them from Python floats (double), each rounded once to
  // float where the CPU kernel takes it as a float scalar
  const double bc1 = 1.0 - pow(a->beta1, (double)a->step);
  const double bc2 = 1.0 - pow(a->beta2, (double)a->step);
  const double w = 1.0 - a->beta1;
  AdamScalars sc;
  sc.neg_step = (float)(-(a->lr / bc1));
  sc.lerp_c = w < 0.5 ? (float)w : (float)w - 1.0f;
  sc.b2 = (float)a->beta2;
  sc.one_m_b2 = (float)(1.0 - a->beta2);
  sc.bc2_sqrt = (float)pow(bc2, 0.5);  // bias_correction2 ** 0.5
  sc.eps = (float)a->eps;
  sc.wd = (float)a->weight_decay;
  sc.inv_bc2_sqrt = 1.0f / sc.bc2_sqrt;  // IEEE single division on the host: RN(1/bc2_sqrt)
  const float gdiv = a->grad_div > 1.0 ? (float)a->grad_div : 0.f;
  const int parts = a->parts ? a->parts : (DCUE_ADAM_DENSE | DCUE_ADAM_EMBEDDING);
  const long n = poff[DCUE_N_DENSE_SEGMENTS];
  if (parts & DCUE_ADAM_DENSE) {  // Adam + the conv-weight repack in one sweep
    DCUE_LAUNCH(k_adam_dense_pack, dim3(512), dim3(256), 0, s, md->params, md->grads, md->exp_avg,
                       md->exp_avg_sq, n, sc, pack_args(md, poff), md->wpack, gdiv);
    DCUE_LAUNCH_CHECK();
  }
  if ((parts & DCUE_ADAM_EMBEDDING) && md->emb_step) {
    DCUE_LAUNCH(k_adam_touched, dim3(256), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                       md->emb_exp_avg_sq, md->emb_grad, md->emb_rows, md->emb_step, md->emb_log,
                       md->dims.user_embdim, a->step, sc, 0.f);
    DCUE_LAUNCH_CHECK();
    // this step's slice of the rolling flush (or the caller issues it later: StepOpts)
    return flush_slice ? launch_emb_flush_rows(md, a->step, s) : DCUE_OK;
  } else if ((parts & DCUE_ADAM_EMBEDDING) && md->dims.n_users > 0) {
    long blocks = (md->dims.n_users + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    TimerScope tsc;
    int st = timer_begin(&tsc, DCUE_TIMED_ADAM_EMBED, s);
    if (st) return st;
    DCUE_LAUNCH(k_adam_embed, dim3((unsigned)blocks), dim3(256), 0, s, md->emb,
                       md->emb_exp_avg, md->emb_exp_avg_sq, md->emb_grad, md->emb_slot,
                       (long)md->dims.n_users, md->dims.user_embdim, sc);
    DCUE_LAUNCH_CHECK();
    if ((st = timer_end(&tsc))) return st;
  }
  return DCUE_OK;
}

// ------------------------------------------------------------------------- weight packing
// conv layer l forward B operand: [k][cin/4][cout][4]; dgrad (l >= 2): [k'][cout/4][cin][4] with
// k' = ks-1-k.
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

PackArgs pack_args(const dcue_model* md, const int64_t* poff) {
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
  return pa;
}

int launch_pack(const dcue_model* md, const int64_t* poff, hipStream_t s) {
  const PackArgs pa = pack_args(md, poff);
  DCUE_LAUNCH(k_pack, dim3(64, 5), dim3(256), 0, s, md->params, md->wpack, pa);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
