// SGD + Nesterov and Ranger (RAdam + Lookahead) over the flat dense buffer and the user table --
// gfx950. Reference: DCUE._init_nn, nn/dcue.py:148-157 (optimize='sgd' | 'ranger'), optim/ranger.py.
//
// Per element, each form below is the rounding of torch 2.10's CPU kernel for the reference's tensor
// op (oracle/optim_oracle.py restates them; tests/test_adam_cpu.py pins that restatement bit for bit
// against the reference's Ranger and torch.optim.SGD). Built with fp contraction off: only the
// explicit __fmaf_rn are fused.
//
// The user table has a dense gradient in the reference (nn.Embedding, sparse=False), so every row
// steps every step, rows outside the batch with g = 0 -- the same literal sweep as NativeAdam's
// non-deferred mode (a row's compact gradient comes from emb_slot / emb_grad and its slot is cleared).
#include "dcue_internal.h"

namespace dcue {

struct OptScalars {
  int kind, rect, sync, first;  // rect: RAdam rectified step; sync: lookahead step; first: SGD step 1
  float b1, one_m_b1, b2, one_m_b2;
  float neg_wd_lr, neg_step, eps, alpha;  // Ranger
  float wd, momentum, neg_lr;             // SGD
};

// torch.optim.SGD(momentum, dampening=0, nesterov=True), torch/optim/sgd.py _single_tensor_sgd:
//   g = grad.add(p, alpha=wd); buf = clone(g) | buf.mul_(m).add_(g); g = g.add(buf, alpha=m);
//   p.add_(g, alpha=-lr)
__device__ __forceinline__ void sgd_elem(float& p, float g, float& buf, const OptScalars& s) {
#pragma clang fp contract(off)
  if (s.wd != 0.f) g = __fmaf_rn(p, s.wd, g);
  buf = s.first ? g : __fmaf_rn(g, 1.0f, __fmul_rn(buf, s.momentum));
  g = __fmaf_rn(buf, s.momentum, g);
  p = __fmaf_rn(g, s.neg_lr, p);
}

// optim/ranger.py:121-163 for one element: moments, optional decoupled decay, the rectified (or
// momentum-only) step, and every k-th step the lookahead interpolation into the slow weights.
__device__ __forceinline__ void ranger_elem(float& p, float g, float& m, float& v, float& slow,
                                            const OptScalars& s) {
#pragma clang fp contract(off)
  v = __fmaf_rn(__fmul_rn(s.one_m_b2, g), g, __fmul_rn(v, s.b2));  // mul_(b2).addcmul_(1-b2, g, g)
  m = __fmaf_rn(g, s.one_m_b1, __fmul_rn(m, s.b1));               // mul_(b1).add_(1-b1, g)
  if (s.neg_wd_lr != 0.f) p = __fmaf_rn(p, s.neg_wd_lr, p);        // add_(-wd*lr, p)
  if (s.rect) {
    const float denom = __fadd_rn(__builtin_sqrtf(v), s.eps);      // correctly rounded sqrt
    p = __fadd_rn(p, __fdiv_rn(__fmul_rn(s.neg_step, m), denom));  // addcdiv_(-step*lr, m, denom)
  } else {
    p = __fmaf_rn(m, s.neg_step, p);                               // add_(-step*lr, m)
  }
  if (s.sync) {                                                    // slow.add_(alpha, p - slow)
    slow = __fmaf_rn(__fsub_rn(p, slow), s.alpha, slow);
    p = slow;
  }
}

__device__ __forceinline__ void opt_elem(float& p, float g, float* a, float* b, float* c, long i,
                                         const OptScalars& s) {
  if (s.kind == DCUE_OPT_SGD) {
    sgd_elem(p, g, a[i], s);
  } else {
    ranger_elem(p, g, a[i], b[i], c[i], s);
  }
}

__global__ __launch_bounds__(256) void k_opt_dense(float* __restrict__ p, float* __restrict__ g, float* a,
                                                   float* b, float* c, long n, OptScalars s, float gdiv) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (gdiv > 0.f) g[i] = gi = __fdiv_rn(gi, gdiv);  // DDP mean of an all-reduced sum
    float pi = p[i];
    opt_elem(pi, gi, a, b, c, i, s);
    p[i] = pi;
  }
}

// one wave per user row; a row without a gradient this step takes g = 0, then its slot is cleared
__global__ __launch_bounds__(256) void k_opt_embed(float* __restrict__ p, float* a, float* b, float* c,
                                                   const float* __restrict__ gcompact, int32_t* slot,
                                                   long n_rows, int E, OptScalars s) {
  const int lane = threadIdx.x & 63;
  const long wave0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave0; r < n_rows; r += nwaves) {
    const int sl = slot[r];
    const float* gr = sl >= 0 ? gcompact + (long)sl * E : nullptr;
    for (int k = lane; k < E; k += 64) {
      const long i = r * E + k;
      float pi = p[i];
      opt_elem(pi, gr ? gr[k] : 0.f, a, b, c, i, s);
      p[i] = pi;
    }
    if (lane == 0 && sl >= 0) slot[r] = -1;
  }
}

int launch_opt(const dcue_model* md, const dcue_opt_args* a, const dcue_opt_state* st, long n_dense,
               hipStream_t s) {
  OptScalars sc = {};
  sc.kind = a->kind;
  const double t = (double)a->step;
  if (a->kind == DCUE_OPT_SGD) {
    sc.first = a->step == 1;
    sc.wd = (float)a->weight_decay;
    sc.momentum = (float)a->beta1;
    sc.neg_lr = (float)(-a->lr);
  } else {
    // optim/ranger.py:132-145, Python-float arithmetic in the reference's operation order
    const double beta1 = a->beta1, beta2 = a->beta2;
    const double beta2_t = pow(beta2, t);
    const double n_sma_max = 2 / (1 - beta2) - 1;
    const double n_sma = n_sma_max - 2 * t * beta2_t / (1 - beta2_t);
    double step_size;
    sc.rect = n_sma > a->n_sma_threshold;
    if (sc.rect)
      step_size = sqrt((1 - beta2_t) * (n_sma - 4) / (n_sma_max - 4) * (n_sma - 2) / n_sma * n_sma_max /
                       (n_sma_max - 2)) / (1 - pow(beta1, t));
    else
      step_size = 1.0 / (1 - pow(beta1, t));
    sc.b1 = (float)beta1;
    sc.one_m_b1 = (float)(1 - beta1);
    sc.b2 = (float)beta2;
    sc.one_m_b2 = (float)(1 - beta2);
    sc.neg_wd_lr = (float)(-a->weight_decay * a->lr);
    sc.neg_step = (float)(-step_size * a->lr);
    sc.eps = (float)a->eps;
    sc.alpha = (float)a->alpha;
    sc.sync = a->step % a->k == 0;
  }
  const float gdiv = a->grad_div > 1.0 ? (float)a->grad_div : 0.f;
  DCUE_LAUNCH(k_opt_dense, dim3(512), dim3(256), 0, s, md->params, md->grads, st->dense_a, st->dense_b,
              st->dense_c, n_dense, sc, gdiv);
  DCUE_LAUNCH_CHECK();
  if (md->dims.n_users > 0) {
    long blocks = (md->dims.n_users + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    DCUE_LAUNCH(k_opt_embed, dim3((unsigned)blocks), dim3(256), 0, s, md->emb, st->emb_a, st->emb_b, st->emb_c,
                md->emb_grad, md->emb_slot, (long)md->dims.n_users, md->dims.user_embdim, sc);
    DCUE_LAUNCH_CHECK();
  }
  return DCUE_OK;
}

}  // namespace dcue
