// Everything after the conv stack: small GEMMs (fc projection, user tower) on MFMA, cosine scoring
// + hinge loss, copy bookkeeping of in-batch negatives, embedding-row gradients -- gfx950.
//
// Reference ops replaced:
//   fc Linear(d,d) on BN5 output                           truedcuemel1dbn.py:65,101
//   UserEmbeddings: gather, relu, linear, relu, linear      userembedding.py:33-44
//   nn.CosineSimilarity(dim=1) scoring, pos - neg           dcue/dcue.py:68,94-106
//   hinge loss mean_b sum_n max(0, margin - s)              nn/dcue.py:167-170
//   in-batch copies pos[rand] -> neg[i][j]                  nn/dcue.py:698-709
// These are tiny (B=64 rows, d<=256, E<=1024): the kernels are shaped for latency -- one wave per
// 16x16 output tile, per batch row or per item -- with fixed summation orders throughout (bitwise
// reproducible run to run).
#include "dcue_internal.h"
#include "tgemm.h"

DCUE_KTRACE_READER(tail)  // diagnostic builds only (dcue_common.h)

namespace dcue {

// ------------------------------------------------------------------------ batch bookkeeping
// copies of each item (BatchNorm weights): catalogue = 1 each; gather = its positive (items < B)
// plus the negatives that reference it. One wave per item, 64 references per ballot.
__global__ __launch_bounds__(256) void k_item_counts(dcue_batch b, float* counts) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= b.n_items) return;
  if (b.layout == DCUE_LAYOUT_CATALOGUE) {
    if (lane == 0) counts[i] = 1.f;
    return;
  }
  const int nneg = b.n_rows * b.n_neg;
  int cnt = i < b.n_rows ? 1 : 0;
  constexpr int kBatch = 16;  // loads in flight per lane before the ballots
  for (int e0 = 0; e0 < nneg; e0 += 64 * kBatch) {
    int32_t v[kBatch];
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      const int e = e0 + 64 * q + lane;
      v[q] = e < nneg ? b.neg_item[e] : -1;
    }
#pragma unroll
    for (int q = 0; q < kBatch; ++q) cnt += __popcll(__ballot(v[q] == i));
  }
  if (lane == 0) counts[i] = (float)cnt;
}

int launch_item_counts(const dcue_batch* b, float* counts, hipStream_t s) {
  DCUE_LAUNCH(k_item_counts, dim3((b->n_items + 3) / 4), dim3(256), 0, s, *b, counts);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

template <int TA, int TB, int AKF, int BNF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_tgemm(TGemmArgs g) {
  critical_path_priority();
  __shared__ TgLds L;
  tgemm_block<TA, TB, AKF, BNF>(g, blockIdx.x, blockIdx.y, L, threadIdx.x);
}

// Two independent GEMMs in one launch (their blocks side by side on a 1-D grid: the first
// nb1 = gx1 * gy1 blocks are GEMM 1's). The user tower's backward pairs (dW2, dh1) and (dW1, de):
// each pair reads the same inputs and writes disjoint outputs, one launch instead of two.
template <int TA1, int TB1, int AK1, int BN1, int TA2, int TB2, int AK2, int BN2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_tgemm2(TGemmArgs g1, TGemmArgs g2,
                                                                                          int gx1, int nb1, int gx2) {
  __shared__ TgLds L;
  const int b = blockIdx.x;
  if (b < nb1)
    tgemm_block<TA1, TB1, AK1, BN1>(g1, b % gx1, b / gx1, L, threadIdx.x);
  else
    tgemm_block<TA2, TB2, AK2, BN2>(g2, (b - nb1) % gx2, (b - nb1) / gx2, L, threadIdx.x);
}

// the user tower's backward pairs: g1 = a weight gradient (A = du / dh1 k-strided, B = relu(h1) /
// relu(E[u]) n-contiguous), g2 = an input gradient (A k-contiguous, B n-contiguous, masked)
int launch_tgemm_pair(const TGemmArgs& g1, const TGemmArgs& g2, hipStream_t s) {
  if (g1.M <= 0 || g1.N <= 0 || g2.M <= 0 || g2.N <= 0) return DCUE_ERR_INVALID;
  if (!(g1.sak != 1 && g1.sbn == 1 && g2.sak == 1 && g2.sbn == 1)) return DCUE_ERR_INVALID;
  const int gx1 = (g1.M + 15) / 16, gy1 = (g1.N + 63) / 64;
  const int gx2 = (g2.M + 15) / 16, gy2 = (g2.N + 63) / 64;
  DCUE_LAUNCH((k_tgemm2<0, 1, 0, 1, 0, 0, 1, 1>), dim3((unsigned)(gx1 * gy1 + gx2 * gy2)), dim3(256), 0, s, g1, g2,
              gx1, gx1 * gy1, gx2);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_tgemm(int ta, int tb, const TGemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return DCUE_OK;
  const dim3 grid((unsigned)((g.M + 15) / 16), (unsigned)((g.N + 63) / 64));
  const int akf = g.sak == 1, bnf = g.sbn == 1;
  const int key = ((ta * 3 + tb) * 2 + akf) * 2 + bnf;
#define DCUE_TG(TA_, TB_, AK_, BN_)                                                            \
  case ((TA_ * 3 + TB_) * 2 + AK_) * 2 + BN_:                                                  \
    DCUE_LAUNCH((k_tgemm<TA_, TB_, AK_, BN_>), grid, dim3(256), 0, s, g);               \
    break;
  switch (key) {
    DCUE_TG(0, 0, 0, 0) DCUE_TG(0, 0, 0, 1) DCUE_TG(0, 0, 1, 0) DCUE_TG(0, 0, 1, 1)
    DCUE_TG(0, 1, 0, 0) DCUE_TG(0, 1, 0, 1) DCUE_TG(0, 1, 1, 0) DCUE_TG(0, 1, 1, 1)
    DCUE_TG(0, 2, 0, 0) DCUE_TG(0, 2, 0, 1) DCUE_TG(0, 2, 1, 0) DCUE_TG(0, 2, 1, 1)
    DCUE_TG(1, 0, 0, 0) DCUE_TG(1, 0, 0, 1) DCUE_TG(1, 0, 1, 0) DCUE_TG(1, 0, 1, 1)
    DCUE_TG(2, 0, 0, 0) DCUE_TG(2, 0, 0, 1) DCUE_TG(2, 0, 1, 0) DCUE_TG(2, 0, 1, 1)
    default: return DCUE_ERR_INVALID;
  }
#undef DCUE_TG
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ------------------------------------------------------------------- scores and hinge loss
__device__ __forceinline__ int copy_item(const dcue_batch& b, int row, int c) {
  if (c == 0) return row;
  if (b.layout == DCUE_LAYOUT_CATALOGUE) return b.n_rows + row * b.n_neg + (c - 1);
  return b.neg_item[(long)row * b.n_neg + (c - 1)];
}

// One workgroup (4 waves) per row; wave w scores copies w, w+4, ...:
// torch cosine_similarity = sum((x/max(|x|,eps)) * (y/max(|y|,eps))) -- normalise, then dot.
// cosv[b][c] (c=0 positive), norms[b][0]=|u|, norms[b][1+c]=|f_c|; scores = pos - neg;
// hinge[b][j] = max(0, margin - s); dhinge = d(mean_b sum_j hinge)/ds (torch.max splits ties 1/2).
__global__ __launch_bounds__(256) void k_score_fwd(const float* __restrict__ uf,
                                                   const float* __restrict__ f, dcue_batch b, int d,
                                                   float margin, float* scores, float* cosv,
                                                   float* norms, float* hinge, float* dhinge) {
  __shared__ float cs[1025];
  const int row = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = b.n_neg, per = (d + 63) / 64;
  const float eps = 1e-8f;
  float u[4];
  float su = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = lane + 64 * e;
    u[e] = (e < per && k < d) ? uf[(long)row * d + k] : 0.f;
    su += u[e] * u[e];
  }
  const float nu = sqrtf(wave_sum(su));
  const float du = fmaxf(nu, eps);
  if (wave == 0 && lane == 0) norms[(long)row * (N + 2)] = nu;
  for (int c = wave; c <= N; c += 4) {
    const long item = copy_item(b, row, c);
    float v[4], sf = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      v[e] = (e < per && k < d) ? f[item * d + k] : 0.f;
      sf += v[e] * v[e];
    }
    const float nf = sqrtf(wave_sum(sf));
    const float dfn = fmaxf(nf, eps);
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) dot += (u[e] / du) * (v[e] / dfn);
    const float cv = wave_sum(dot);
    if (lane == 0) {
      norms[(long)row * (N + 2) + 1 + c] = nf;
      cosv[(long)row * (N + 1) + c] = cv;
      cs[c] = cv;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const float sc = cs[0] - cs[1 + j];
    const float h = margin - sc;
    scores[(long)row * N + j] = sc;
    hinge[(long)row * N + j] = h > 0.f ? h : 0.f;
    dhinge[(long)row * N + j] = h > 0.f ? -1.f / (float)b.n_rows : (h == 0.f ? -0.5f / (float)b.n_rows : 0.f);
  }
}

// loss = mean over rows of the row's summed hinge (row sums in j order, rows in order)
__global__ __launch_bounds__(256) void k_loss_mean(const float* hinge, int B, int N, float* loss) {
  __shared__ float rs[1024];
  for (int r = threadIdx.x; r < B; r += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < N; ++j) s += hinge[(long)r * N + j];
    rs[r] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int r = 0; r < B; ++r) s += rs[r];
    *loss = s / (float)B;
  }
}

int launch_score_fwd(const float* uf, const float* f, const dcue_batch* b, int d, float margin,
                     float* scores, float* cosv, float* norms, float* hinge, float* loss,
                     float* dhinge, hipStream_t s) {
  if (d > 256 || b->n_neg > 1024 || b->n_rows > 1024) return DCUE_ERR_UNSUPPORTED;
  DCUE_LAUNCH(k_score_fwd, dim3(b->n_rows), dim3(256), 0, s, uf, f, *b, d, margin, scores, cosv,
                     norms, hinge, dhinge);
  DCUE_LAUNCH_CHECK();
  DCUE_LAUNCH(k_loss_mean, dim3(1), dim3(256), 0, s, hinge, b->n_rows, b->n_neg, loss);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// Forward + hinge backward of one row per workgroup (plans: the loss gradient is known here, so
// k_score_bwd's pass is folded in). Same arithmetic and summation orders as k_score_fwd,
// k_loss_mean and k_score_bwd; the loss mean (k_loss_mean's sums) is taken by the next kernel,
// k_item_grad, from the row sums. CPW > 0: at most CPW copies per wave -- every copy's index and
// feature row are loaded at once, up front, and the rows stay in registers for the backward (one
// load round instead of two per copy); CPW == 0: any N, copy by copy.
template <int CPW>
__global__ __launch_bounds__(256) void k_score_fused(const float* __restrict__ uf,
                                                     const float* __restrict__ f, dcue_batch b, int d,
                                                     float margin, float* scores, float* cosv,
                                                     float* norms, float* rowsum, float* dU,
                                                     float* dfcopy, DevWait uf_wait) {
  critical_path_priority();
  DCUE_KTW(0, 6);
  DCUE_KT(0, 0);
  constexpr int CMAX = CPW > 0 ? 4 * CPW : 1025;
  __shared__ float cs[CMAX], dcs[CMAX], hs[CMAX];
  __shared__ float gus[4][256];
  const int row = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = b.n_neg, per = (d + 63) / 64;
  const float eps = 1e-8f;
  constexpr int CR = CPW > 0 ? CPW : 1;  // register-resident copies
  float v[CR][4];
  float nfr[CR];
  if constexpr (CPW > 0) {
    int item[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const int c = wave + 4 * q;
      item[q] = c <= N ? copy_item(b, row, c) : row;
    }
#pragma unroll
    for (int q = 0; q < CPW; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = lane + 64 * e;
        v[q][e] = (wave + 4 * q <= N && e < per && k < d) ? f[(long)item[q] * d + k] : 0.f;
      }
  }
  // (plans: uf comes from the user stream; the copies' features above are this stream's)
  dev_wait(uf_wait);
  float u[4];
  float su = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = lane + 64 * e;
    u[e] = (e < per && k < d) ? uf[(long)row * d + k] : 0.f;
    su += u[e] * u[e];
  }
  const float nu = sqrtf(wave_sum(su));
  DCUE_KT(0, 2);
  const float du = fmaxf(nu, eps);
  if (wave == 0 && lane == 0) norms[(long)row * (N + 2)] = nu;
  auto score_copy = [&](int c, const float (&w)[4]) {
    float sf = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) sf += w[e] * w[e];
    const float nf = sqrtf(wave_sum(sf));
    const float dfn = fmaxf(nf, eps);
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) dot += (u[e] / du) * (w[e] / dfn);
    const float cv = wave_sum(dot);
    if (lane == 0) {
      norms[(long)row * (N + 2) + 1 + c] = nf;
      cosv[(long)row * (N + 1) + c] = cv;
      cs[c] = cv;
    }
    return nf;
  };
  if constexpr (CPW > 0) {
    // score_copy's arithmetic for the wave's CPW copies at once: each cross-lane sum's six
    // shuffle steps run for all copies together, so their latencies overlap instead of adding up
    // (the same operations per value in the same order as score_copy: the same bits)
    float sq[CPW], dq[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      float sf = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) sf += v[q][e] * v[q][e];
      sq[q] = sf;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int q = 0; q < CPW; ++q) sq[q] += __shfl_xor(sq[q], off, 64);
    float un[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) un[e] = u[e] / du;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      nfr[q] = sqrtf(sq[q]);
      const float dfn = fmaxf(nfr[q], eps);
      float dot = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) dot += un[e] * (v[q][e] / dfn);
      dq[q] = dot;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int q = 0; q < CPW; ++q) dq[q] += __shfl_xor(dq[q], off, 64);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < CPW; ++q) {
        const int c = wave + 4 * q;
        if (c <= N) {
          norms[(long)row * (N + 2) + 1 + c] = nfr[q];
          cosv[(long)row * (N + 1) + c] = dq[q];
          cs[c] = dq[q];
        }
      }
    }
  } else {
    for (int c = wave; c <= N; c += 4) {
      const long item = copy_item(b, row, c);
      float w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = lane + 64 * e;
        w[e] = (e < per && k < d) ? f[item * d + k] : 0.f;
      }
      score_copy(c, w);
    }
  }
  DCUE_KT(0, 1);
  __syncthreads();
  const float invB = 1.f / (float)b.n_rows;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const float sc = cs[0] - cs[1 + j];
    const float h = margin - sc;
    scores[(long)row * N + j] = sc;
    hs[j] = h > 0.f ? h : 0.f;
    // dL/dscore (torch.max splits ties 1/2); d score / d neg cos = -1
    const float dh = h > 0.f ? -1.f * invB : (h == 0.f ? -0.5f * invB : 0.f);
    dcs[1 + j] = -dh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f, dpos = 0.f;
    for (int j = 0; j < N; ++j) {
      s += hs[j];
      dpos += -dcs[1 + j];  // the positive collects every score's gradient, in j order
    }
    dcs[0] = dpos;
    rowsum[row] = s;
  }
  __syncthreads();
  DCUE_KT(0, 3);
  // backward of the cosines: d cos/dx = (yhat - cos*xhat)/|x|
  const float nuc = fmaxf(nu, eps);
  float uh[4], gu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    uh[e] = u[e] / nuc;
    gu[e] = 0.f;
  }
  const float rnuc = 1.f / nuc;
  auto back_copy = [&](int c, const float (&w)[4], float nf_raw) {
    const float dc = dcs[c];
    const float cv = cs[c];
    const float nf = fmaxf(nf_raw, eps);
    const float rnf = 1.f / nf;  // divisions as products, as k_score_bwd (the same bits)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      if (e < per && k < d) {
        const float fh = w[e] * rnf;
        gu[e] += dc * (fh - cv * uh[e]) * rnuc;
        dfcopy[((long)row * (N + 1) + c) * d + k] = dc * (uh[e] - cv * fh) * rnf;
      }
    }
  };
  if constexpr (CPW > 0) {
#pragma unroll
    for (int q = 0; q < CPW; ++q)
      if (wave + 4 * q <= N) back_copy(wave + 4 * q, v[q], nfr[q]);
  } else {
    for (int c = wave; c <= N; c += 4) {
      const long item = copy_item(b, row, c);
      float w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = lane + 64 * e;
        w[e] = (e < per && k < d) ? f[item * d + k] : 0.f;
      }
      back_copy(c, w, norms[(long)row * (N + 2) + 1 + c]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = lane + 64 * e;
    if (e < per && k < d) gus[wave][k] = gu[e];
  }
  DCUE_KT(0, 4);
  __syncthreads();
  for (int k = threadIdx.x; k < d; k += blockDim.x)
    dU[(long)row * d + k] = ((gus[0][k] + gus[1][k]) + gus[2][k]) + gus[3][k];
  DCUE_KT(0, 5);
  DCUE_KTW(0, 7);
}

// DevWait's producer side: stream-ordered after the producer kernel (whose end released its data)
__global__ void k_signal(unsigned* flag, unsigned val) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

int launch_signal(unsigned* flag, unsigned val, hipStream_t s) {
  DCUE_LAUNCH(k_signal, dim3(1), dim3(64), 0, s, flag, val);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_score_fused(const float* uf, const float* f, const dcue_batch* b, int d, float margin,
                       float* scores, float* cosv, float* norms, float* rowsum, float* du,
                       float* dfcopy, hipStream_t s, DevWait uf_wait) {
  if (d > 256 || b->n_neg > 1024 || b->n_rows > 1024) return DCUE_ERR_UNSUPPORTED;
  if (b->n_neg + 1 <= 16)
    DCUE_LAUNCH(k_score_fused<4>, dim3(b->n_rows), dim3(256), 0, s, uf, f, *b, d, margin, scores, cosv,
                norms, rowsum, du, dfcopy, uf_wait);
  else if (b->n_neg + 1 <= 32)
    DCUE_LAUNCH(k_score_fused<8>, dim3(b->n_rows), dim3(256), 0, s, uf, f, *b, d, margin, scores, cosv,
                norms, rowsum, du, dfcopy, uf_wait);
  else
    DCUE_LAUNCH(k_score_fused<0>, dim3(b->n_rows), dim3(256), 0, s, uf, f, *b, d, margin, scores, cosv,
                norms, rowsum, du, dfcopy, uf_wait);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// dL/dscores -> dL/du (waves' partial sums combined in wave order) and dL/df per copy.
// d cos/dx = (yhat - cos*xhat)/|x| (non-degenerate norms).
__global__ __launch_bounds__(256) void k_score_bwd(const float* __restrict__ uf,
                                                   const float* __restrict__ f, dcue_batch b, int d,
                                                   const float* dscores, const float* cosv,
                                                   const float* norms, float* dU, float* dfcopy) {
  __shared__ float gus[4][256];
  const int row = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = b.n_neg, per = (d + 63) / 64;
  const float eps = 1e-8f;
  const float nu = fmaxf(norms[(long)row * (N + 2)], eps);
  const float rnu = 1.f / nu;
  float u[4], gu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = lane + 64 * e;
    u[e] = (e < per && k < d) ? uf[(long)row * d + k] / nu : 0.f;
    gu[e] = 0.f;
  }
  float dpos = 0.f;  // scores = pos_cos - neg_cos: the positive collects every score's gradient
  for (int j = 0; j < N; ++j) dpos += dscores[(long)row * N + j];
  for (int c = wave; c <= N; c += 4) {
    const long item = copy_item(b, row, c);
    const float dc = c == 0 ? dpos : -dscores[(long)row * N + c - 1];
    const float cv = cosv[(long)row * (N + 1) + c];
    const float nf = fmaxf(norms[(long)row * (N + 2) + 1 + c], eps);
    const float rnf = 1.f / nf;  // the backward's divisions as products (k_score_fused: the same)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      if (e < per && k < d) {
        const float fh = f[item * d + k] * rnf;
        gu[e] += dc * (fh - cv * u[e]) * rnu;
        dfcopy[((long)row * (N + 1) + c) * d + k] = dc * (u[e] - cv * fh) * rnf;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = lane + 64 * e;
    if (e < per && k < d) gus[wave][k] = gu[e];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < d; k += blockDim.x)
    dU[(long)row * d + k] = ((gus[0][k] + gus[1][k]) + gus[2][k]) + gus[3][k];
}

int launch_score_bwd(const float* uf, const float* f, const dcue_batch* b, int d,
                     const float* dscores, const float* cosv, const float* norms, float* du,
                     float* dfcopy, hipStream_t s) {
  DCUE_LAUNCH(k_score_bwd, dim3(b->n_rows), dim3(256), 0, s, uf, f, *b, d, dscores, cosv, norms,
                     du, dfcopy);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

constexpr int kItemGradCap = 4096;  // copies per item (B*N + 1 in gather layout)

// df[i] = sum over item i's copies. One workgroup per item: the four waves scan contiguous
// quarters of neg_item with ballots and their hit lists are laid end to end in wave order, which
// lists the copies in (positive, (b,j) row-major) order; each wave then sums a contiguous quarter of
// the list with all its row loads in flight, and the quarters are added in wave order
// (deterministic). With `fc` set the fc input gradient of the item follows in the same workgroup --
// g5[i][n] = sum_k df[i][k] W[k][n] (k in order, the two k halves added) -- with its share of BN5's
// backward sums (sum g5, sum g5*xhat5) into the accumulators. Everything the block reads that does
// not depend on the scan (W into LDS when d <= 128, the item's y5 row, the BN5 stats, the row sums
// for the loss) is loaded up front, so the block waits on memory about three times, not eight.
struct ItemGradFc {
  const float* rowsum;     // nullable: the fused score's per-row hinge sums -> loss (block 0)
  float* loss;
  const float* W;          // fc.weight [d][d] (null: df only)
  float* g5;               // [M][d]
  unsigned long long* acc; // BN5 backward accumulators [2][d]
  const float *y5, *mean5, *invstd5;
  unsigned* g5max;         // nullable: max |g5| per column (ordered keys; split-f16 wgrad bound)
  unsigned* dfmax;         // nullable: max |df| per column
};

constexpr int kItemGradWLds = 128;  // W staged in LDS up to d = 128 (64 KB)
template <bool WLDS>
__global__ __launch_bounds__(256) void k_item_grad(const float* __restrict__ dfcopy, dcue_batch b, int d,
                                                   float* df, ItemGradFc fc) {
  critical_path_priority();
  constexpr int kCap = kItemGradCap;
  __shared__ int list[kCap];      // per-wave hit lists, kCap / 4 each
  __shared__ int lst[kCap + 1];   // the item's copies in order
  __shared__ int s_len, wlen[4], wofs[4];
  __shared__ float part[4][256];
  __shared__ float dfs[256];
  __shared__ float rs[1024];
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [d][d] when WLDS
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x;
  const int N = b.n_neg, B = b.n_rows;
  const bool gather = b.layout != DCUE_LAYOUT_CATALOGUE;

  // ---- up-front loads
  const int nneg = B * N;
  const int e_lo = (int)(((long)nneg * wave) / 4), e_hi = (int)(((long)nneg * (wave + 1)) / 4);
  constexpr int kBatch = 8;
  int32_t nv[kBatch];
  if (gather) {
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      const int e = e_lo + 64 * q + lane;
      nv[q] = e < e_hi ? b.neg_item[e] : -1;
    }
  }
  if constexpr (WLDS) {
    if (fc.W) {
      const int n4 = d * d / 4;
      for (int q = threadIdx.x; q < n4; q += blockDim.x)
        reinterpret_cast<float4*>(wl)[q] = reinterpret_cast<const float4*>(fc.W)[q];
    }
  }
  float y5v = 0.f, mu5 = 0.f, is5 = 0.f;
  const bool col = fc.W && threadIdx.x < d;
  if (col) {
    y5v = fc.y5[(long)i * d + threadIdx.x];
    mu5 = fc.mean5[threadIdx.x];
    is5 = fc.invstd5[threadIdx.x];
  }
  if (fc.rowsum && i == 0)
    for (int r = threadIdx.x; r < B; r += blockDim.x) rs[r] = fc.rowsum[r];

  if (!gather) {
    const long cidx = i < B ? (long)i * (N + 1) : (long)((i - B) / N) * (N + 1) + 1 + (i - B) % N;
    for (int k = threadIdx.x; k < d; k += blockDim.x) {
      const float v = dfcopy[cidx * d + k];
      df[(long)i * d + k] = v;
      dfs[k] = v;
    }
  } else {
    {  // scan: this wave's quarter of the negatives (the first batch is already loaded)
      int len = 0;
      for (int e0 = e_lo; e0 < e_hi; e0 += 64 * kBatch) {
        if (e0 != e_lo) {
#pragma unroll
          for (int q = 0; q < kBatch; ++q) {
            const int e = e0 + 64 * q + lane;
            nv[q] = e < e_hi ? b.neg_item[e] : -1;
          }
        }
#pragma unroll
        for (int q = 0; q < kBatch; ++q) {
          const int e = e0 + 64 * q + lane;
          const bool hit = nv[q] == i;
          const unsigned long long bal = __ballot(hit);
          const int pos = len + __popcll(bal & ((1ull << lane) - 1ull));
          if (hit && pos < kCap / 4) {
            const int row = e / N;
            list[wave * (kCap / 4) + pos] = row * (N + 1) + 1 + (e - row * N);
          }
          len += __popcll(bal);
        }
      }
      if (lane == 0) wlen[wave] = len;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // compact: positive, then the quarters in order
      int n = 0;
      if (i < B) lst[n++] = i * (N + 1);
      for (int w = 0; w < 4; ++w) {
        const int m = wlen[w] < kCap / 4 ? wlen[w] : kCap / 4;
        wofs[w] = n;
        n += m;
      }
      s_len = n;
    }
    __syncthreads();
    for (int w = 0; w < 4; ++w) {
      const int m = wlen[w] < kCap / 4 ? wlen[w] : kCap / 4;
      for (int q = threadIdx.x; q < m; q += blockDim.x) lst[wofs[w] + q] = list[w * (kCap / 4) + q];
    }
    __syncthreads();
    const int len = s_len;
    const int q0 = (len * wave) / 4, q1 = (len * (wave + 1)) / 4;  // this wave's quarter
    const int per = (d + 63) / 64;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    constexpr int kRows = 8;
    for (int qb = q0; qb < q1; qb += kRows) {
      float v[kRows][4];
#pragma unroll
      for (int r = 0; r < kRows; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = lane + 64 * e;
          v[r][e] = (qb + r < q1 && e < per && k < d) ? dfcopy[(long)lst[qb + r] * d + k] : 0.f;
        }
#pragma unroll
      for (int r = 0; r < kRows; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += v[r][e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      if (e < per && k < d) part[wave][k] = acc[e];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < d; k += blockDim.x) {
      const float v = ((part[0][k] + part[1][k]) + part[2][k]) + part[3][k];
      df[(long)i * d + k] = v;
      dfs[k] = v;
    }
  }
  if (fc.W) {
    __syncthreads();
    // g5[i][n] = sum_k df[i][k] W[k][n]: the k range split in halves over the block's two thread
    // halves (first half + second half, fixed order)
    const int hk = (d + 1) / 2;
    for (int t = threadIdx.x; t < 2 * d; t += blockDim.x) {
      const int n = t % d, h = t / d;
      const int k0 = h * hk, k1 = h ? d : hk;
      float g = 0.f;
      if constexpr (WLDS) {
        for (int k = k0; k < k1; ++k) g += dfs[k] * wl[k * d + n];
      } else {
        for (int k = k0; k < k1; k += 16) {  // sixteen weight loads in flight, then the ordered sum
          float wv[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) wv[q] = k + q < k1 ? fc.W[(long)(k + q) * d + n] : 0.f;
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (k + q < k1) g += dfs[k + q] * wv[q];
        }
      }
      part[h][n] = g;
    }
    __syncthreads();
    if (col) {
      const int n = threadIdx.x;
      const float g = part[0][n] + part[1][n];
      fc.g5[(long)i * d + n] = g;
      if (fc.g5max) atomicMax(fc.g5max + n, ord_key(fabsf(g)));
      const float xh = (y5v - mu5) * is5;
      acc128_add(acc_at(fc.acc, d, 0, n), g);
      acc128_add(acc_at(fc.acc, d, 1, n), g * xh);
    }
  }
  if (fc.dfmax) {
    __syncthreads();
    for (int k = threadIdx.x; k < d; k += blockDim.x) atomicMax(fc.dfmax + k, ord_key(fabsf(dfs[k])));
  }
  if (fc.rowsum && i == 0) {  // loss = mean of the row sums in row order (k_loss_mean's sums)
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int r = 0; r < B; ++r) s += rs[r];
      *fc.loss = s / (float)B;
    }
  }
}

// IT items per workgroup: the fc weight is staged once per IT items (k_item_grad stages it once per
// item: 64 KB of L2 reads per item, 86 MB a catalogue step, which made that kernel 80 us), and
// BN5's sums leave the block once per column. Item i's copies: catalogue, its one copy; gather, the
// prologue's list (positive first, then (row, j) order). Wave w sums items w, w+4, ... copy by copy
// in list order (eight row loads in flight); the fc input gradient g5 = df W splits k in halves over
// the two thread halves, items inner (fixed order); BN5's per-column sums add the block's items in
// order, then enter the exact accumulators.
template <int IT, bool WLDS>
__global__ __launch_bounds__(256) void k_item_grad_multi(const float* __restrict__ dfcopy, dcue_batch b, int d,
                                                         float* df, const int32_t* __restrict__ copy_ptr,
                                                         const int32_t* __restrict__ copy_idx, ItemGradFc fc) {
  critical_path_priority();
  __shared__ float dfs[IT][256];
  __shared__ float part[2][IT][128];
  __shared__ float rs[1024];
  __shared__ float pw[IT == 1 ? 4 : 1][256];  // one item per workgroup: the four waves' copy sums
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [d][d] when WLDS
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i0 = blockIdx.x * IT;
  const int N = b.n_neg, B = b.n_rows, M = b.n_items;
  const bool gather = b.layout != DCUE_LAYOUT_CATALOGUE;
  const int per = (d + 63) / 64;
  DCUE_KTW(1, 6);
  DCUE_KT(1, 0);
  if constexpr (WLDS) {
    if (fc.W) {
      // four loads in flight before their LDS stores (a load-store loop waits one L2 round trip
      // per float4)
      const int n4 = d * d / 4;
      const float4* W4 = reinterpret_cast<const float4*>(fc.W);
      float4* L4 = reinterpret_cast<float4*>(wl);
      int q = threadIdx.x;
      for (; q + 768 < n4; q += 1024) {
        const float4 a = W4[q], b1 = W4[q + 256], c = W4[q + 512], e = W4[q + 768];
        L4[q] = a;
        L4[q + 256] = b1;
        L4[q + 512] = c;
        L4[q + 768] = e;
      }
      for (; q < n4; q += 256) L4[q] = W4[q];
    }
  }
  DCUE_KT(1, 1);
  if (fc.rowsum && blockIdx.x == 0)
    for (int r = threadIdx.x; r < B; r += blockDim.x) rs[r] = fc.rowsum[r];
  if constexpr (IT == 1) {
    // one item: its copies over the four waves (wave w: copies c0 + w, c0 + w + 4, ...), each
    // wave's sum in copy order, then the four sums in wave order (deterministic)
    const int i = i0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < M) {
      int c0 = 0, c1 = 1;
      long cat_idx = 0;
      if (gather) {
        c0 = copy_ptr[i];
        c1 = copy_ptr[i + 1];
      } else {
        cat_idx = i < B ? (long)i * (N + 1) : (long)((i - B) / N) * (N + 1) + 1 + (i - B) % N;
      }
      constexpr int kRows = 8;
      for (int qb = c0 + wave; qb < c1; qb += 4 * kRows) {
        long ci[kRows];
#pragma unroll
        for (int r = 0; r < kRows; ++r)
          ci[r] = qb + 4 * r < c1 ? (gather ? (long)copy_idx[qb + 4 * r] : cat_idx) : -1;
        float v[kRows][4];
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = lane + 64 * e;
            v[r][e] = (ci[r] >= 0 && e < per && k < d) ? dfcopy[ci[r] * d + k] : 0.f;
          }
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += v[r][e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      if (e < per && k < d) pw[wave][k] = acc[e];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < d; k += blockDim.x) {
      const float v = ((pw[0][k] + pw[1][k]) + pw[2][k]) + pw[3][k];
      dfs[0][k] = v;
      if (i < M) df[(long)i * d + k] = v;
    }
  }
  for (int it = wave; IT > 1 && it < IT; it += 4) {
    const int i = i0 + it;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < M) {
      int c0, c1;
      long cat_idx = 0;
      if (gather) {
        c0 = copy_ptr[i];
        c1 = copy_ptr[i + 1];
      } else {
        c0 = 0;
        c1 = 1;
        cat_idx = i < B ? (long)i * (N + 1) : (long)((i - B) / N) * (N + 1) + 1 + (i - B) % N;
      }
      constexpr int kRows = 8;
      for (int qb = c0; qb < c1; qb += kRows) {
        long ci[kRows];
#pragma unroll
        for (int r = 0; r < kRows; ++r) ci[r] = qb + r < c1 ? (gather ? (long)copy_idx[qb + r] : cat_idx) : -1;
        float v[kRows][4];
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = lane + 64 * e;
            v[r][e] = (ci[r] >= 0 && e < per && k < d) ? dfcopy[ci[r] * d + k] : 0.f;
          }
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += v[r][e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = lane + 64 * e;
        if (e < per && k < d) df[(long)i * d + k] = acc[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = lane + 64 * e;
      if (e < per && k < d) dfs[it][k] = acc[e];
    }
  }
  DCUE_KT(1, 2);
  if (fc.dfmax) {  // max |df| per column over the block's items
    __syncthreads();
    if (threadIdx.x < d) {
      float m = 0.f;
#pragma unroll
      for (int it = 0; it < IT; ++it)
        if (i0 + it < M) m = fmaxf(m, fabsf(dfs[it][threadIdx.x]));
      atomicMax(fc.dfmax + threadIdx.x, ord_key(m));
    }
  }
  if (fc.W) {
    __syncthreads();
    // g5[i][n] = sum_k df[i][k] W[k][n], k in two halves (first + second); d <= 128 here
    const int hk = (d + 1) / 2;
    for (int t = threadIdx.x; t < 2 * d; t += blockDim.x) {
      const int n = t % d, h = t / d;
      const int k0 = h * hk, k1 = h ? d : hk;
      float g[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) g[it] = 0.f;
      for (int k = k0; k < k1; ++k) {
        const float w = WLDS ? wl[k * d + n] : fc.W[(long)k * d + n];
#pragma unroll
        for (int it = 0; it < IT; ++it) g[it] += dfs[it][k] * w;
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) part[h][it][n] = g[it];
    }
    DCUE_KT(1, 3);
    __syncthreads();
    DCUE_KT(1, 4);
    if (threadIdx.x < d) {
      const int n = threadIdx.x;
      const float mu5 = fc.mean5[n], is5 = fc.invstd5[n];
      float sg = 0.f, sgx = 0.f, gm = 0.f;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int i = i0 + it;
        if (i < M) {
          const float g = part[0][it][n] + part[1][it][n];
          fc.g5[(long)i * d + n] = g;
          gm = fmaxf(gm, fabsf(g));
          sg += g;
          sgx += g * ((fc.y5[(long)i * d + n] - mu5) * is5);
        }
      }
      acc128_add(acc_at(fc.acc, d, 0, n), sg);
      acc128_add(acc_at(fc.acc, d, 1, n), sgx);
      if (fc.g5max) atomicMax(fc.g5max + n, ord_key(gm));
    }
  }
  DCUE_KT(1, 5);
  if (fc.rowsum && blockIdx.x == 0) {  // loss = mean of the row sums in row order (k_loss_mean's sums)
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int r = 0; r < B; ++r) s += rs[r];
      *fc.loss = s / (float)B;
    }
  }
  DCUE_KTW(1, 7);
}

template <int IT, bool WLDS>
static int item_grad_multi(const float* dfcopy, const dcue_batch* b, int d, float* df, const int32_t* copy_ptr,
                           const int32_t* copy_idx, const ItemGradFc& fc, size_t lds, hipStream_t s) {
  static bool attr = false;
  if (WLDS && !attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_item_grad_multi<IT, WLDS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(float) * 128 * 128)));
    attr = true;
  }
  DCUE_LAUNCH((k_item_grad_multi<IT, WLDS>), dim3((unsigned)((b->n_items + IT - 1) / IT)), dim3(256), lds, s,
              dfcopy, *b, d, df, copy_ptr, copy_idx, fc);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_item_grad(const float* dfcopy, const dcue_batch* b, int d, float* df, const float* fcW, float* g5,
                     unsigned long long* acc5, const float* y5, const float* mean5, const float* invstd5,
                     const float* rowsum, float* loss, const int32_t* copy_ptr, const int32_t* copy_idx,
                     unsigned* g5max, unsigned* dfmax, hipStream_t s) {
  if (d > 256 || (rowsum && b->n_rows > 1024)) return DCUE_ERR_UNSUPPORTED;
  const bool gather = b->layout == DCUE_LAYOUT_GATHER;
  if ((!gather || copy_ptr) && (!fcW || d <= 128)) {  // multi-item workgroups
    const ItemGradFc fc = {rowsum, loss, fcW, g5, acc5, y5, mean5, invstd5, g5max, dfmax};
    // W staged in LDS (64 KB per workgroup at d = 128), or read from L2 in the g5 loop
    // (DCUE_ITEMGRAD_WLDS=0: A/B diagnostic)
    static const bool wlds_on = [] {
      const char* e = getenv("DCUE_ITEMGRAD_WLDS");
      return !(e && e[0] == '0');
    }();
    const bool wlds = fcW && d % 4 == 0 && wlds_on;
    const size_t lds = wlds ? sizeof(float) * d * d : 0;
    // many items (catalogue M = B(1+N)): 16 per workgroup; a few (in-batch M = B): 4
    // (DCUE_ITEMGRAD_IT = 1, 2, 4 or 16 forces one: A/B diagnostic)
    static const int forced = [] {
      const char* e = getenv("DCUE_ITEMGRAD_IT");
      return e ? atoi(e) : 0;
    }();
    if (forced == 1)
      return wlds ? item_grad_multi<1, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                  : item_grad_multi<1, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
    if (forced == 2)
      return wlds ? item_grad_multi<2, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                  : item_grad_multi<2, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
    if (forced == 4)
      return wlds ? item_grad_multi<4, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                  : item_grad_multi<4, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
    if (b->n_items >= 512 || forced == 16)
      return wlds ? item_grad_multi<16, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                  : item_grad_multi<16, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
    if (b->n_items >= 256)
      return wlds ? item_grad_multi<4, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                  : item_grad_multi<4, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
    // in-batch M = B = 64: one item per workgroup (measured GPU-only, A/B: 3 us under four per workgroup)
    return wlds ? item_grad_multi<1, true>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s)
                : item_grad_multi<1, false>(dfcopy, b, d, df, copy_ptr, copy_idx, fc, lds, s);
  }
  if (b->layout == DCUE_LAYOUT_GATHER && (long)b->n_rows * b->n_neg + 1 > kItemGradCap) return DCUE_ERR_UNSUPPORTED;
  const ItemGradFc fc = {rowsum, loss, fcW, g5, acc5, y5, mean5, invstd5, g5max, dfmax};
  if (fcW && d <= kItemGradWLds && d % 4 == 0) {
    const size_t lds = sizeof(float) * d * d;
    static bool attr = false;
    if (!attr) {
      DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_item_grad<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)(sizeof(float) * kItemGradWLds * kItemGradWLds)));
      attr = true;
    }
    DCUE_LAUNCH(k_item_grad<true>, dim3(b->n_items), dim3(256), lds, s, dfcopy, *b, d, df, fc);
  } else {
    DCUE_LAUNCH(k_item_grad<false>, dim3(b->n_items), dim3(256), 0, s, dfcopy, *b, d, df, fc);
  }
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// Compact embedding gradient: one slot per distinct user (its first row), rows summed in order.
// Compact embedding gradient: row b = sum of de over the batch rows of user users[b], kept at the
// user's first occurrence (emb_rows[b] = user, -1 at repeats). Deferred Adam also learns which step
// the gradient is for (the step after the last one recorded).
__global__ void k_emb_grad(const float* __restrict__ de, const int64_t* users, int B, int E,
                           float scale, float* emb_grad, int32_t* slot, int64_t* emb_rows,
                           dcue_emb_log* log) {
  const int b = blockIdx.x;
  const int64_t u = users[b];
  if (b == 0 && threadIdx.x == 0 && log) {
    log->n_touched = B;
    log->grad_step = log->step_done + 1;
  }
  for (int r = 0; r < b; ++r)
    if (users[r] == u) {
      if (threadIdx.x == 0 && emb_rows) emb_rows[b] = -1;
      return;
    }
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    float v = 0.f;
    for (int r = b; r < B; ++r)
      if (users[r] == u) v += de[(long)r * E + k];
    emb_grad[(long)b * E + k] = v * scale;
  }
  if (threadIdx.x == 0) {
    slot[u] = b;
    if (emb_rows) emb_rows[b] = u;
  }
}

int launch_emb_grad(const float* de, const int64_t* users, int B, int E, float scale,
                    float* emb_grad, int32_t* slot, int64_t* emb_rows, dcue_emb_log* log,
                    hipStream_t s) {
  DCUE_LAUNCH(k_emb_grad, dim3(B), dim3(256), 0, s, de, users, B, E, scale, emb_grad, slot,
                     emb_rows, log);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ------------------------------------------------------------------------- layout helpers
// [M][128][T=131] (the reference's per-track tensor layout, NCL) -> [M][131][128] track rows.
// 32x32 tiles through LDS so both the read and the write are coalesced.
__global__ __launch_bounds__(256) void k_transpose_ncl(const float* __restrict__ in, int M, float* out) {
  __shared__ float tile[32][33];
  const int m = blockIdx.z;
  const int c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r, t = t0 + tx;
    tile[r][tx] = (c < kMels && t < kFrames) ? in[((long)m * kMels + c) * kFrames + t] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int t = t0 + r, c = c0 + tx;
    if (c < kMels && t < kFrames) out[((long)m * kFrames + t) * kMels + c] = tile[tx][r];
  }
}

__global__ void k_build_catalogue(const int64_t* pos, const int64_t* neg, int B, int N, int32_t* item_track) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long tot = (long)B * (1 + N);
  if (e >= tot) return;
  // a -1 from the catalogue sampler (a user with no candidate negative; the host raises the
  // reference's ValueError before such a batch is sampled) never becomes an out-of-table read
  const int64_t id = e < B ? pos[e] : neg[e - B];
  item_track[e] = (int32_t)(id < 0 ? 0 : id);
}

}  // namespace dcue

extern "C" int dcue_transpose_spectrograms(const float* ncl, int32_t M, float* out, void* stream) {
  if (!ncl || !out || M <= 0) return DCUE_ERR_INVALID;
  dim3 grid((dcue::kFrames + 31) / 32, dcue::kMels / 32, (unsigned)M);
  DCUE_LAUNCH(dcue::k_transpose_ncl, grid, dim3(256), 0, (hipStream_t)stream, ncl, M, out);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

extern "C" int dcue_build_catalogue_batch(const int64_t* pos_items, const int64_t* neg_items, int32_t B,
                                          int32_t N, int32_t* item_track, void* stream) {
  if (!pos_items || (N > 0 && !neg_items) || !item_track || B <= 0 || N < 0) return DCUE_ERR_INVALID;
  const long tot = (long)B * (1 + N);
  DCUE_LAUNCH(dcue::k_build_catalogue, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, pos_items, neg_items, B, N, item_track);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

namespace dcue {

// DCBR's MSE head (torch.nn.MSELoss, reduction 'mean', over the [M][d] item factors; van den Oord
// et al. 2013), in two launches:
//   k_mse_rows  one wave per row (4 rows per 256-thread workgroup, a grid over the rows): lane l
//               reads columns 4l..4l+3 (+256 ...) as float4 -- the row's 4*ld bytes in one coalesced
//               pass -- writes df = 2 (f - y) / (M d) and the row's sum of squares (lane partials,
//               then a fixed butterfly: deterministic) into rowsq[r]
//   k_mse_loss  one workgroup: thread t sums rowsq[t], rowsq[t + 256], ... in order, then a fixed
//               tree; loss = sum / (M d)
// ld (the storage width) is a multiple of 4 (32, 64, 128 or 256).
__global__ __launch_bounds__(256) void k_mse_rows(const float* __restrict__ f, const float* __restrict__ y, int M,
                                                  int d, int ld, float* __restrict__ df, float* __restrict__ rowsq) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  const float scale = 2.f / ((float)M * (float)d);
  float acc = 0.f;
  for (int c = lane * 4; c < ld; c += 256) {
    const long e = (long)r * ld + c;
    const float4 fv = *reinterpret_cast<const float4*>(f + e);
    const float4 yv = *reinterpret_cast<const float4*>(y + e);
    float4 dv;
    dv.x = c + 0 < d ? fv.x - yv.x : 0.f;
    dv.y = c + 1 < d ? fv.y - yv.y : 0.f;
    dv.z = c + 2 < d ? fv.z - yv.z : 0.f;
    dv.w = c + 3 < d ? fv.w - yv.w : 0.f;
    acc = fmaf(dv.x, dv.x, acc);
    acc = fmaf(dv.y, dv.y, acc);
    acc = fmaf(dv.z, dv.z, acc);
    acc = fmaf(dv.w, dv.w, acc);
    *reinterpret_cast<float4*>(df + e) = make_float4(dv.x * scale, dv.y * scale, dv.z * scale, dv.w * scale);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) rowsq[r] = acc;
}

__global__ __launch_bounds__(256) void k_mse_loss(const float* __restrict__ rowsq, int M, int d, float* loss) {
  __shared__ float part[256];
  float acc = 0.f;
  for (int r = threadIdx.x; r < M; r += blockDim.x) acc += rowsq[r];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = part[0] / ((float)M * (float)d);
}

int launch_mse_grad(const float* f, const float* y, int M, int d, int ld, float* df, float* rowsq, float* loss,
                    hipStream_t s) {
  if (M <= 0 || d <= 0 || d > ld || (ld & 3)) return DCUE_ERR_INVALID;
  DCUE_LAUNCH(k_mse_rows, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, f, y, M, d, ld, df, rowsq);
  DCUE_LAUNCH_CHECK();
  DCUE_LAUNCH(k_mse_loss, dim3(1), dim3(256), 0, s, rowsq, M, d, loss);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
