// BatchNorm statistics, small dense layers, cosine scoring + hinge loss, Adam -- gfx950.
//
// Reference ops replaced:
//   BatchNorm1d train/eval statistics + running-stat update     truedcuemel1dbn.py:24-61 (torch BN)
//   UserEmbeddings (gather, relu, linear, relu, linear)          userembedding.py:33-44
//   fc Linear(d,d)                                              truedcuemel1dbn.py:65,101
//   nn.CosineSimilarity(dim=1) scoring, pos - neg               dcue/dcue.py:68,94-106
//   hinge loss mean_b sum_n max(0, margin - s)                  nn/dcue.py:167-170
//   torch.optim.Adam.step (single-tensor semantics)             nn/dcue.py:143-147, 209
#include "dcue_internal.h"

namespace dcue {

// --------------------------------------------------------------------------- BN statistics
// bn0 input statistics over the gathered spectrograms, weighted by item copy counts.
template <int SRC>
__global__ __launch_bounds__(256) void k_input_stats(const void* tracks, const int32_t* item_track,
                                                     const float* counts, int M, int rows_per_blk,
                                                     float* partials) {
  __shared__ float red[8][2][kMels];
  const int q = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const long rows = (long)M * kFrames;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(r0 + rows_per_blk, rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), ss = s;
  for (long r = r0 + slot; r < r1; r += 8) {
    const long i = r / kFrames;
    const int p = (int)(r - i * kFrames);
    const long off = ((long)item_track[i] * kFrames + p) * kMels + 4 * q;
    float x[4];
    if constexpr (SRC == SRC_TRACK_F16) {
      const uint2 raw = *reinterpret_cast<const uint2*>(reinterpret_cast<const __half*>(tracks) + off);
      const __half2 h0 = *reinterpret_cast<const __half2*>(&raw.x);
      const __half2 h1 = *reinterpret_cast<const __half2*>(&raw.y);
      x[0] = __low2float(h0); x[1] = __high2float(h0); x[2] = __low2float(h1); x[3] = __high2float(h1);
    } else {
      const float4 v = ld4(reinterpret_cast<const float*>(tracks) + off);
      x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
    }
    const float w = counts ? counts[i] : 1.f;
    s.x += w * x[0]; s.y += w * x[1]; s.z += w * x[2]; s.w += w * x[3];
    ss.x += w * x[0] * x[0]; ss.y += w * x[1] * x[1]; ss.z += w * x[2] * x[2]; ss.w += w * x[3] * x[3];
  }
  st4(&red[slot][0][4 * q], s);
  st4(&red[slot][1][4 * q], ss);
  __syncthreads();
  {
    const int c = threadIdx.x & 127, which = threadIdx.x >> 7;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += red[k][which][c];
    partials[((long)blockIdx.x * 2 + which) * kMels + c] = v;
  }
}

int launch_input_stats(int src, const void* tracks, const int32_t* item_track, const float* counts,
                       int M, float* partials, int* nparts, hipStream_t s) {
  const long rows = (long)M * kFrames;
  int nb = (int)((rows + 255) / 256);
  if (nb > 1024) nb = 1024;
  const int rpb = (int)((rows + nb - 1) / nb);
  nb = (int)((rows + rpb - 1) / rpb);
  *nparts = nb;
  if (src == SRC_TRACK_F16)
    hipLaunchKernelGGL(k_input_stats<SRC_TRACK_F16>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, partials);
  else
    hipLaunchKernelGGL(k_input_stats<SRC_TRACK_F32>, dim3(nb), dim3(256), 0, s, tracks, item_track,
                       counts, M, rpb, partials);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// partials [nparts][2][C] -> mean, invstd, a = gamma*invstd; train mode also updates running stats
// (momentum 0.1, unbiased running variance) and num_batches_tracked, as torch BatchNorm1d does.
// Eval mode (train == 0) takes mean/var from the running stats. Sums are combined in fp64.
__global__ __launch_bounds__(256) void k_bn_finalize(const float* __restrict__ partials, int nparts,
                                                     int C, double count, const float* gamma,
                                                     float* rmean, float* rvar, int64_t* nbt,
                                                     int train, float* mean, float* invstd,
                                                     float* a) {
  __shared__ double red[4][2][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0, ss = 0.0;
  if (train && c < C)
    for (int p = sl; p < nparts; p += 4) {
      s += (double)partials[((long)p * 2 + 0) * C + c];
      ss += (double)partials[((long)p * 2 + 1) * C + c];
    }
  red[sl][0][cl] = s;
  red[sl][1][cl] = ss;
  __syncthreads();
  if (sl == 0 && c < C) {
    const float eps = 1e-5f, momentum = 0.1f;
    float mu, var;
    if (train) {
      s = red[0][0][cl] + red[1][0][cl] + red[2][0][cl] + red[3][0][cl];
      ss = red[0][1][cl] + red[1][1][cl] + red[2][1][cl] + red[3][1][cl];
      const double m = s / count;
      double v = ss / count - m * m;
      if (v < 0.0) v = 0.0;
      mu = (float)m;
      var = (float)v;
      const double unbiased = count > 1.0 ? v * count / (count - 1.0) : v;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
      if (c == 0) nbt[0] += 1;
    } else {
      mu = rmean[c];
      var = rvar[c];
    }
    const float is = 1.f / sqrtf(var + eps);
    mean[c] = mu;
    invstd[c] = is;
    a[c] = gamma[c] * is;
  }
}

int launch_bn_finalize(const float* partials, int nparts, int C, double count, const float* gamma,
                       float* rmean, float* rvar, int64_t* nbt, int train, float* mean,
                       float* invstd, float* a, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 63) / 64), dim3(256), 0, s, partials, nparts, C, count,
                     gamma, rmean, rvar, nbt, train, mean, invstd, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// backward partial sums over rows of g and g*xhat (xhat from the stored pre-BN activation).
__global__ __launch_bounds__(256) void k_bwd_partials(const float* __restrict__ g,
                                                      const float* __restrict__ y,
                                                      const float* mean, const float* invstd,
                                                      long rows, int C, int rows_per_blk,
                                                      float* partials) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [slots][2][C]
  const int quads = C / 4;
  const int nslots = 256 / quads;
  const int q = threadIdx.x % quads, slot = threadIdx.x / quads;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(r0 + rows_per_blk, rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), sx = s;
  if (slot < nslots) {
    const float4 mu = ld4(mean + 4 * q), is = ld4(invstd + 4 * q);
    for (long r = r0 + slot; r < r1; r += nslots) {
      const float4 gv = ld4(g + r * C + 4 * q), yv = ld4(y + r * C + 4 * q);
      s.x += gv.x; s.y += gv.y; s.z += gv.z; s.w += gv.w;
      sx.x += gv.x * ((yv.x - mu.x) * is.x);
      sx.y += gv.y * ((yv.y - mu.y) * is.y);
      sx.z += gv.z * ((yv.z - mu.z) * is.z);
      sx.w += gv.w * ((yv.w - mu.w) * is.w);
    }
    st4(&red[(slot * 2 + 0) * C + 4 * q], s);
    st4(&red[(slot * 2 + 1) * C + 4 * q], sx);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C; e += 256) {
    const int which = e / C, c = e - which * C;
    float v = 0.f;
    for (int k = 0; k < nslots; ++k) v += red[(k * 2 + which) * C + c];
    partials[((long)blockIdx.x * 2 + which) * C + c] = v;
  }
}

int launch_bwd_partials(const float* g, const float* y, const float* mean, const float* invstd,
                        long rows, int C, float* partials, int* nparts, hipStream_t s) {
  int nb = (int)((rows + 63) / 64);
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  const int rpb = (int)((rows + nb - 1) / nb);
  nb = (int)((rows + rpb - 1) / rpb);
  if (nb < 1) nb = 1;
  *nparts = nb;
  const int nslots = 256 / (C / 4);
  const size_t lds = (size_t)nslots * 2 * C * sizeof(float);
  hipLaunchKernelGGL(k_bwd_partials, dim3(nb), dim3(256), lds, s, g, y, mean, invstd, rows, C, rpb,
                     partials);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

__global__ __launch_bounds__(256) void k_bwd_finalize(const float* __restrict__ partials, int nparts,
                                                      int C, float* sD, float* sDx, float* dgamma,
                                                      float* dbeta) {
  __shared__ double red[4][2][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0, sx = 0.0;
  if (c < C)
    for (int p = sl; p < nparts; p += 4) {
      s += (double)partials[((long)p * 2 + 0) * C + c];
      sx += (double)partials[((long)p * 2 + 1) * C + c];
    }
  red[sl][0][cl] = s;
  red[sl][1][cl] = sx;
  __syncthreads();
  if (sl == 0 && c < C) {
    s = red[0][0][cl] + red[1][0][cl] + red[2][0][cl] + red[3][0][cl];
    sx = red[0][1][cl] + red[1][1][cl] + red[2][1][cl] + red[3][1][cl];
    sD[c] = (float)s;
    sDx[c] = (float)sx;
    dbeta[c] = (float)s;   // BN output = gamma*xhat + beta
    dgamma[c] = (float)sx;
  }
}

int launch_bwd_finalize(const float* partials, int nparts, int C, float* sD, float* sDx,
                        float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(k_bwd_finalize, dim3((C + 63) / 64), dim3(256), 0, s, partials, nparts, C, sD,
                     sDx, dgamma, dbeta);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// column sums of A[M][N] (bias gradients); one thread per column, rows in order
__global__ void k_colsum(const float* __restrict__ A, int M, int N, float* out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float v = 0.f;
  for (int m = 0; m < M; ++m) v += A[(long)m * N + n];
  out[n] = v;
}

int launch_colsum(const float* A, int M, int N, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_colsum, dim3((N + 127) / 128), dim3(128), 0, s, A, M, N, out);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ---------------------------------------------------------------------------- small GEMM
// C(m,n) = sum_k T(A(m,k)) B(k,n) + bias[n], 64x64 tiles, 4x4 per thread, K chunks of 16 in LDS.
// For the user tower (B x 300 x 300), fc (M x d x d) and their backward products: tiny shapes
// where launch latency, not the MFMA rate, is the cost.
template <int TA>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < g.K; k0 += 16) {
    for (int e = threadIdx.x; e < 16 * 64; e += 256) {
      const int kk = e / 64, mm = e - kk * 64;
      const int m = m0 + mm, k = k0 + kk;
      float v = 0.f;
      if (m < g.M && k < g.K) {
        const long row = g.arow ? g.arow[m] : m;
        v = g.A[row * g.sam + (long)k * g.sak];
        if constexpr (TA == 1) v = v > 0.f ? v : 0.f;
        if constexpr (TA == 2) v = (v - g.tmean[k]) * g.ta[k] + g.tbeta[k];
        if constexpr (TA == 3) v = (v - g.tmean[m]) * g.ta[m] + g.tbeta[m];
      }
      As[kk][mm] = v;
      const int n = n0 + mm;
      Bs[kk][mm] = (n < g.N && k < g.K) ? g.B[(long)k * g.sbk + (long)n * g.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + ty * 4 + i, n = n0 + tx * 4 + j;
      if (m < g.M && n < g.N) {
        float v = acc[i][j] + (g.bias ? g.bias[n] : 0.f);
        const long off = (long)m * g.scm + (long)n * g.scn;
        if (g.cmask && !(g.cmask[off] > 0.f)) v = 0.f;
        g.C[off] = v;
      }
    }
}

int launch_gemm(int ta, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return DCUE_OK;
  dim3 grid((g.N + 63) / 64, (g.M + 63) / 64);
  switch (ta) {
    case 0: hipLaunchKernelGGL(k_gemm<0>, grid, dim3(256), 0, s, g); break;
    case 1: hipLaunchKernelGGL(k_gemm<1>, grid, dim3(256), 0, s, g); break;
    case 2: hipLaunchKernelGGL(k_gemm<2>, grid, dim3(256), 0, s, g); break;
    case 3: hipLaunchKernelGGL(k_gemm<3>, grid, dim3(256), 0, s, g); break;
    default: return DCUE_ERR_INVALID;
  }
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

__global__ void k_gather_rows(const float* __restrict__ table, const int64_t* rows, int n, int E,
                              float* out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)n * E) return;
  const long r = idx / E, k = idx - r * E;
  out[idx] = table[rows[r] * E + k];
}

int launch_gather_rows(const float* table, const int64_t* rows, int n, int E, float* out,
                       hipStream_t s) {
  const long tot = (long)n * E;
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, table, rows,
                     n, E, out);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ------------------------------------------------------------------- copies, scores, loss
__device__ __forceinline__ int copy_item(const dcue_batch& b, int row, int c) {
  if (c == 0) return row;
  if (b.layout == DCUE_LAYOUT_CATALOGUE) return b.n_rows + row * b.n_neg + (c - 1);
  return b.neg_item[(long)row * b.n_neg + (c - 1)];
}

// copies of each item (BatchNorm weights): catalogue = 1 each; gather = positives + negative refs
__global__ void k_item_counts(dcue_batch b, float* counts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.n_items) return;
  float c = i < b.n_rows ? 1.f : 0.f;
  if (b.layout == DCUE_LAYOUT_CATALOGUE) {
    c = 1.f;
  } else {
    const long nneg = (long)b.n_rows * b.n_neg;
    for (long e = 0; e < nneg; ++e) c += (b.neg_item[e] == i) ? 1.f : 0.f;
  }
  counts[i] = c;
}

int launch_item_counts(const dcue_batch* b, float* counts, hipStream_t s) {
  hipLaunchKernelGGL(k_item_counts, dim3((b->n_items + 127) / 128), dim3(128), 0, s, *b, counts);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// One wave per row b: torch cosine_similarity = sum((x/max(|x|,eps)) * (y/max(|y|,eps))).
// cosv[b][0] = cos(u, pos), cosv[b][1+j] = cos(u, neg_j); norms[b][0] = |u|, norms[b][1+c] = |f_c|.
__global__ __launch_bounds__(64) void k_score_fwd(const float* __restrict__ uf,
                                                  const float* __restrict__ f, dcue_batch b, int d,
                                                  float margin, float* scores, float* cosv,
                                                  float* norms, float* row_loss, float* dhinge) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const int N = b.n_neg, per = (d + 63) / 64;
  const float eps = 1e-8f;
  float u[4];
  float su = 0.f;
  for (int e = 0; e < per; ++e) {
    const int k = lane + 64 * e;
    u[e] = k < d ? uf[(long)row * d + k] : 0.f;
    su += u[e] * u[e];
  }
  const float nu = sqrtf(wave_sum(su));
  const float du = fmaxf(nu, eps);
  if (lane == 0) norms[(long)row * (N + 2)] = nu;
  float pcos = 0.f, loss = 0.f;
  for (int c = 0; c <= N; ++c) {
    const long item = copy_item(b, row, c);
    float v[4], sf = 0.f;
    for (int e = 0; e < per; ++e) {
      const int k = lane + 64 * e;
      v[e] = k < d ? f[item * d + k] : 0.f;
      sf += v[e] * v[e];
    }
    const float nf = sqrtf(wave_sum(sf));
    const float df = fmaxf(nf, eps);
    float dot = 0.f;
    for (int e = 0; e < per; ++e) dot += (u[e] / du) * (v[e] / df);
    const float cs = wave_sum(dot);
    if (lane == 0) {
      norms[(long)row * (N + 2) + 1 + c] = nf;
      cosv[(long)row * (N + 1) + c] = cs;
    }
    if (c == 0) {
      pcos = cs;
    } else {
      const float sc = pcos - cs;
      if (lane == 0) scores[(long)row * N + (c - 1)] = sc;
      const float h = margin - sc;
      loss += h > 0.f ? h : 0.f;
      // d/ds of mean_b sum_n max(0, margin - s): torch.max splits the gradient evenly on a tie
      if (lane == 0)
        dhinge[(long)row * N + (c - 1)] = h > 0.f ? -1.f / (float)b.n_rows : (h == 0.f ? -0.5f / (float)b.n_rows : 0.f);
    }
  }
  if (lane == 0) row_loss[row] = loss;
}

__global__ void k_loss_mean(const float* row_loss, int B, float* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += row_loss[b];
    *loss = s / (float)B;
  }
}

int launch_score_fwd(const float* uf, const float* f, const dcue_batch* b, int d, float margin,
                     float* scores, float* cosv, float* norms, float* row_loss, float* loss,
                     float* dhinge, hipStream_t s) {
  if (d > 256) return DCUE_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_score_fwd, dim3(b->n_rows), dim3(64), 0, s, uf, f, *b, d, margin, scores, cosv,
                     norms, row_loss, dhinge);
  DCUE_LAUNCH_CHECK();
  if (loss) {
    hipLaunchKernelGGL(k_loss_mean, dim3(1), dim3(64), 0, s, row_loss, b->n_rows, loss);
    DCUE_LAUNCH_CHECK();
  }
  return DCUE_OK;
}

// dL/dscores [B][N] (the hinge's, written by k_score_fwd, or the caller's) -> dL/du, dL/df per copy.
// d cos/dx = (yhat - cos*xhat)/|x| (non-degenerate norms).
__global__ __launch_bounds__(64) void k_score_bwd(const float* __restrict__ uf,
                                                  const float* __restrict__ f, dcue_batch b, int d,
                                                  const float* dscores, const float* cosv,
                                                  const float* norms, float* dU, float* dfcopy) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const int N = b.n_neg, per = (d + 63) / 64;
  const float eps = 1e-8f;
  const float nu = fmaxf(norms[(long)row * (N + 2)], eps);
  float u[4], gu[4];
  for (int e = 0; e < per; ++e) {
    const int k = lane + 64 * e;
    u[e] = k < d ? uf[(long)row * d + k] / nu : 0.f;
    gu[e] = 0.f;
  }
  float dpos = 0.f;  // scores = pos_cos - neg_cos: the positive collects every score's gradient
  for (int j = 0; j < N; ++j) dpos += dscores[(long)row * N + j];
  for (int c = 0; c <= N; ++c) {
    const long item = copy_item(b, row, c);
    const float dc = c == 0 ? dpos : -dscores[(long)row * N + c - 1];
    const float cs = cosv[(long)row * (N + 1) + c];
    const float nf = fmaxf(norms[(long)row * (N + 2) + 1 + c], eps);
    for (int e = 0; e < per; ++e) {
      const int k = lane + 64 * e;
      if (k < d) {
        const float fh = f[item * d + k] / nf;
        gu[e] += dc * (fh - cs * u[e]) / nu;
        dfcopy[((long)row * (N + 1) + c) * d + k] = dc * (u[e] - cs * fh) / nf;
      }
    }
  }
  for (int e = 0; e < per; ++e) {
    const int k = lane + 64 * e;
    if (k < d) dU[(long)row * d + k] = gu[e];
  }
}

int launch_score_bwd(const float* uf, const float* f, const dcue_batch* b, int d,
                     const float* dscores, const float* cosv, const float* norms, float* du,
                     float* dfcopy, hipStream_t s) {
  hipLaunchKernelGGL(k_score_bwd, dim3(b->n_rows), dim3(64), 0, s, uf, f, *b, d, dscores, cosv,
                     norms, du, dfcopy);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// df[i] = sum of the gradients of item i's copies (fixed order: positive, then (b, j) row-major).
__global__ void k_item_grad(const float* __restrict__ dfcopy, dcue_batch b, int d, float* df) {
  const int i = blockIdx.x;
  const int N = b.n_neg, B = b.n_rows;
  for (int k = threadIdx.x; k < d; k += blockDim.x) {
    float v;
    if (b.layout == DCUE_LAYOUT_CATALOGUE) {
      if (i < B) v = dfcopy[((long)i * (N + 1)) * d + k];
      else {
        const int r = (i - B) / N, j = (i - B) - r * N;
        v = dfcopy[((long)r * (N + 1) + 1 + j) * d + k];
      }
    } else {
      v = i < B ? dfcopy[((long)i * (N + 1)) * d + k] : 0.f;
      for (int r = 0; r < B; ++r)
        for (int j = 0; j < N; ++j)
          if (b.neg_item[(long)r * N + j] == i) v += dfcopy[((long)r * (N + 1) + 1 + j) * d + k];
    }
    df[(long)i * d + k] = v;
  }
}

int launch_item_grad(const float* dfcopy, const dcue_batch* b, int d, float* df, hipStream_t s) {
  hipLaunchKernelGGL(k_item_grad, dim3(b->n_items), dim3(128), 0, s, dfcopy, *b, d, df);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// Compact embedding gradient: one slot per distinct user (its first row), rows summed in order.
__global__ void k_emb_grad(const float* __restrict__ de, const int64_t* users, int B, int E,
                           float scale, float* emb_grad, int32_t* slot) {
  const int b = blockIdx.x;
  const int64_t u = users[b];
  for (int r = 0; r < b; ++r)
    if (users[r] == u) return;
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    float v = 0.f;
    for (int r = b; r < B; ++r)
      if (users[r] == u) v += de[(long)r * E + k];
    emb_grad[(long)b * E + k] = v * scale;
  }
  if (threadIdx.x == 0) slot[u] = b;
}

int launch_emb_grad(const float* de, const int64_t* users, int B, int E, float scale,
                    float* emb_grad, int32_t* slot, hipStream_t s) {
  hipLaunchKernelGGL(k_emb_grad, dim3(B), dim3(128), 0, s, de, users, B, E, scale, emb_grad, slot);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ------------------------------------------------------------------------------------ Adam
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
// forward B operand of layer l: [k][cin/4][cout][4]; dgrad (l >= 2): [k'][cout/4][cin][4], k' = ks-1-k
struct PackSeg {
  long src, fwd, bwd;  // offsets (floats): W in params, forward pack, dgrad pack (-1: none)
  int cout, cin, ks;
};
struct PackArgs {
  PackSeg seg[5];
};

__global__ void k_pack(const float* __restrict__ params, float* wpack, PackArgs pa) {
  const int l = blockIdx.y;
  const PackSeg sg = pa.seg[l];
  const long n = (long)sg.cout * sg.cin * sg.ks;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long o = e / ((long)sg.cin * sg.ks);
    const long rem = e - o * sg.cin * sg.ks;
    const long c = rem / sg.ks, k = rem - c * sg.ks;
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
  PackArgs pa;
  long off = 0;
  for (int l = 1; l <= 5; ++l) {
    const LayerGeom gm = layer_geom(l);
    PackSeg& sg = pa.seg[l - 1];
    sg.cin = l == 1 ? kMels : H;
    sg.cout = l == 5 ? d : H;
    sg.ks = gm.ks;
    sg.src = poff[2 + 4 * (l - 1)];  // conv.layer{l}.weight
    const long n = (long)sg.cout * sg.cin * sg.ks;
    sg.fwd = off;
    off += n;
    if (l >= 2) { sg.bwd = off; off += n; } else sg.bwd = -1;
  }
  hipLaunchKernelGGL(k_pack, dim3(64, 5), dim3(256), 0, s, md->params, md->wpack, pa);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue

// ------------------------------------------------------------------------- layout helpers
namespace dcue {

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
  item_track[e] = (int32_t)(e < B ? pos[e] : neg[e - B]);
}

}  // namespace dcue

extern "C" int dcue_transpose_spectrograms(const float* ncl, int32_t M, float* out, void* stream) {
  if (!ncl || !out || M <= 0) return DCUE_ERR_INVALID;
  dim3 grid((dcue::kFrames + 31) / 32, dcue::kMels / 32, (unsigned)M);
  hipLaunchKernelGGL(dcue::k_transpose_ncl, grid, dim3(256), 0, (hipStream_t)stream, ncl, M, out);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

extern "C" int dcue_build_catalogue_batch(const int64_t* pos_items, const int64_t* neg_items, int32_t B,
                                          int32_t N, int32_t* item_track, void* stream) {
  if (!pos_items || (N > 0 && !neg_items) || !item_track || B <= 0 || N < 0) return DCUE_ERR_INVALID;
  const long tot = (long)B * (1 + N);
  hipLaunchKernelGGL(dcue::k_build_catalogue, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, pos_items, neg_items, B, N, item_track);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}
