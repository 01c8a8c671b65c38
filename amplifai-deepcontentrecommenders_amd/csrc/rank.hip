// Ranking metrics of DCUE's evaluation (nn/dcue.py:380-476): per query (a user for DCUE.score, a
// song for DCUE.score_song), cosine scores against every candidate, then tie-aware AUC and average
// precision, computed exactly from integer rank counts instead of a sort of every score row.
//
// Per batch of queries:
//   k_rank_normalize  x / max(||x||, 1e-8) per row (nn.CosineSimilarity), zero-padded to DP = d up
//                     to a multiple of 16, for the batch's queries (candidates once per call)
//   k_rank_scores     S[q][c] = qn . cn on v_mfma_f32_16x16x4_f32: 64 queries x 64 candidates per
//                     workgroup, both operands staged through LDS
//   k_rank_thresholds the query's positives (CSR row, restricted to candidates in a list) gathered
//                     from S, bitonic-sorted in LDS -> ascending thresholds t_0..t_{n-1} + class bits;
//                     zeroes the query's histograms
//   k_rank_hist       every candidate score s, per list it belongs to: bucket ub(s) = #{t_j <= s} of
//                     a "less-than" histogram and, when s equals a threshold run, its run start of an
//                     "equal" histogram (LDS atomics, flushed with global atomics)
//   k_rank_finalize   prefix sums turn the histograms into, per positive p and list c, the number of
//                     list items scoring below / equal to p; minus the positives' own counts these
//                     are the Mann-Whitney counts of negatives (ties 1/2) and the "scores >= p"
//                     counts of average precision; fp64 AUC / AP per query
// Scores of the positives are read back from the same S the histograms stream, so a positive meets
// its own threshold as an exact tie (no recomputation can differ by an ulp).
#include "dcue_internal.h"

namespace dcue {

constexpr int kRankCap = 4096;    // positives (within the lists) per query
constexpr int kRankTile = 64;     // queries x candidates per scoring workgroup
constexpr int kRankChunk = 8192;  // candidates per histogram workgroup

__host__ __device__ constexpr int rank_dp(int d) { return (d + 15) & ~15; }

// one wave per row: y = x / max(||x||_2, eps), zero padding to DP (rows[] may gather)
__global__ __launch_bounds__(256) void k_rank_normalize(const float* __restrict__ x, const int32_t* rows,
                                                        int64_t n, int d, int dp, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int64_t src = rows ? (int64_t)rows[r] : r;
  const float* xr = x + src * d;
  float ss = 0.f;
  for (int k = lane; k < d; k += 64) ss = fmaf(xr[k], xr[k], ss);
  ss = wave_sum(ss);
  const float nrm = fmaxf(sqrtf(ss), 1e-8f);
  float* yr = y + r * dp;
  for (int k = lane; k < dp; k += 64) yr[k] = k < d ? xr[k] / nrm : 0.f;
}

// S[q][c] for q < nq, c < nc. Wave w owns candidate columns 16w..16w+15 of the tile and all four
// 16-query row tiles; k is split across the four lane groups (g = lane>>4 covers k = g*DP/4 + j), so
// every lane reads DP/4 consecutive floats of its row.
__global__ __launch_bounds__(256) void k_rank_scores(const float* __restrict__ qn, int nq,
                                                     const float* __restrict__ cn, int64_t nc, int dp,
                                                     float* __restrict__ S, int64_t ldS) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int st = dp + 4;  // row stride: lanes of one k step on different banks
  float* As = lds;
  float* Bs = lds + kRankTile * st;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int q0 = blockIdx.y * kRankTile;
  const int64_t c0 = (int64_t)blockIdx.x * kRankTile;
  const int dp4 = dp >> 2;
  for (int e = tid; e < kRankTile * dp4; e += 256) {
    const int r = e / dp4, k4 = e - r * dp4;
    const int q = q0 + r;
    const int64_t c = c0 + r;
    st4(&As[r * st + 4 * k4], q < nq ? ld4(qn + (int64_t)q * dp + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f));
    st4(&Bs[r * st + 4 * k4], c < nc ? ld4(cn + c * dp + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kq = dp >> 2;  // k range per lane group
  const float* brow = &Bs[(16 * w + l16) * st + g * kq];
  for (int j = 0; j < kq; j += 4) {
    const float4 b = ld4(brow + j);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 a = ld4(&As[(16 * m + l16) * st + g * kq + j]);
      acc[m] = mfma4(a.x, b.x, acc[m]);
      acc[m] = mfma4(a.y, b.y, acc[m]);
      acc[m] = mfma4(a.z, b.z, acc[m]);
      acc[m] = mfma4(a.w, b.w, acc[m]);
    }
  }
  const int64_t c = c0 + 16 * w + l16;
  if (c < nc) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + 16 * m + 4 * g + r;
        if (q < nq) S[(int64_t)q * ldS + c] = acc[m][r];
      }
  }
}

__device__ __forceinline__ uint32_t float_order(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float order_float(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

struct RankWs {
  float* thr;        // [QB][cap] ascending thresholds
  uint8_t* thr_cls;  // [QB][cap] list bits of each threshold's positive
  int32_t* n_thr;    // [QB]
  int32_t* hist;     // [QB][4][cap+1]: lt list0, lt list1, eq list0, eq list1
  int32_t* status;   // [1] first query index over the cap, else -1
  int32_t* nonfin;   // [QB] a score the reference's sklearn call would see is NaN / inf
};

// one workgroup per query of the batch
__global__ __launch_bounds__(256) void k_rank_thresholds(const float* __restrict__ S, int64_t ldS,
                                                         const int32_t* __restrict__ queries,
                                                         const int64_t* __restrict__ pos_ptr,
                                                         const int32_t* __restrict__ pos_idx,
                                                         const uint8_t* __restrict__ cls, int64_t nc,
                                                         int pos_mask, RankWs w) {
  __shared__ uint64_t key[kRankCap];
  __shared__ int cnt, bad;
  const int i = blockIdx.x, tid = threadIdx.x;
  const int q = queries[i];
  const int64_t b = pos_ptr[q], e = pos_ptr[q + 1];
  if (tid == 0) cnt = bad = 0;
  __syncthreads();
  for (int64_t p = b + tid; p < e; p += 256) {
    const int c = pos_idx[p];
    const uint8_t k = (c >= 0 && c < nc) ? cls[c] : 0;
    if (k & pos_mask) {
      const float sc = S[(int64_t)i * ldS + c];
      if (!isfinite(sc)) bad = 1;
      const int slot = atomicAdd(&cnt, 1);
      if (slot < kRankCap) key[slot] = ((uint64_t)float_order(sc) << 8) | k;
    }
  }
  __syncthreads();
  if (tid == 0) w.nonfin[i] = bad;  // (k_rank_hist adds the list items' scores)
  const int n = cnt;
  int32_t* h = w.hist + (int64_t)i * 4 * (kRankCap + 1);
  for (int k = tid; k < 4 * (n + 1) && n <= kRankCap; k += 256) h[(k / (n + 1)) * (kRankCap + 1) + k % (n + 1)] = 0;
  if (n > kRankCap) {
    if (tid == 0) {
      atomicCAS(w.status, -1, i);
      w.n_thr[i] = 0;
    }
    return;
  }
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int k = n + tid; k < np2; k += 256) key[k] = ~0ull;
  __syncthreads();
  // bitonic sort, ascending
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < np2 / 2; t += 256) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = key[lo], c = key[hi];
        if ((a > c) == up) {
          key[lo] = c;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int k = tid; k < n; k += 256) {
    w.thr[(int64_t)i * kRankCap + k] = order_float((uint32_t)(key[k] >> 8));
    w.thr_cls[(int64_t)i * kRankCap + k] = (uint8_t)(key[k] & 0xff);
  }
  if (tid == 0) w.n_thr[i] = n;
}

__device__ __forceinline__ int upper_bound_f(const float* t, int n, float s) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (t[mid] <= s) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int lower_bound_f(const float* t, int n, float s) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (t[mid] < s) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// grid (candidate chunks, queries of the batch)
// score_mask: the list bits whose items' scores the reference hands to sklearn (which raises on a
// non-finite one): both lists for DCUE.score, the label-0 list (plus the positives, checked in
// k_rank_thresholds) for score_song
__global__ __launch_bounds__(256) void k_rank_hist(const float* __restrict__ S, int64_t ldS,
                                                   const uint8_t* __restrict__ cls, int64_t nc, int score_mask,
                                                   RankWs w) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int i = blockIdx.y, tid = threadIdx.x;
  const int n = w.n_thr[i];
  float* t = lds;
  int* hl = reinterpret_cast<int*>(lds + kRankCap);  // [4][n+1]
  const int nb = n + 1;
  for (int k = tid; k < n; k += 256) t[k] = w.thr[(int64_t)i * kRankCap + k];
  for (int k = tid; k < 4 * nb; k += 256) hl[k] = 0;
  __syncthreads();
  const int64_t c_begin = (int64_t)blockIdx.x * kRankChunk;
  const int64_t c_end = min(c_begin + kRankChunk, nc);
  const float* Sr = S + (int64_t)i * ldS;
  bool bad = false;
  for (int64_t c = c_begin + tid; c < c_end; c += 256) {
    const uint8_t k = cls[c];
    if (!k) continue;
    const float s = Sr[c];
    bad |= (k & score_mask) && !isfinite(s);
    const int ub = upper_bound_f(t, n, s);
    const int lb = (ub > 0 && t[ub - 1] == s) ? lower_bound_f(t, ub, s) : ub;
    if (k & 1) {
      atomicAdd(&hl[ub], 1);
      if (lb < ub) atomicAdd(&hl[2 * nb + lb], 1);
    }
    if (k & 2) {
      atomicAdd(&hl[nb + ub], 1);
      if (lb < ub) atomicAdd(&hl[3 * nb + lb], 1);
    }
  }
  if (__any(bad) && (tid & 63) == 0) atomicOr(&w.nonfin[i], 1);
  __syncthreads();
  int32_t* h = w.hist + (int64_t)i * 4 * (kRankCap + 1);
  for (int k = tid; k < 4 * nb; k += 256) {
    const int v = hl[k];
    if (v) atomicAdd(&h[(k / nb) * (kRankCap + 1) + k % nb], v);
  }
}

// block-wide inclusive scan of int over n+1 entries in LDS (n <= kRankCap), in place
__device__ void block_scan_inplace(int* a, int len, int* tmp) {
  const int tid = threadIdx.x;
  const int per = (len + 255) / 256;
  const int b = tid * per, e = min(b + per, len);
  int s = 0;
  for (int k = b; k < e; ++k) s += a[k];
  tmp[tid] = s;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int k = 0; k < 256; ++k) {
      const int v = tmp[k];
      tmp[k] = run;
      run += v;
    }
  }
  __syncthreads();
  int run = tmp[tid];
  for (int k = b; k < e; ++k) {
    run += a[k];
    a[k] = run;
  }
  __syncthreads();
}

// one workgroup per query of the batch
__global__ __launch_bounds__(256) void k_rank_finalize(RankWs w, int mode, int q_offset, double* auc,
                                                       double* ap, int32_t* flag) {
  __shared__ int lt0[kRankCap + 1], lt1[kRankCap + 1], c0[kRankCap + 1], c1[kRankCap + 1];
  __shared__ float t[kRankCap];
  __shared__ int tmp[256];
  __shared__ double red[3][256];
  const int i = blockIdx.x, tid = threadIdx.x;
  const int n = w.n_thr[i], nb = n + 1;
  const int32_t* h = w.hist + (int64_t)i * 4 * (kRankCap + 1);
  const float* thr = w.thr + (int64_t)i * kRankCap;
  const uint8_t* tc = w.thr_cls + (int64_t)i * kRankCap;
  for (int k = tid; k < nb; k += 256) {
    lt0[k] = h[k];
    lt1[k] = h[(kRankCap + 1) + k];
    // exclusive class counts among the sorted thresholds: c[k] = #{j < k with the bit}
    c0[k] = k > 0 ? (tc[k - 1] & 1) : 0;
    c1[k] = k > 0 ? ((tc[k - 1] >> 1) & 1) : 0;
    if (k < n) t[k] = thr[k];
  }
  __syncthreads();
  block_scan_inplace(lt0, nb, tmp);
  block_scan_inplace(lt1, nb, tmp);
  block_scan_inplace(c0, nb, tmp);
  block_scan_inplace(c1, nb, tmp);
  const long n0 = lt0[n], n1 = lt1[n];  // candidates per list
  const long p0 = c0[n], p1 = c1[n];    // positives per list
  const long mtot = mode == 0 ? p0 + p1 : n;
  double u_pos = 0.0, u_neg = 0.0, ap_sum = 0.0;
  for (int j = tid; j < n; j += 256) {
    const float s = t[j];
    const int lb = lower_bound_f(t, n, s), ub = upper_bound_f(t, n, s);
    const uint8_t k = tc[j];
    // list items below / equal to t_j, then minus the positives among them
    const long lt_all0 = lt0[j], lt_all1 = lt1[j];
    const long eq_all0 = h[2 * (kRankCap + 1) + lb], eq_all1 = h[3 * (kRankCap + 1) + lb];
    const long ltn0 = lt_all0 - c0[lb], ltn1 = lt_all1 - c1[lb];
    const long eqn0 = eq_all0 - (c0[ub] - c0[lb]), eqn1 = eq_all1 - (c1[ub] - c1[lb]);
    if (mode == 0) {
      if (k & 1) u_pos += (double)ltn1 + 0.5 * (double)eqn1;
      if (k & 2) u_neg += (double)ltn0 + 0.5 * (double)eqn0;
      const long mult = (k & 1) + ((k >> 1) & 1);
      const long pos_ge = mtot - (c0[lb] + c1[lb]);
      const long all_ge = (n0 - lt_all0) + (n1 - lt_all1);
      ap_sum += (double)mult * ((double)pos_ge / (double)all_ge);
    } else {
      // every threshold is a positive; the label-0 list is all of list 0, positives included
      u_pos += (double)lt_all0 + 0.5 * (double)eq_all0;
      const long pos_ge = n - lb;
      ap_sum += (double)pos_ge / (double)((n0 - lt_all0) + pos_ge);
    }
  }
  red[0][tid] = u_pos;
  red[1][tid] = u_neg;
  red[2][tid] = ap_sum;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, bsum = 0.0, c = 0.0;
    for (int k = 0; k < 256; ++k) {
      a += red[0][k];
      bsum += red[1][k];
      c += red[2][k];
    }
    double r_auc, r_ap;
    if (mode == 0) {
      // pos set: list-0 positives + list-1 negatives; neg set: list-0 negatives + list-1 positives
      const long nn1 = n1 - p1, nn0 = n0 - p0;
      const double a_pos = nn1 == 0 ? 1.0 : p0 == 0 ? 0.0 : a / ((double)p0 * (double)nn1);
      const double a_neg = nn0 == 0 ? 1.0 : p1 == 0 ? 0.0 : bsum / ((double)p1 * (double)nn0);
      const long sz_pos = p0 + nn1, sz_neg = nn0 + p1, total = sz_pos + sz_neg;
      r_auc = total ? ((double)sz_pos / (double)total) * a_pos + ((double)sz_neg / (double)total) * a_neg : 0.0;
      r_ap = mtot ? c / (double)mtot : 0.0;
      // bit 1: average_precision_score sees every list item's score (nn/dcue.py:447)
      flag[q_offset + i] = (p0 > 0) | (w.nonfin[i] ? 2 : 0);
    } else {
      // targets = [1] * n positives + [0] * n0 list items (nn/dcue.py:463-474)
      if (n0 == 0) {
        r_auc = 1.0;
        r_ap = 1.0;
      } else if (n == 0) {
        r_auc = 0.0;
        r_ap = 0.0;
      } else {
        r_auc = a / ((double)n * (double)n0);
        r_ap = c / (double)n;
      }
      // bit 1: roc_auc_score / average_precision_score run only with both labels (:467-474)
      flag[q_offset + i] = (n > 0) | (w.nonfin[i] && n > 0 && n0 > 0 ? 2 : 0);
    }
    auc[q_offset + i] = r_auc;
    ap[q_offset + i] = r_ap;
  }
}

__global__ void k_repeat_mean(float* f, int64_t n, int n_iter) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float x = f[k];
  float acc = 0.f;
  for (int it = 0; it < n_iter; ++it) acc += x;
  f[k] = acc / (float)n_iter;
}

static size_t rank_carve(int64_t n_cand, int32_t d, int32_t qb, void* base, float** cn, float** qn,
                         float** S, RankWs* w) {
  Arena ar{reinterpret_cast<char*>(base), 0, 0};
  const int dp = rank_dp(d);
  *cn = ar.take<float>((size_t)n_cand * dp);
  *qn = ar.take<float>((size_t)qb * dp);
  *S = ar.take<float>((size_t)qb * n_cand);
  w->thr = ar.take<float>((size_t)qb * kRankCap);
  w->thr_cls = ar.take<uint8_t>((size_t)qb * kRankCap);
  w->n_thr = ar.take<int32_t>(qb);
  w->hist = ar.take<int32_t>((size_t)qb * 4 * (kRankCap + 1));
  w->status = ar.take<int32_t>(1);
  w->nonfin = ar.take<int32_t>(qb);
  return ar.used;
}

}  // namespace dcue

using namespace dcue;

extern "C" {

int dcue_rank_workspace_bytes(int64_t n_cand, int32_t d, int32_t query_batch, size_t* bytes) {
  if (!bytes || n_cand < 0 || d <= 0 || d > 256 || query_batch <= 0) return DCUE_ERR_INVALID;
  float *cn, *qn, *S;
  RankWs w;
  *bytes = rank_carve(n_cand, d, query_batch, nullptr, &cn, &qn, &S, &w);
  return DCUE_OK;
}

int dcue_rank_metrics(const float* query_feat, int64_t n_query_rows, const float* cand_feat,
                      int64_t n_cand, int32_t d, const int32_t* queries, int32_t n_queries,
                      const int64_t* pos_ptr, const int32_t* pos_idx, const uint8_t* cand_class,
                      int32_t mode, int32_t query_batch, void* ws, size_t ws_bytes, double* auc,
                      double* ap, int32_t* has_pos, void* stream) {
  if (!query_feat || !cand_feat || !queries || !pos_ptr || !cand_class || !ws || !auc || !ap ||
      !has_pos || d <= 0 || d > 256 || n_cand <= 0 || n_query_rows <= 0 || n_queries < 0 ||
      query_batch <= 0 || (mode != DCUE_RANK_SPLIT && mode != DCUE_RANK_SINGLE))
    return DCUE_ERR_INVALID;
  if (n_queries == 0) return DCUE_OK;
  if (n_cand > INT32_MAX) return DCUE_ERR_UNSUPPORTED;
  float *cn, *qn, *S;
  RankWs w;
  if (rank_carve(n_cand, d, query_batch, nullptr, &cn, &qn, &S, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  rank_carve(n_cand, d, query_batch, ws, &cn, &qn, &S, &w);
  hipStream_t s = (hipStream_t)stream;
  const int dp = rank_dp(d);
  const size_t lds_scores = (size_t)2 * kRankTile * (dp + 4) * sizeof(float);
  const size_t lds_hist = (size_t)kRankCap * sizeof(float) + (size_t)4 * (kRankCap + 1) * sizeof(int);
  static bool attr = false;
  if (!attr) {
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_scores,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(2 * kRankTile * (256 + 4) * sizeof(float))));
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_hist, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_hist));
    attr = true;
  }
  DCUE_HIP_CHECK(hipMemsetAsync(w.status, 0xff, sizeof(int32_t), s));
  DCUE_LAUNCH(k_rank_normalize, dim3((unsigned)((n_cand + 3) / 4)), dim3(256), 0, s, cand_feat,
              (const int32_t*)nullptr, n_cand, d, dp, cn);
  DCUE_LAUNCH_CHECK();
  for (int32_t q0 = 0; q0 < n_queries; q0 += query_batch) {
    const int nq = n_queries - q0 < query_batch ? n_queries - q0 : query_batch;
    DCUE_LAUNCH(k_rank_normalize, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, query_feat,
                queries + q0, (int64_t)nq, d, dp, qn);
    DCUE_LAUNCH_CHECK();
    DCUE_LAUNCH(k_rank_scores, dim3((unsigned)((n_cand + kRankTile - 1) / kRankTile), (unsigned)((nq + kRankTile - 1) / kRankTile)),
                dim3(256), lds_scores, s, qn, nq, cn, n_cand, dp, S, n_cand);
    DCUE_LAUNCH_CHECK();
    DCUE_LAUNCH(k_rank_thresholds, dim3((unsigned)nq), dim3(256), 0, s, S, n_cand, queries + q0, pos_ptr,
                pos_idx, cand_class, n_cand, mode == DCUE_RANK_SPLIT ? 3 : 2, w);
    DCUE_LAUNCH_CHECK();
    DCUE_LAUNCH(k_rank_hist, dim3((unsigned)((n_cand + kRankChunk - 1) / kRankChunk), (unsigned)nq), dim3(256),
                lds_hist, s, S, n_cand, cand_class, n_cand, mode == DCUE_RANK_SPLIT ? 3 : 1, w);
    DCUE_LAUNCH_CHECK();
    DCUE_LAUNCH(k_rank_finalize, dim3((unsigned)nq), dim3(256), 0, s, w, mode, q0, auc, ap, has_pos);
    DCUE_LAUNCH_CHECK();
  }
  int32_t status = -1;
  DCUE_HIP_CHECK(hipMemcpyAsync(&status, w.status, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DCUE_HIP_CHECK(hipStreamSynchronize(s));
  if (status >= 0) {
    set_last_error("dcue_rank_metrics: a query has more than 4096 positives in the candidate lists",
                   hipErrorInvalidValue, __FILE__, __LINE__);
    return DCUE_ERR_UNSUPPORTED;
  }
  return DCUE_OK;
}

int dcue_factor_repeat_mean(float* f, int64_t n, int32_t n_iter, void* stream) {
  if (!f || n < 0 || n_iter < 1) return DCUE_ERR_INVALID;
  if (n == 0) return DCUE_OK;
  DCUE_LAUNCH(k_repeat_mean, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, f, n,
              (int)n_iter);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // extern "C"
