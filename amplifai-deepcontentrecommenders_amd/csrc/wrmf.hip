// WRMF target factors for the DCBR path (BASELINE config 5) -- gfx950.
//
// No reference code exists: dcrecommend/dcbr is git-ignored in the reference (.gitignore:13), so
// this restates the published algorithms and is parity-unpinned against the reference (pinned
// against oracle/wrmf_oracle.py, a numpy fp64 restatement):
//   * WRMF / implicit ALS (Hu, Koren, Volinsky, "Collaborative Filtering for Implicit Feedback
//     Datasets", ICDM 2008): preference p_rj = 1 on observed pairs, confidence c_rj = 1 + alpha v_rj,
//     and one half-step solves every row of one side with the other side fixed:
//       x_r = (F^T F + F^T (C_r - I) F + lambda I)^{-1} F^T C_r p_r
//           = (G + sum_{j in r} (c_rj - 1) f_j f_j^T + lambda I)^{-1} sum_{j in r} c_rj f_j.
//   * DCBR (van den Oord, Dieleman, Schrauwen, "Deep content-based music recommendation", NIPS
//     2013): the audio ConvNet regresses the item factors under an MSE loss (dcue_dcbr_step).
//
// Data layout: factors row-major [n][dim] fp32; the observed pairs of the rows being solved as a
// CSR (indptr int64 [n_rows + 1], indices int32 [nnz] into the fixed side, values fp32 or NULL).
//
// Kernels:
//   k_wrmf_gram    G = F^T F over row chunks: a workgroup sums its chunk's rank-1 terms in
//                  registers (thread t owns G[t & 127][(t >> 7) * 64 + 0..63]); partials [chunk][d][d]
//   k_wrmf_gram_reduce  the chunk partials in a fixed order (deterministic)
//   k_wrmf_solve   one workgroup per row (grid-stride): A = G + lambda I + the row's rank-1 terms
//                  and b in LDS, then an in-LDS Cholesky A = L L^T and the two triangular solves.
// All of it in fp64: A's condition number is max eig(G + ...)/lambda, 1e4-1e6 for typical lambda,
// which an fp32 Cholesky (or an fp32 Gram matrix) turns into 1e-3 relative errors. dim <= 128: A
// is [128][129] doubles (132 KB, one workgroup per CU); the factors stay fp32 in HBM.
#include "dcue_internal.h"

namespace dcue {

constexpr int kWrmfMaxDim = 128;
typedef double wacc_t;
constexpr int kWrmfPitch = kWrmfMaxDim + 1;  // odd pitch: column walks hit distinct banks
constexpr int kWrmfGramChunk = 2048;         // fixed-side rows per gram workgroup
constexpr int kWrmfStage = 16;               // observed factors staged in LDS per pass

__global__ __launch_bounds__(256) void k_wrmf_gram(const float* __restrict__ F, long n, int dim,
                                                   wacc_t* __restrict__ part) {
  __shared__ float rows[kWrmfStage][kWrmfMaxDim];
  const int t = threadIdx.x;
  const int i = t & 127, j0 = (t >> 7) * 64;
  wacc_t acc[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) acc[q] = 0.0;
  const long r0 = (long)blockIdx.x * kWrmfGramChunk;
  const long r1 = min(r0 + kWrmfGramChunk, n);
  for (long rb = r0; rb < r1; rb += kWrmfStage) {
    const int nr = (int)min((long)kWrmfStage, r1 - rb);
    for (int e = t; e < kWrmfStage * kWrmfMaxDim; e += blockDim.x) {
      const int r = e / kWrmfMaxDim, c = e - r * kWrmfMaxDim;
      rows[r][c] = (r < nr && c < dim) ? F[(rb + r) * dim + c] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < nr; ++r) {
      const wacc_t a = rows[r][i];
#pragma unroll
      for (int q = 0; q < 64; ++q) acc[q] = fma(a, (wacc_t)rows[r][j0 + q], acc[q]);
    }
    __syncthreads();
  }
  if (i < dim) {
    wacc_t* out = part + (size_t)blockIdx.x * dim * dim + (size_t)i * dim;
#pragma unroll
    for (int q = 0; q < 64; ++q)
      if (j0 + q < dim) out[j0 + q] = acc[q];
  }
}

__global__ __launch_bounds__(256) void k_wrmf_gram_reduce(const wacc_t* __restrict__ part, int nchunk, int dim,
                                                          wacc_t* __restrict__ G) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long dd = (long)dim * dim;
  if (e >= dd) return;
  wacc_t s = 0.0;
  for (int z = 0; z < nchunk; ++z) s += part[(size_t)z * dd + e];
  G[e] = s;
}

__global__ __launch_bounds__(256) void k_wrmf_solve(float* __restrict__ X, long n_rows, const float* __restrict__ F,
                                                    int dim, const wacc_t* __restrict__ G,
                                                    const int64_t* __restrict__ indptr,
                                                    const int32_t* __restrict__ indices,
                                                    const float* __restrict__ values, float alpha, float lambda) {
  extern __shared__ __attribute__((aligned(16))) wacc_t wl[];
  wacc_t* A = wl;                                  // [dim][kWrmfPitch], lower triangle used
  wacc_t* bv = A + kWrmfMaxDim * kWrmfPitch;       // b, then x
  __shared__ wacc_t dg[kWrmfMaxDim];               // 1 / L's diagonal
  float* st = reinterpret_cast<float*>(bv + kWrmfMaxDim);  // [kWrmfStage][dim] staged f_j
  float* cs = st + kWrmfStage * kWrmfMaxDim;       // [kWrmfStage] c_j - 1
  const int t = threadIdx.x;
  for (long r = blockIdx.x; r < n_rows; r += gridDim.x) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    if (p1 <= p0) {  // no observed pair: b = 0, so x = 0
      for (int c = t; c < dim; c += blockDim.x) X[r * dim + c] = 0.f;
      continue;
    }
    // A = G + lambda I (lower triangle and diagonal), b = 0
    for (int i = t >> 4; i < dim; i += 16)
      for (int j = t & 15; j <= i; j += 16) A[i * kWrmfPitch + j] = G[i * dim + j] + (i == j ? (wacc_t)lambda : 0.0);
    for (int c = t; c < dim; c += blockDim.x) bv[c] = 0.0;
    __syncthreads();
    // the row's observed factors: A += (c - 1) f f^T, b += c f, kWrmfStage at a time
    for (long pb = p0; pb < p1; pb += kWrmfStage) {
      const int ns = (int)min((long)kWrmfStage, p1 - pb);
      for (int e = t; e < ns * dim; e += blockDim.x) {
        const int s = e / dim, c = e - s * dim;
        st[s * kWrmfMaxDim + c] = F[(long)indices[pb + s] * dim + c];
      }
      if (t < ns) cs[t] = alpha * (values ? values[pb + t] : 1.f);  // c - 1
      __syncthreads();
      for (int i = t >> 4; i < dim; i += 16)
        for (int j = t & 15; j <= i; j += 16) {
          wacc_t a = A[i * kWrmfPitch + j];
          for (int s = 0; s < ns; ++s)
            a = fma((wacc_t)cs[s] * st[s * kWrmfMaxDim + i], (wacc_t)st[s * kWrmfMaxDim + j], a);
          A[i * kWrmfPitch + j] = a;
        }
      for (int c = t; c < dim; c += blockDim.x) {
        wacc_t b = bv[c];
        for (int s = 0; s < ns; ++s) b = fma(1.0 + (wacc_t)cs[s], (wacc_t)st[s * kWrmfMaxDim + c], b);
        bv[c] = b;
      }
      __syncthreads();
    }
    // Cholesky, right-looking, two barriers per column: every thread reads the pivot, the column
    // below it is scaled, then the trailing lower triangle loses the column's outer product. The
    // diagonal of L goes to dg[] (A[k][k] stays the pivot's square until every thread has read it)
    for (int k = 0; k < dim; ++k) {
      const wacc_t piv = sqrt(A[k * kWrmfPitch + k]);
      const wacc_t inv = 1.0 / piv;
      if (t == 0) dg[k] = inv;  // the solves multiply by 1 / L[k][k]
      for (int i = k + 1 + t; i < dim; i += blockDim.x) A[i * kWrmfPitch + k] *= inv;
      __syncthreads();
      // 16 x 16 threads over (row, column) of the trailing lower triangle
      for (int i = k + 1 + (t >> 4); i < dim; i += 16) {
        const wacc_t lik = A[i * kWrmfPitch + k];
        for (int j = k + 1 + (t & 15); j <= i; j += 16)
          A[i * kWrmfPitch + j] = fma(-lik, A[j * kWrmfPitch + k], A[i * kWrmfPitch + j]);
      }
      __syncthreads();
    }
    // L y = b, then L^T x = y: wave 0 alone, lane l holding entries l and l + 64 in registers (no
    // barriers; y_k / x_k broadcast by shuffle from the owning lane; x/L[k][k] as x * (1/L[k][k]),
    // one rounding more than the division, far below the fp32 output's)
    if (t < 64) {
      wacc_t v0 = t < dim ? bv[t] : 0.0, v1 = t + 64 < dim ? bv[t + 64] : 0.0;
      for (int k = 0; k < dim; ++k) {
        const wacc_t own = k < 64 ? v0 : v1;
        const wacc_t yk = __shfl(own, k & 63, 64) * dg[k];
        if (t == (k & 63)) {
          if (k < 64) v0 = yk; else v1 = yk;
        }
        if (t > k && t < dim) v0 = fma(-A[t * kWrmfPitch + k], yk, v0);
        if (t + 64 > k && t + 64 < dim) v1 = fma(-A[(t + 64) * kWrmfPitch + k], yk, v1);
      }
      for (int k = dim - 1; k >= 0; --k) {
        const wacc_t own = k < 64 ? v0 : v1;
        const wacc_t xk = __shfl(own, k & 63, 64) * dg[k];
        if (t == (k & 63)) {
          if (k < 64) v0 = xk; else v1 = xk;
        }
        if (t < k) v0 = fma(-A[k * kWrmfPitch + t], xk, v0);
        if (t + 64 < k) v1 = fma(-A[k * kWrmfPitch + t + 64], xk, v1);
      }
      if (t < dim) bv[t] = v0;
      if (t + 64 < dim) bv[t + 64] = v1;
    }
    __syncthreads();
    for (int c = t; c < dim; c += blockDim.x) X[r * dim + c] = (float)bv[c];
    __syncthreads();  // bv and A are rewritten by the next row
  }
}

size_t wrmf_solve_lds_bytes() {
  return sizeof(wacc_t) * ((size_t)kWrmfMaxDim * kWrmfPitch + kWrmfMaxDim) +
         sizeof(float) * ((size_t)kWrmfStage * kWrmfMaxDim + kWrmfStage);
}

long wrmf_gram_chunks(long n_fixed) { return (n_fixed + kWrmfGramChunk - 1) / kWrmfGramChunk; }

}  // namespace dcue

extern "C" {

int dcue_wrmf_workspace_bytes(int32_t dim, int64_t n_fixed, size_t* bytes_host) {
  if (!bytes_host || dim <= 0 || dim > dcue::kWrmfMaxDim || n_fixed < 0) return DCUE_ERR_INVALID;
  const long nch = dcue::wrmf_gram_chunks(n_fixed < 1 ? 1 : n_fixed);
  *bytes_host = sizeof(dcue::wacc_t) * ((size_t)nch * dim * dim + (size_t)dim * dim) + 256;
  return DCUE_OK;
}

int dcue_wrmf_half_step(float* solve, int64_t n_rows, const float* fixed, int64_t n_fixed, int32_t dim,
                        const int64_t* indptr, const int32_t* indices, const float* values, float alpha,
                        float lambda, void* ws, size_t ws_bytes, void* stream) {
  using namespace dcue;
  if (dim <= 0 || dim > kWrmfMaxDim) return DCUE_ERR_UNSUPPORTED;
  if (!solve || !fixed || !indptr || (!indices && n_rows > 0) || n_rows < 0 || n_fixed <= 0 || !ws ||
      !(lambda > 0.f) || alpha < 0.f)
    return DCUE_ERR_INVALID;
  size_t need = 0;
  int st = dcue_wrmf_workspace_bytes(dim, n_fixed, &need);
  if (st) return st;
  if (ws_bytes < need) return DCUE_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const long nch = wrmf_gram_chunks(n_fixed);
  wacc_t* part = reinterpret_cast<wacc_t*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
  wacc_t* G = part + (size_t)nch * dim * dim;
  DCUE_LAUNCH(k_wrmf_gram, dim3((unsigned)nch), dim3(256), 0, s, fixed, (long)n_fixed, (int)dim, part);
  DCUE_LAUNCH_CHECK();
  const long dd = (long)dim * dim;
  DCUE_LAUNCH(k_wrmf_gram_reduce, dim3((unsigned)((dd + 255) / 256)), dim3(256), 0, s, part, (int)nch, (int)dim, G);
  DCUE_LAUNCH_CHECK();
  if (n_rows == 0) return DCUE_OK;
  const size_t lds = wrmf_solve_lds_bytes();
  // the dynamic-LDS limit is a per-device function attribute: set it on every call (cheap), so a
  // process that also solves on another device gets it there too
  DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_wrmf_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
  const long grid = n_rows < 4096 ? n_rows : 4096;  // grid-stride over rows
  DCUE_LAUNCH(k_wrmf_solve, dim3((unsigned)grid), dim3(256), lds, s, solve, (long)n_rows, fixed, (int)dim, G,
              indptr, indices, values, alpha, lambda);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // extern "C"
