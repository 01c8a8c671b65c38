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
//                  and b in LDS, then an in-LDS blocked Cholesky A = L L^T (16-column steps: a
//                  register-resident diagonal factor, a panel solve, a rank-16 trailing update --
//                  three barriers per 16 columns) and the two blocked triangular solves.
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
    // Pad to D16 = dim rounded up to 16 with the identity (x = 0 there), then a blocked right-looking
    // Cholesky A = L L^T, 16 columns per step, three barriers per step instead of two per column:
    //  (1) wave 0 factors the 16 x 16 diagonal block in registers (lane i holds row i; pivots and
    //      columns broadcast by shuffles, no barrier); 1 / L[k][k] goes to dg[];
    //  (2) every row below solves its 16 panel entries against that block (one thread per row);
    //  (3) the trailing lower triangle takes the panel's rank-16 update (16 x 16 thread tiles).
    const int D16 = (dim + 15) & ~15;
    for (int i = dim + (t >> 4); i < D16; i += 16)
      for (int j = t & 15; j <= i; j += 16) A[i * kWrmfPitch + j] = i == j ? 1.0 : 0.0;
    for (int c = dim + t; c < D16; c += blockDim.x) bv[c] = 0.0;
    __syncthreads();
    const int ti = t >> 4, tj = t & 15;
    for (int k0 = 0; k0 < D16; k0 += 16) {
      if (t < 64) {
        const int i = t & 15;
        wacc_t row[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) row[j] = j <= i ? A[(k0 + i) * kWrmfPitch + k0 + j] : 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const wacc_t piv = sqrt(__shfl(row[k], k, 64));
          const wacc_t inv = 1.0 / piv;
          if (i == k) row[k] = piv;
          if (i > k) row[k] *= inv;
#pragma unroll
          for (int j = k + 1; j < 16; ++j) {
            const wacc_t ljk = __shfl(row[k], j, 64);  // L[j][k], scaled above
            if (i >= j) row[j] = fma(-row[k], ljk, row[j]);
          }
          if (t == k) dg[k0 + k] = inv;
        }
        if (t < 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (j <= i) A[(k0 + i) * kWrmfPitch + k0 + j] = row[j];
        }
      }
      __syncthreads();
      for (int r = k0 + 16 + t; r < D16; r += blockDim.x) {  // panel: L[r][k0..k0+15]
        wacc_t x[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = A[r * kWrmfPitch + k0 + j];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          wacc_t v = x[j];
#pragma unroll
          for (int q = 0; q < j; ++q) v = fma(-x[q], A[(k0 + j) * kWrmfPitch + k0 + q], v);
          x[j] = v * dg[k0 + j];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) A[r * kWrmfPitch + k0 + j] = x[j];
      }
      __syncthreads();
      const int nb2 = (D16 - k0 - 16) >> 4;  // trailing 16-row blocks
      for (int bi = 0; bi < nb2; ++bi)
        for (int bj = 0; bj <= bi; ++bj) {
          const int i = k0 + 16 + 16 * bi + ti, j = k0 + 16 + 16 * bj + tj;
          if (j > i) continue;
          wacc_t acc = A[i * kWrmfPitch + j];
#pragma unroll
          for (int q = 0; q < 16; ++q) acc = fma(-A[i * kWrmfPitch + k0 + q], A[j * kWrmfPitch + k0 + q], acc);
          A[i * kWrmfPitch + j] = acc;
        }
      __syncthreads();
    }
    // L y = b, then L^T x = y, blocked the same way: wave 0 solves a diagonal block (lane i holds
    // entry i, the solved entries broadcast by shuffles), then every thread removes the block's
    // contribution from the remaining rows (below for L, above for L^T)
    for (int k0 = 0; k0 < D16; k0 += 16) {
      if (t < 64) {
        const int i = t & 15;
        wacc_t y = bv[k0 + i];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const wacc_t yk = __shfl(y, k, 64) * dg[k0 + k];
          if (i == k) y = yk;
          else if (i > k) y = fma(-A[(k0 + i) * kWrmfPitch + k0 + k], yk, y);
        }
        if (t < 16) bv[k0 + i] = y;
      }
      __syncthreads();
      for (int r = k0 + 16 + t; r < D16; r += blockDim.x) {
        wacc_t v = bv[r];
#pragma unroll
        for (int q = 0; q < 16; ++q) v = fma(-A[r * kWrmfPitch + k0 + q], bv[k0 + q], v);
        bv[r] = v;
      }
      __syncthreads();
    }
    for (int k0 = D16 - 16; k0 >= 0; k0 -= 16) {
      if (t < 64) {
        const int i = t & 15;
        wacc_t x = bv[k0 + i];
#pragma unroll
        for (int k = 15; k >= 0; --k) {
          const wacc_t xk = __shfl(x, k, 64) * dg[k0 + k];
          if (i == k) x = xk;
          else if (i < k) x = fma(-A[(k0 + k) * kWrmfPitch + k0 + i], xk, x);  // L^T[i][k] = L[k][i]
        }
        if (t < 16) bv[k0 + i] = x;
      }
      __syncthreads();
      for (int r = t; r < k0; r += blockDim.x) {
        wacc_t v = bv[r];
#pragma unroll
        for (int q = 0; q < 16; ++q) v = fma(-A[(k0 + q) * kWrmfPitch + r], bv[k0 + q], v);
        bv[r] = v;
      }
      __syncthreads();
    }
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
