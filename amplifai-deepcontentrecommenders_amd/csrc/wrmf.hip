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
//   k_wrmf_solve   one workgroup per row (grid-stride): A and b accumulated in register tiles, a
//                  right-looking Cholesky of [[A, b], [b^T, *]] (16-column steps) whose last row
//                  is L^{-1} b, then L^T x = y (see the kernel)
// All of it in fp64: A's condition number is max eig(G + ...)/lambda, 1e4-1e6 for typical lambda,
// which an fp32 Cholesky (or an fp32 Gram matrix) turns into 1e-3 relative errors. dim <= 128; the
// factors stay fp32 in HBM.
#include "dcue_internal.h"


namespace dcue {

constexpr int kWrmfMaxDim = 128;
typedef double wacc_t;
// rows 0..128 (128: the augmented row) of the tile-padded triangle, then an 8-double dummy row
constexpr int kWrmfDummy = 32 * (kWrmfMaxDim / 8) * (kWrmfMaxDim / 8 + 1) + 8 * (kWrmfMaxDim / 8 + 1);
constexpr int kWrmfTri = kWrmfDummy + 8;
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

// G in a D16 x D16 layout (D16 = dim rounded up to 16), zero past dim: the solve reads whole 8 x 8
// tiles without bounds checks
__global__ __launch_bounds__(256) void k_wrmf_gram_reduce(const wacc_t* __restrict__ part, int nchunk, int dim,
                                                          wacc_t* __restrict__ G) {
  const int D16 = (dim + 15) & ~15;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)D16 * D16) return;
  const int i = (int)(e / D16), j = (int)(e - (long)i * D16);
  wacc_t s = 0.0;
  if (i < dim && j < dim) {
    const long dd = (long)dim * dim;
    for (int z = 0; z < nchunk; ++z) s += part[(size_t)z * dd + (long)i * dim + j];
  }
  G[e] = s;
}

// uniform broadcast of lane `lane`'s value (v_readlane, no LDS round trip); `lane` is uniform
__device__ inline double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
// 1 / sqrt(x) to fp64 precision: the hardware estimate and two Newton steps
__device__ inline double rsqrt_d(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
#pragma unroll
  for (int it = 0; it < 2; ++it) y = fma(y, fma(-h * y, y, 0.5), y);
  return y;
}
// packed lower triangle with rows padded to whole 8-column tiles: row r holds columns
// 0 .. 8 (r / 8) + 7, so a diagonal tile is stored whole (its upper part lands in the row's own padding)
__device__ inline int woff(int r) {
  const int m = r >> 3;
  return 32 * m * (m + 1) + 8 * (m + 1) * (r - 8 * m);
}

// One workgroup per row (grid-stride), two workgroups per CU (80 KB of LDS each, <= 256 VGPRs). The
// row's system is the augmented matrix [[A, b], [b^T, *]] of size D16 + 1 (D16 = dim rounded up to
// 16, padded with the identity): its Cholesky factor's last row is y = L^{-1} b, so the forward
// solve comes out of the factorisation and only L^T x = y remains.
//   * A lives in registers as 8 x 8 tiles of the lower triangle (thread t owns tile t; the
//     augmented row b^T adds one tile per tile column, of which row 0 is real): the accumulation
//     A = G + lambda I + sum (c - 1) f f^T, b = sum c f is 64 FMAs per staged factor per tile, and
//     the right-looking Cholesky's trailing update is a register-tile rank-16 update.
//   * Per 16-column step: the diagonal block's three tiles go to LDS (packed lower triangle, rows
//     padded to whole tiles, woff); wave 0 factors it in lanes 0-15 (v_readlane broadcasts);
//     the panel tiles below solve against it in their owners' registers (first tile column, then
//     the second after removing the first's part) and are stored; the trailing tiles read the panel
//     from LDS. Four barriers per step.
//   * L^T x = y: wave 0, lane l holding x[l] and x[l + 64], eight rows of L at a time.
// Tiles are numbered by tile column descending, so the trailing tiles of every step are a prefix
// of the thread range (the later steps keep fewer waves busy). Loop-invariant per-thread values are
// passed through empty asm at the row and step boundaries, so their address arithmetic is redone
// there instead of being hoisted into live registers (which would spill at 256 VGPRs).
__global__ __launch_bounds__(256, 2) void k_wrmf_solve(float* __restrict__ X, long n_rows, const float* __restrict__ F,
                                                    int dim, const wacc_t* __restrict__ G,
                                                    const int64_t* __restrict__ indptr,
                                                    const int32_t* __restrict__ indices,
                                                    const float* __restrict__ values, float alpha, float lambda) {
  extern __shared__ __attribute__((aligned(16))) wacc_t wl[];
  wacc_t* Ls = wl;                                          // packed lower triangle, rows 0..D16
  wacc_t* dg = Ls + kWrmfTri;                               // 1 / L[k][k]
  float* st = reinterpret_cast<float*>(dg + kWrmfMaxDim);   // [kWrmfStage][kWrmfMaxDim] staged f_j
  float* cs = st + kWrmfStage * kWrmfMaxDim;                // [kWrmfStage] c_j - 1
  const int t = threadIdx.x, lane = t & 63;
  const int D16 = (dim + 15) & ~15, NT = D16 >> 3, RA = D16;  // RA: the augmented row (b^T, then y^T)
  // this thread's tile (TI, TJ): tile columns descending, rows TJ..NT (NT: the augmented row)
  int TI = -1, TJ = -1;
  {
    int base = 0;
    for (int tj = NT - 1; tj >= 0; --tj) {
      const int cnt = NT - tj + 1;
      if (t >= base && t < base + cnt) {
        TJ = tj;
        TI = tj + (t - base);
      }
      base += cnt;
    }
  }
  const bool has_tile = TJ >= 0, aug = TI == NT;
  const int r0t = 8 * TI, c0t = 8 * TJ;
  for (long r = blockIdx.x; r < n_rows; r += gridDim.x) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    if (p1 <= p0) {  // no observed pair: b = 0, so x = 0
      for (int c = t; c < dim; c += blockDim.x) X[r * dim + c] = 0.f;
      continue;
    }
    // per-thread tile coordinates, opaque to the compiler per row: address arithmetic is redone
    // here instead of being hoisted out of the row loop into (too many) live registers
    int r0 = r0t, c0 = c0t;
    asm volatile("" : "+v"(r0), "+v"(c0));
    wacc_t acc[8][8];
    // A = G + lambda I (identity on the padding), the augmented row's b = 0. G has pitch D16 and is
    // zero past dim; the loads are unconditional (clamped rows) so they issue back to back
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const wacc_t* g = G + (size_t)min(max(r0 + i, 0), D16 - 1) * D16 + max(c0, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = g[j];
    }
    if (!has_tile || aug) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;
    } else if (TI == TJ) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i][i] += r0 + i < dim ? (wacc_t)lambda : 1.0;
    }
    // the row's observed factors: A += (c - 1) f f^T, b += c f, kWrmfStage at a time
    for (long pb = p0; pb < p1; pb += kWrmfStage) {
      const int ns = (int)min((long)kWrmfStage, p1 - pb);
      for (int e = t; e < ns * D16; e += blockDim.x) {
        const int s = e / D16, c = e - s * D16;
        st[s * kWrmfMaxDim + c] = c < dim ? F[(long)indices[pb + s] * dim + c] : 0.f;
      }
      if (t < ns) cs[t] = alpha * (values ? values[pb + t] : 1.f);  // c - 1
      __syncthreads();
      if (has_tile) {
#pragma unroll 1
        for (int s = 0; s < ns; ++s) {
          const wacc_t w = (wacc_t)cs[s];
          wacc_t fc[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) fc[j] = (wacc_t)st[s * kWrmfMaxDim + c0 + j];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            // (c - 1) f_i on A's rows; the augmented tile's row 0 takes c (b += c f), its rows 1-7 nothing
            const wacc_t fi = (wacc_t)st[s * kWrmfMaxDim + (aug ? 0 : r0 + i)];
            const wacc_t wi = aug ? (i == 0 ? 1.0 + w : 0.0) : w * fi;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = fma(wi, fc[j], acc[i][j]);
          }
        }
      }
      __syncthreads();
    }
    // tile -> LDS (its lower part; the augmented tile's row 0)
    // L's row of tile row i (the augmented tile's rows all read row RA; only row 0 is stored)
    auto rowi = [&](int i) { return aug ? RA : r0 + i; };
    auto store_tile = [&]() {  // whole tile (the augmented tile's rows 1-7 go to the dummy row)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        wacc_t* dst = Ls + (aug && i ? kWrmfDummy : woff(rowi(i)) + c0);
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[j] = acc[i][j];
      }
    };
    // in place on a panel tile: X L_cc^T = acc for the 8 columns c0.. (L_cc: L[c0..c0+7][c0..c0+7])
    auto solve_cols = [&]() {
      for (int q = 0; q < 8; ++q) {
        const wacc_t d = dg[c0 + q];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][q] *= d;
#pragma unroll
        for (int j = q + 1; j < 8; ++j) {
          const wacc_t l = Ls[woff(c0 + j) + c0 + q];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i][j] = fma(-acc[i][q], l, acc[i][j]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    const bool diag_tile = !aug && (TI >> 1) == (TJ >> 1);  // inside a 16 x 16 diagonal block
    if (has_tile && TJ < 2 && diag_tile) store_tile();
    for (int k0 = 0; k0 < D16; k0 += 16) {
      const int kt = k0 >> 3;  // tile column of the step's first 8 columns
      asm volatile("" : "+v"(r0), "+v"(c0));
      __syncthreads();
      if (t < 64) {
        // the 16 x 16 diagonal block, factored in wave 0's lanes 0-15 (lane i holds row i)
        int i = lane;
        asm volatile("" : "+v"(i));  // lane predicates are formed here, not hoisted out of the k0 loop
        wacc_t row[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) row[j] = (i < 16 && j <= i) ? Ls[woff(k0 + i) + k0 + j] : 0.0;
        wacc_t myinv = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const wacc_t pk = readlane_d(row[k], k);
          const wacc_t inv = rsqrt_d(pk);
          if (i == k) {
            row[k] = pk * inv;
            myinv = inv;
          } else if (i > k) {
            row[k] *= inv;
          }
#pragma unroll
          for (int j = k + 1; j < 16; ++j) {
            const wacc_t ljk = readlane_d(row[k], j);
            if (i >= j) row[j] = fma(-row[k], ljk, row[j]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (i < 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (j <= i) Ls[woff(k0 + i) + k0 + j] = row[j];
          dg[k0 + i] = myinv;
        }
      }
      __syncthreads();
      // the panel below the block, in its owners' registers: first tile column (columns k0..k0+7)
      const bool below = has_tile && TI >= kt + 2;
      if (below && TJ == kt) {
        solve_cols();
        store_tile();
      }
      __syncthreads();
      // second tile column: remove the first column's part, then solve against L[k0+8..][k0+8..]
      if (below && TJ == kt + 1) {
#pragma unroll 1
        for (int q = 0; q < 8; ++q) {
          wacc_t xa[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) xa[i] = Ls[woff(rowi(i)) + k0 + q];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const wacc_t l = Ls[woff(c0 + j) + k0 + q];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i][j] = fma(-xa[i], l, acc[i][j]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        solve_cols();
        store_tile();
      }
      __syncthreads();
      // trailing tiles: acc -= L[rows][k0:k0+16] L[cols][k0:k0+16]^T; then the next diagonal block's tiles
      if (has_tile && c0 >= k0 + 16) {
#pragma unroll 1
        for (int q = 0; q < 16; ++q) {
          wacc_t fc[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) fc[j] = Ls[woff(c0 + j) + k0 + q];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const wacc_t li = Ls[woff(rowi(i)) + k0 + q];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = fma(-li, fc[j], acc[i][j]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (c0 < k0 + 32 && diag_tile) store_tile();
      }
    }
    __syncthreads();
    // L^T x = y (y: the augmented row), wave 0; eight rows of L loaded ahead of each chain
    if (t < 64) {
      const wacc_t* y = Ls + woff(RA);
      wacc_t xlo = lane < D16 ? y[lane] : 0.0, xhi = lane + 64 < D16 ? y[lane + 64] : 0.0;
      for (int kb = D16 - 8; kb >= 0; kb -= 8) {
        wacc_t llo[8], lhi[8], dk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = kb + 7 - u;
          llo[u] = lane < k ? Ls[woff(k) + lane] : 0.0;
          lhi[u] = lane + 64 < k ? Ls[woff(k) + lane + 64] : 0.0;
          dk[u] = dg[k];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = kb + 7 - u;
          const bool hi = k >= 64;
          const wacc_t xk = readlane_d(hi ? xhi : xlo, k & 63) * dk[u];
          if (lane == (k & 63)) {
            if (hi) xhi = xk;
            else xlo = xk;
          }
          xlo = fma(-llo[u], xk, xlo);
          xhi = fma(-lhi[u], xk, xhi);
        }
      }
      if (lane < dim) X[r * dim + lane] = (float)xlo;
      if (lane + 64 < dim) X[r * dim + lane + 64] = (float)xhi;
    }
    __syncthreads();  // Ls and dg are rewritten by the next row
  }
}

size_t wrmf_solve_lds_bytes() {
  return sizeof(wacc_t) * ((size_t)kWrmfTri + kWrmfMaxDim) + sizeof(float) * ((size_t)kWrmfStage * kWrmfMaxDim + kWrmfStage);
}

long wrmf_gram_chunks(long n_fixed) { return (n_fixed + kWrmfGramChunk - 1) / kWrmfGramChunk; }

}  // namespace dcue

extern "C" {

int dcue_wrmf_workspace_bytes(int32_t dim, int64_t n_fixed, size_t* bytes_host) {
  if (!bytes_host || dim <= 0 || dim > dcue::kWrmfMaxDim || n_fixed < 0) return DCUE_ERR_INVALID;
  const long nch = dcue::wrmf_gram_chunks(n_fixed < 1 ? 1 : n_fixed);
  const size_t d16 = (size_t)((dim + 15) & ~15);
  *bytes_host = sizeof(dcue::wacc_t) * ((size_t)nch * dim * dim + d16 * d16) + 256;
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
  const long dd = (long)((dim + 15) & ~15) * ((dim + 15) & ~15);
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
