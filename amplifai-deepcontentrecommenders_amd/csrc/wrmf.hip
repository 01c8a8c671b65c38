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
//   k_wrmf_gram_mfma  G = F^T F over 512-row chunks on fp64 MFMA (lower block triangle, stored with
//                  its transpose); partials [chunk][d][d]. k_wrmf_gram (DCUE_WRMF_GRAM=scalar): the
//                  same with fp64 FMAs (thread t owns G[t & 127][(t >> 7) * 64 + 0..63])
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
constexpr int kWrmfGramChunk = 512;          // fixed-side rows per gram step (a multiple of 8)
// at most this many gram workgroups (2 per CU): past 512 x 512 fixed rows each workgroup strides over
// several chunks, so the fp64 partials ([workgroups][d][d], 64 MB at d = 128) and the reduce's
// traffic stay bounded however large the fixed side grows
constexpr long kWrmfGramMaxBlocks = 512;
constexpr int kWrmfStage = 16;               // observed factors staged in LDS per pass

__global__ __launch_bounds__(256) void k_wrmf_gram(const float* __restrict__ F, long n, int dim,
                                                   wacc_t* __restrict__ part) {
  __shared__ float rows[kWrmfStage][kWrmfMaxDim];
  const int t = threadIdx.x;
  const int i = t & 127, j0 = (t >> 7) * 64;
  wacc_t acc[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) acc[q] = 0.0;
  for (long r0 = (long)blockIdx.x * kWrmfGramChunk; r0 < n; r0 += (long)gridDim.x * kWrmfGramChunk)
  for (long rb = r0, r1 = min(r0 + kWrmfGramChunk, n); rb < r1; rb += kWrmfStage) {
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

// The same partials on fp64 MFMA (v_mfma_f64_16x16x4_f64, the default): G_IJ += F_chunk[:, I]^T
// F_chunk[:, J] four rows per MFMA, both operands straight from global memory in the MFMA operand
// layout (lane l: row l >> 4 of the step, column 16 X + (l & 15)). Only the lower block triangle is
// computed -- wave w owns block rows w and NB8 - 1 - w (NB8 = 8 tile rows at dim <= 128: 9 tiles
// per wave) -- and each tile is stored with its transpose, so the partials keep k_wrmf_gram's
// full [chunk][d][d] layout and k_wrmf_gram_reduce is shared.
typedef double wgf64x4 __attribute__((ext_vector_type(4)));
template <int W>  // the wave: block rows IA = W and IB = 7 - W, compile-time so every index is
__device__ __forceinline__ void wrmf_gram_wave(const float* __restrict__ F, long n, int dim,
                                               wacc_t* __restrict__ out) {
  constexpr int IA = W, IB = 7 - W;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int NB = (dim + 15) >> 4;
  // slots: (IA, J) for J <= IA, then (IB, J) for J <= IB -- 9 in all
  wgf64x4 acc[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) acc[q] = wgf64x4{0.0, 0.0, 0.0, 0.0};
  // the step's operands: v[X] = F[r + lk][16 X + li] (0 past the chunk or past dim); the loads are
  // unconditional (clamped), their values selected
  long r1 = 0;  // the current chunk's end
  auto load = [&](const long r, float (&v)[8]) {
    const long row = r + lk;
    const float* src = F + (row < r1 ? row : r1 - 1) * dim;
#pragma unroll
    for (int X = 0; X < 8; ++X) {
      const int c = 16 * X + li;
      const float x = src[c < dim ? c : dim - 1];
      v[X] = row < r1 && c < dim ? x : 0.f;
    }
  };
  auto step = [&](const float (&cur)[8]) {
    if (IA < NB) {
#pragma unroll
      for (int J = 0; J <= IA; ++J)
        acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)cur[IA], (double)cur[J], acc[J], 0, 0, 0);
    }
    if (IB < NB) {
#pragma unroll
      for (int J = 0; J <= IB; ++J)
        acc[IA + 1 + J] =
            __builtin_amdgcn_mfma_f64_16x16x4f64((double)cur[IB], (double)cur[J], acc[IA + 1 + J], 0, 0, 0);
    }
  };
  // two steps (8 rows) per iteration, the next two steps' loads in flight during these MFMAs (rows
  // past the chunk load as zeros, so the last pair may run half empty)
  float c0[8], c1[8], n0[8], n1[8];
  // the workgroup's chunks: blockIdx.x, + gridDim.x, ... (one chunk each below 512 x 512 rows)
#pragma unroll 1
  for (long r0 = (long)blockIdx.x * kWrmfGramChunk; r0 < n; r0 += (long)gridDim.x * kWrmfGramChunk) {
    r1 = min(r0 + kWrmfGramChunk, n);
    load(r0, c0);
    load(r0 + 4, c1);
#pragma unroll 1
    for (long r = r0; r < r1; r += 8) {
      load(r + 8, n0);
      load(r + 12, n1);
      step(c0);
      step(c1);
#pragma unroll
      for (int X = 0; X < 8; ++X) {
        c0[X] = n0[X];
        c1[X] = n1[X];
      }
    }
  }
  // tile (I, J) and, off the diagonal, its transpose (C layout: lane l holds column l & 15, rows
  // (l >> 4) + 4 q)
  auto store = [&](const int I, const int J, const wgf64x4& t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 16 * I + lk + 4 * q, j = 16 * J + li;
      if (i < dim && j < dim) {
        out[(size_t)i * dim + j] = t[q];
        if (I != J) out[(size_t)j * dim + i] = t[q];
      }
    }
  };
  if (IA < NB) {
#pragma unroll
    for (int J = 0; J <= IA; ++J) store(IA, J, acc[J]);
  }
  if (IB < NB) {
#pragma unroll
    for (int J = 0; J <= IB; ++J) store(IB, J, acc[IA + 1 + J]);
  }
}

__global__ __launch_bounds__(256, 2) void k_wrmf_gram_mfma(const float* __restrict__ F, long n, int dim,
                                                          wacc_t* __restrict__ part) {
  wacc_t* out = part + (size_t)blockIdx.x * dim * dim;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: wrmf_gram_wave<0>(F, n, dim, out); break;
    case 1: wrmf_gram_wave<1>(F, n, dim, out); break;
    case 2: wrmf_gram_wave<2>(F, n, dim, out); break;
    default: wrmf_gram_wave<3>(F, n, dim, out); break;
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
  if (i < dim && j < dim) {  // (four partial sums over z mod 4, combined in a fixed order)
    const long dd = (long)dim * dim;
    const wacc_t* src = part + (long)i * dim + j;
    wacc_t q[4] = {0.0, 0.0, 0.0, 0.0};
    int z = 0;
#pragma unroll 2
    for (; z + 4 <= nchunk; z += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] += src[(size_t)(z + u) * dd];
    for (; z < nchunk; ++z) q[z & 3] += src[(size_t)z * dd];
    s = (q[0] + q[1]) + (q[2] + q[3]);
  }
  G[e] = s;
}

// whether a row's pair weights alpha * v include a negative one (block-uniform; values NULL: all 1)
__device__ inline bool wrmf_row_has_negative(const float* __restrict__ values, long p0, long p1, float alpha) {
  if (!values || !(alpha > 0.f)) return false;
  bool neg = false;
  for (long p = p0 + threadIdx.x; p < p1; p += blockDim.x) neg |= alpha * values[p] < 0.f;
  return __syncthreads_or(neg);
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
                                                    const float* __restrict__ values, float alpha, float lambda,
                                                    int phases) {
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
    for (long pb = p0; pb < ((phases & 1) ? p1 : p0); pb += kWrmfStage) {
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
    for (int k0 = 0; k0 < ((phases & 2) ? D16 : 0); k0 += 16) {
      const int kt = k0 >> 3;  // tile column of the step's first 8 columns
      asm volatile("" : "+v"(r0), "+v"(c0));
      __syncthreads();
      if (t < 64 && (phases & 8)) {
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
      const bool below = has_tile && TI >= kt + 2 && (phases & 16);
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
      if (has_tile && c0 >= k0 + 16 && (phases & 32)) {
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
    if (t < 64 && (phases & 4)) {
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

// ------------------------------------------------------------------------------------------------
// k_wrmf_solve_mfma: the same per-row system on fp64 MFMA (v_mfma_f64_16x16x4_f64), D16 = 16 NB.
// One workgroup per row (grid-stride), 4 waves, two workgroups per CU. The augmented matrix
// [[A, b], [b^T, *]] is held as 16 x 16 tiles (I, J), J <= I, of the lower block triangle plus the
// augmented block row I = NB (only its row 0, b^T, is real): tile number
// tau(I, J) = J (NB + 1) - J (J - 1) / 2 + (I - J), owned by wave tau % 4 in its register slot tau / 4
// (C/D layout of the f64 MFMA: lane l holds column l & 15, rows (l >> 4) + 4 r, r = 0..3).
//   * accumulation: A_IJ += sum_s (c_s - 1) f_s[16 I + i] f_s[16 J + j], b += c_s f_s, as MFMAs of
//     K = 4 staged factors (A operand lane l: row l & 15, factor l >> 4);
//   * right-looking block Cholesky, per block column kb: wave 0 factors the diagonal tile (lanes
//     hold rows, v_readlane broadcasts) and inverts the factor (lane j: column j of L_kk^{-1}); the
//     panel L_Ikb = A_Ikb L_kk^{-T} and the trailing updates A_IJ -= L_Ikb L_Jkb^T are MFMAs with
//     operands read from LDS (the off-diagonal factor tiles stay there for the back substitution);
//     the augmented row's panel is y_kb = (L^{-1} b)_kb;
//   * L^T x = y block by block in wave 0 (four lanes per row, a shuffle reduction).
// LDS: off-diagonal factor tiles (I > J, I < NB) 16 x 16 each, column-major (an MFMA operand's
// 16 rows are 16 consecutive doubles: conflict-free), the inverses of the diagonal factors packed
// lower column-major (136 doubles each; the diagonal tile itself is factored there packed
// row-major first), y, x, the 1 / L[k][k] of the current block, and the staged factors (fp32) with
// their weights.
DCUE_KTRACE_READER(wrmf)  // diagnostic builds only (dcue_common.h): k_wrmf_solve_mfma, wave 0 / wave 1 cycles
#ifdef DCUE_KTRACE
#define WM_T(slot)                          \
  do {                                      \
    const unsigned long long n_ = clock64(); \
    kt[slot] += n_ - kt0;                   \
    kt0 = n_;                               \
  } while (0)
#else
#define WM_T(slot) \
  do {             \
  } while (0)
#endif
typedef double wf64x4 __attribute__((ext_vector_type(4)));
template <int NB>
constexpr int wm_ntiles() { return NB * (NB + 1) / 2 + NB; }
__host__ __device__ constexpr int wm_lt_doubles(int NB) { return (NB * (NB - 1) / 2) * 256; }
template <int NB>
__device__ __forceinline__ int wm_lt(int I, int J) { return (I * (I - 1) / 2 + J) * 256; }  // I > J, I < NB
__device__ __forceinline__ int wm_pk(int i, int j) { return i * (i + 1) / 2 + j; }          // j <= i < 16
// packed lower triangle, column-major: column k holds rows k..15 contiguously (lane-contiguous reads)
__device__ __forceinline__ int wm_ck(int i, int k) { return 16 * k - k * (k - 1) / 2 + (i - k); }  // k <= i

// the staged factors (two buffers of kWrmfStage rows, fp32, with their weights) share the region of
// the off-diagonal factor tiles: accumulation and factorization never overlap within a row
__host__ __device__ constexpr int wm_stage_floats(int NB) { return kWrmfStage * 16 * NB + 2 * kWrmfStage; }
__host__ __device__ constexpr int wm_region_doubles(int NB) {
  return wm_lt_doubles(NB) > wm_stage_floats(NB) ? wm_lt_doubles(NB) : wm_stage_floats(NB);  // >= 2 buffers
}
template <int NB>
size_t wm_lds_bytes() {
  return sizeof(double) * ((size_t)wm_region_doubles(NB) + 136 * NB + 16 * NB + 16 * NB + 16 + 16);
}

template <int NB>
__global__ __launch_bounds__(256, 2) void k_wrmf_solve_mfma(float* __restrict__ X, long n_rows,
                                                         const float* __restrict__ F, int dim,
                                                         const wacc_t* __restrict__ G,
                                                         const int64_t* __restrict__ indptr,
                                                         const int32_t* __restrict__ indices,
                                                         const float* __restrict__ values, float alpha,
                                                         float lambda, int phases, int min_pairs) {
  constexpr int D16 = 16 * NB, NT = wm_ntiles<NB>(), NS = (NT + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) double wsm[];
  double* Lt = wsm;                               // off-diagonal factor tiles [i][j]
  double* Li = Lt + wm_region_doubles(NB);        // diagonal factor inverses, packed lower
  double* ys = Li + 136 * NB;                     // y = L^{-1} b
  double* xs = ys + 16 * NB;                      // x
  double* rs = xs + 16 * NB;                      // back substitution: the block's right-hand side
  // staging buffer b: [kWrmfStage][D16] factors, then c_s - 1 and c_s (over Lt: see wm_stage_floats)
  float* const stb = reinterpret_cast<float*>(wsm);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform: tile coordinates in SGPRs)
  const int li = lane & 15, lk = lane >> 4;
  // this wave's tiles
  int TI[NS], TJ[NS];
#pragma unroll
  for (int sl = 0; sl < NS; ++sl) {
    const int tau = 4 * sl + wave;
    int I = -1, J = -1, base = 0;
    for (int j = 0; j < NB; ++j) {
      const int cnt = NB - j + 1;
      if (tau >= base && tau < base + cnt) {
        J = j;
        I = j + (tau - base);
      }
      base += cnt;
    }
    TI[sl] = tau < NT ? I : -1;
    TJ[sl] = tau < NT ? J : -1;
  }
#ifdef DCUE_KTRACE
  // per-phase cycles of one thread of wave 0 and of wave 1: 0 G, 1 accumulation, 2 diagonal blocks,
  // 3 barriers, 4 panels, 5 trailing, 6 back substitution + store, 7 rows
  unsigned long long kt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kt0 = clock64();
#endif
  for (long r = blockIdx.x; r < n_rows; r += gridDim.x) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    // (rows with at most min_pairs pairs are solved by k_wrmf_solve_lowrank -- unless a weight is
    // negative: its Woodbury system S = W^-1 + P F^T is then indefinite and unpivoted elimination
    // could meet a near-zero pivot, while A = G + lambda I + F^T W F may still be SPD; those come here)
    // (rows without pairs are zeroed below, also when k_wrmf_solve_lowrank is off: min_pairs 0)
    if (p1 > p0 && p1 - p0 <= min_pairs && !wrmf_row_has_negative(values, p0, p1, alpha)) continue;
    if (p1 <= p0) {  // no observed pair: b = 0, so x = 0
      for (int c = t; c < dim; c += blockDim.x) X[r * dim + c] = 0.f;
      continue;
    }
#ifdef DCUE_KTRACE
    ++kt[7];
#endif
    WM_T(6);
    // A = G + lambda I (identity on the padding); the augmented row b = 0
    wf64x4 acc[NS];
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      const int I = TI[sl], J = TJ[sl];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // (the load is unconditional, its use selected: a load under a branch would be waited for
        // at the branch's join, one tile at a time, instead of all of them in flight together)
        const int i = lk + 4 * q;
        const bool in = I >= 0 && I < NB;
        double v = G[(size_t)(16 * (in ? I : 0) + i) * D16 + 16 * (in ? J : 0) + li];
        if (I == J && i == li) v += 16 * I + i < dim ? (double)lambda : 1.0;
        acc[sl][q] = in ? v : 0.0;
      }
    }
    WM_T(0);
    // the row's observed factors, kWrmfStage at a time: K = 4 factors per MFMA. The next pass's
    // gather is in flight (registers) during this pass's MFMAs and lands in the other buffer after them
    constexpr int SD = kWrmfStage * D16, PER = (SD + 255) / 256;
    float pre[PER], wpre = 0.f;
    auto gather = [&](const long pb) {
      const int ns = (int)min((long)kWrmfStage, p1 - pb);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = t + 256 * u, sf = e / D16, c = e - sf * D16;
        pre[u] = e < SD && sf < ns && c < dim ? F[(long)indices[pb + sf] * dim + c] : 0.f;
      }
      if (t < kWrmfStage) wpre = t < ns ? alpha * (values ? values[pb + t] : 1.f) : 0.f;
      return ns;
    };
    auto put = [&](const int buf, const int ns) {
      float* st = stb + buf * wm_stage_floats(NB);
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (t + 256 * u < SD) st[t + 256 * u] = pre[u];
      if (t < kWrmfStage) {
        st[SD + t] = wpre;
        st[SD + kWrmfStage + t] = t < ns ? 1.f + wpre : 0.f;
      }
    };
    if ((phases & 1) && p1 > p0) {
      const int ns0 = gather(p0);
      __syncthreads();  // (the previous row's factorization and back substitution over this region)
      put(0, ns0);
    }
#pragma unroll 1
    for (long pb = p0, buf = 0; pb < ((phases & 1) ? p1 : p0); pb += kWrmfStage, buf ^= 1) {
      __syncthreads();  // (buffer buf written; every wave done with the other one)
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) asm volatile("" : "+s"(TI[sl]), "+s"(TJ[sl]));  // (as below)
      const bool more = pb + kWrmfStage < p1;
      int ns1 = 0;
      if (more) ns1 = gather(pb + kWrmfStage);
      const float* st = stb + buf * wm_stage_floats(NB);
      const float* ws = st + SD;
      const float* cs = ws + kWrmfStage;
      // operands one MFMA ahead: (kk, sl)'s loads are issued before the MFMA of the step before it
      float na, nb;
      auto ld = [&](const int kk, const int sl) {
        const int sf = 4 * kk + lk, I = TI[sl], J = TJ[sl];
        na = st[sf * D16 + 16 * (I < NB && I >= 0 ? I : 0) + li];
        nb = st[sf * D16 + 16 * (J >= 0 ? J : 0) + li];
      };
      ld(0, 0);
#pragma unroll
      for (int kk = 0; kk < kWrmfStage / 4; ++kk) {
        const int sf = 4 * kk + lk;
        const double w = (double)ws[sf], c = (double)cs[sf];
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
          const int I = TI[sl];
          const float ca = na, cb = nb;
          if (sl + 1 < NS) ld(kk, sl + 1);
          else if (kk + 1 < kWrmfStage / 4) ld(kk + 1, 0);
          if (I >= 0) {
            const double a = I == NB ? (li == 0 ? c : 0.0) : w * (double)ca;
            acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (double)cb, acc[sl], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);  // (one step of loads in flight: register budget)
        }
      }
      if (more) put(buf ^ 1, ns1);
    }
    WM_T(1);
    // block Cholesky
    // (a) + (b) for diagonal block kb
    auto factor_diag = [&](const int kb) {
      // (a) the diagonal tile to Li[kb] (packed lower)
#pragma unroll
      for (int sl = 0; sl < NS; ++sl)
        if (TI[sl] == kb && TJ[sl] == kb) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = lk + 4 * q;
            if (li <= i) Li[136 * kb + wm_pk(i, li)] = acc[sl][q];
          }
        }
      __syncthreads();
      // (b) wave 0: factor it and invert the factor in one pass, in registers. Lane j < 16 holds row j
      // of A, lane 16 + j column j of X (= I at the start; lanes 32-63 repeat them, unused). Step k
      // scales every lane's element k by 1 / L[k][k] -- row k's pivot becomes L[k][k], rows below
      // their L[j][k], and X's row k is divided by L[k][k] -- then broadcasts L[c][k] (c > k) through
      // SGPRs and each lane applies R[c] -= L[c][k] R[k]: A's trailing update (lanes j < 16, whose
      // upper-triangle elements take harmless garbage) and X's forward substitution (X ends as
      // L_kk^{-1}) in the same instructions, without LDS round trips or divergence
      if (wave == 0 && (phases & 8)) {
        double* Lk = Li + 136 * kb;
        const int j = lane & 15;
        const bool xl = lane >= 16;
        double R[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) R[c] = xl ? (c == j ? 1.0 : 0.0) : (c <= j ? Lk[wm_pk(j, c)] : 0.0);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const double inv = rsqrt_d(readlane_d(R[k], k));
          R[k] *= inv;
#pragma unroll
          for (int c = k + 1; c < 16; ++c) R[c] = fma(-readlane_d(R[k], c), R[k], R[c]);
        }
        // L_kk^{-1} over the block's slot, packed column-major (its A_kk input was read above)
        if (xl && lane < 32) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (i >= j) Lk[wm_ck(i, j)] = R[i];
        }
      }
      WM_T(2);
    };
    auto trailing = [&](const int kb) {
      // (d) trailing: A_IJ -= L_Ikb L_Jkb^T for kb < J <= I
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        const int I = TI[sl], J = TJ[sl];
        if (J <= kb || I < 0 || !(phases & 32)) continue;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * kk + lk;
          // (operand addresses selected, the loads themselves unconditional: see the G loads)
          const double ra = *(I < NB ? Lt + wm_lt<NB>(I, kb) + k * 16 + li : ys + 16 * kb + k);
          const double a = I < NB || li == 0 ? ra : 0.0;
          const double b = Lt[wm_lt<NB>(J, kb) + k * 16 + li];  // L_Jkb^T[k][j] = L_Jkb[j][k]
          acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(-a, b, acc[sl], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      WM_T(5);
    };
#pragma unroll 1
    for (int kb = 0; kb < NB; ++kb) {
      // tile coordinates opaque per step: their address arithmetic is redone here instead of being
      // hoisted out of the step loop into live registers
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) asm volatile("" : "+s"(TI[sl]), "+s"(TJ[sl]));
      __syncthreads();  // (the previous block's trailing reads of Lt; the first: the staging reads)
      WM_T(3);
      factor_diag(kb);
      __syncthreads();  // (L_kk^{-1} in Li[kb])
      WM_T(3);
      // (c) panel: L_Ikb = A_Ikb L_kk^{-T}. A_Ikb goes through its own LDS slot (ys for the augmented
      // row) into the MFMA A layout and L_Ikb comes back over it -- all within the owning wave, whose
      // LDS accesses run in order: no barrier until the trailing update reads other waves' tiles
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        const int I = TI[sl];
        if (TJ[sl] != kb || I <= kb) continue;
        if (I < NB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) Lt[wm_lt<NB>(I, kb) + li * 16 + lk + 4 * q] = acc[sl][q];
        } else if (lk == 0) {
          ys[16 * kb + li] = acc[sl][0];
        }
        if (phases & 16) {
          wf64x4 d = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = 4 * kk + lk;
            const double ra = *(I < NB ? Lt + wm_lt<NB>(I, kb) + k * 16 + li : ys + 16 * kb + k);
            const double a = I < NB || li == 0 ? ra : 0.0;
            const double rb = Li[136 * kb + wm_ck(k <= li ? li : k, k)];
            const double b = k <= li ? rb : 0.0;  // L^{-T}[k][j] = L^{-1}[j][k]
            d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
          }
          acc[sl] = d;
        }
        if (I < NB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) Lt[wm_lt<NB>(I, kb) + li * 16 + lk + 4 * q] = acc[sl][q];
        } else if (lk == 0) {
          ys[16 * kb + li] = acc[sl][0];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      WM_T(4);
      __syncthreads();
      WM_T(3);
      trailing(kb);
    }
    __syncthreads();
    WM_T(3);
    // L^T x = y, block rows NB-1 .. 0, wave 0: lane (m, q) = (lane & 15, lane >> 4) sums a quarter
    // of each dot product, the quarters meet by shuffles
    if (wave == 0 && (phases & 4)) {
#pragma unroll 1
      for (int I = NB - 1; I >= 0; --I) {
        // r_I[m] = y_I[m] - sum_{J > I} sum_n L_JI[n][m] x_J[n]
        double part = 0.0;
#pragma unroll 1
        for (int J = I + 1; J < NB; ++J) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int n = 4 * lk + u;
            part = fma(Lt[wm_lt<NB>(J, I) + li * 16 + n], xs[16 * J + n], part);
          }
        }
        part += __shfl_xor(part, 16, 64);
        part += __shfl_xor(part, 32, 64);
        if (lane < 16) rs[li] = ys[16 * I + li] - part;
        // x_I[i] = sum_{m >= i} L_II^{-1}[m][i] r[m]
        double xp = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = 4 * lk + u;
          if (m >= li) xp = fma(Li[136 * I + wm_ck(m, li)], rs[m], xp);
        }
        xp += __shfl_xor(xp, 16, 64);
        xp += __shfl_xor(xp, 32, 64);
        if (lane < 16) xs[16 * I + li] = xp;
      }
      for (int c = lane; c < dim; c += 64) X[r * dim + c] = (float)xs[c];
    }
  }
#ifdef DCUE_KTRACE
  WM_T(6);
  if ((t == 0 || t == 64) && blockIdx.x < kKtraceBlocks)
    for (int k = 0; k < 8; ++k) dcue_ktrace_buf[t >> 6][blockIdx.x][k] = kt[k];
#endif
}

// ---- rows with few pairs: the Woodbury identity -------------------------------------------------
// With M = (G + lambda I)^{-1} (the same for every row of the half-step, k_wrmf_ginv) and the row's
// n pairs F_r (n x d), weights w_s = c_s - 1:
//   A_r = M^{-1} + F_r^T W F_r,  A_r^{-1} = M - P^T (W^{-1} + P F_r^T)^{-1} P,  P = F_r M,
//   x_r = A_r^{-1} F_r^T c = P^T (c - u),  S u = P b,  S = W^{-1} + P F_r^T,  b = F_r^T c,
// an n x n system instead of d x d: its serial chain is n pivots, not d. Pairs with w_s = 0 (c_s = 1)
// add nothing to A_r: their rows of S become the identity and their u_s = 0. fp64 throughout.
// k_wrmf_ginv: M by in-place Gauss-Jordan inversion of G + lambda I (SPD: no pivoting) in one
// workgroup's LDS (128 KB at d = 128).
__global__ __launch_bounds__(1024) void k_wrmf_ginv(const wacc_t* __restrict__ G, int dim, float lambda,
                                                    wacc_t* __restrict__ M) {
  const int D = (dim + 15) & ~15, t = threadIdx.x;
  extern __shared__ __attribute__((aligned(16))) double ga[];  // [D][D]
  __shared__ double fcol[kWrmfMaxDim], prow[kWrmfMaxDim];
  for (int e = t; e < D * D; e += blockDim.x) {
    const int i = e / D, j = e - i * D;
    ga[e] = G[e] + (i == j ? (i < dim ? (double)lambda : 1.0) : 0.0);
  }
  for (int k = 0; k < D; ++k) {
    __syncthreads();
    const double p = 1.0 / ga[k * D + k];
    if (t < D) {
      fcol[t] = ga[t * D + k];
      prow[t] = (t == k ? 1.0 : ga[k * D + t]) * p;  // row k / pivot, its pivot entry 1 / pivot
    }
    __syncthreads();
    const int j = t & 127;  // (column t % 128, rows t / 128 + 8 q: no division in the step)
    if (j < D) {
      const double pj = prow[j];
      for (int i = t >> 7; i < D; i += 8) {
        double* e = ga + i * D + j;
        *e = i == k ? pj : fma(-fcol[i], pj, j == k ? 0.0 : *e);
      }
    }
  }
  __syncthreads();
  for (int e = t; e < D * D; e += blockDim.x) M[e] = ga[e];
}

// One workgroup per row with 1 <= n <= 16 NR pairs (rows with none: x = 0; the rest are left to
// k_wrmf_solve_mfma). LDS: P [16 NR][D16 + 2] fp64 (pitch: conflict-free column reads), F_r
// [16 NR][D16] fp32 (S [16 NR][16 NR + 1] fp64 over it once P F_r^T is in registers), c, w, b, P b, u.
template <int NB, int NR>
constexpr size_t wl_lds_bytes() {
  constexpr int D16 = 16 * NB, NP = 16 * NR;
  constexpr size_t f = sizeof(float) * NP * D16, sb = sizeof(double) * NP * (NP + 1);
  return sizeof(double) * ((size_t)NP * (D16 + 2) + 4 * NP + D16 + 2 * 64 + 2) + (f > sb ? f : sb);
}
template <int NB, int NR>
__global__ __launch_bounds__(256) void k_wrmf_solve_lowrank(float* __restrict__ X, long n_rows,
                                                           const float* __restrict__ F, int dim,
                                                           const wacc_t* __restrict__ M,
                                                           const int64_t* __restrict__ indptr,
                                                           const int32_t* __restrict__ indices,
                                                           const float* __restrict__ values, float alpha) {
  constexpr int D16 = 16 * NB, NP = 16 * NR, PP = D16 + 2, SP = NP + 1;
  extern __shared__ __attribute__((aligned(16))) double lsm[];
  double* Ps = lsm;                 // [NP][PP]
  double* cs = Ps + NP * PP;        // c_s
  double* ws = cs + NP;             // w_s = c_s - 1
  double* rh = ws + NP;             // (P b)_s
  double* us = rh + NP;             // u_s
  double* bs = us + NP;             // b = F_r^T c
  double* gb = bs + D16;            // Gauss-Jordan: [2][64] row multiples, [2] pivot inverses
  float* Fs = reinterpret_cast<float*>(gb + 2 * 64 + 2);  // [NP][D16]
  double* Ss = reinterpret_cast<double*>(Fs);      // [NP][SP], after P F_r^T
  const int t = threadIdx.x, lane = t & 63, li = lane & 15, lk = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
#ifdef DCUE_KTRACE
  // per-phase cycles (threads 0 and 64): 0 staging, 1 P, 2 b + S + P b, 3 S store, 4 Gauss-Jordan,
  // 5 x, 6 the skipped rows' checks, 7 rows
  unsigned long long kt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kt0 = clock64();
#endif
  for (long r = blockIdx.x; r < n_rows; r += gridDim.x) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    const int n = (int)(p1 - p0);
    if (n > NP) continue;
    if (wrmf_row_has_negative(values, p0, p1, alpha)) continue;  // (k_wrmf_solve_mfma's, see there)
    if (n <= 0) {
      for (int c = t; c < dim; c += blockDim.x) X[r * dim + c] = 0.f;
      continue;
    }
    WM_T(6);
#ifdef DCUE_KTRACE
    ++kt[7];
#endif
    __syncthreads();  // (the previous row's reads)
    for (int e = t; e < NP * D16; e += blockDim.x) {
      const int sf = e / D16, c = e - sf * D16;
      Fs[e] = sf < n && c < dim ? F[(long)indices[p0 + sf] * dim + c] : 0.f;
    }
    if (t < NP) {
      const double w = t < n ? (double)(alpha * (values ? values[p0 + t] : 1.f)) : 0.0;
      ws[t] = w;
      cs[t] = t < n ? 1.0 + w : 0.0;
    }
    __syncthreads();
    WM_T(0);
    // P = F_r M: 16 x 16 tiles (RI, CJ), RI over the pairs' row tiles, K = D16, B straight from M
    const int nr = (n + 15) >> 4;
    for (int q = wave; q < nr * NB; q += 4) {
      const int RI = q / NB, CJ = q - RI * NB;
      wf64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < D16 / 4; ++kk) {
        const double a = (double)Fs[(16 * RI + li) * D16 + 4 * kk + lk];
        const double b = M[(size_t)(4 * kk + lk) * D16 + 16 * CJ + li];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) Ps[(16 * RI + lk + 4 * e) * PP + 16 * CJ + li] = acc[e];
    }
    WM_T(1);
    // b = F_r^T c
    for (int c = t; c < D16; c += blockDim.x) {
      double v = 0.0;
      for (int sf = 0; sf < n; ++sf) v = fma(cs[sf], (double)Fs[sf * D16 + c], v);
      bs[c] = v;
    }
    __syncthreads();
    // S = P F_r^T: tiles (RI, RJ), one per wave (nr <= 2) or strided; in registers until every
    // wave is done with F_r, then over it
    wf64x4 sacc[(NR * NR + 3) / 4];
#pragma unroll
    for (int m = 0; m < (NR * NR + 3) / 4; ++m) {
      sacc[m] = wf64x4{0.0, 0.0, 0.0, 0.0};
      const int q = wave + 4 * m, RI = q / NR, RJ = q - RI * NR;
      if (q < NR * NR && RI < nr && RJ < nr) {
#pragma unroll
        for (int kk = 0; kk < D16 / 4; ++kk) {
          const double a = Ps[(16 * RI + li) * PP + 4 * kk + lk];
          const double b = (double)Fs[(16 * RJ + li) * D16 + 4 * kk + lk];
          sacc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, sacc[m], 0, 0, 0);
        }
      }
    }
    // (P b)_s: eight lanes per pair
    {
      const int sf = t >> 3, part = t & 7;
      double v = 0.0;
      if (sf < NP)
        for (int c = part; c < D16; c += 8) v = fma(Ps[sf * PP + c], bs[c], v);
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (sf < NP && part == 0) rh[sf] = sf < n && ws[sf] != 0.0 ? v : 0.0;
    }
    __syncthreads();  // (F_r's last reads)
    WM_T(2);
#pragma unroll
    for (int m = 0; m < (NR * NR + 3) / 4; ++m) {
      const int q = wave + 4 * m, RI = q / NR, RJ = q - RI * NR;
      if (q < NR * NR) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 16 * RI + lk + 4 * e, j = 16 * RJ + li;
          // rows of pairs without weight and the padding: the identity (their u = 0)
          const bool live = i < n && j < n && ws[i] != 0.0 && ws[j] != 0.0;
          Ss[i * SP + j] = live ? sacc[m][e] + (i == j ? 1.0 / ws[i] : 0.0) : (i == j ? 1.0 : 0.0);
        }
      }
    }
    __syncthreads();
    WM_T(3);
    // S u = P b by Gauss-Jordan over all four waves: lane j holds row j, wave w columns
    // CW w .. CW w + CW - 1 of [S | P b]. Step k: the pivot column's wave sends every row's multiple
    // S[j][k] / S[k][k] through LDS (double-buffered: one barrier per step); each wave then takes
    // row k of its columns by v_readlane and updates R[c] -= g_j S[k][c] (row k: divided by the
    // pivot). Columns already eliminated take the update unchanged (their row-k entry is 0).
    {
      constexpr int CW = (NP + 1 + 3) / 4;
      const int j = lane < NP ? lane : NP - 1;
      double R[CW];
#pragma unroll
      for (int i = 0; i < CW; ++i) {
        const int c = CW * wave + i;
        R[i] = c < NP ? Ss[j * SP + c] : (c == NP ? rh[j] : 0.0);
      }
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        double* g2 = gb + (k & 1) * 64;
        if (wave == k / CW) {
          const double piv = readlane_d(R[k % CW], k);
          const double inv = 1.0 / piv;
          g2[lane] = lane == k ? 0.0 : R[k % CW] * inv;
          if (lane == 0) gb[128 + (k & 1)] = inv;
        }
        __syncthreads();
        const double g = g2[lane], inv = gb[128 + (k & 1)];
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          const double pk = readlane_d(R[i], k);
          R[i] = lane == k ? pk * inv : fma(-g, pk, R[i]);
        }
      }
      if (wave == NP / CW && lane < NP) us[lane] = R[NP % CW];
    }
    __syncthreads();
    WM_T(4);
    // x = P^T (c - u)
    for (int c = t; c < dim; c += blockDim.x) {
      double v = 0.0;
      for (int sf = 0; sf < n; ++sf) v = fma(Ps[sf * PP + c], cs[sf] - us[sf], v);
      X[r * dim + c] = (float)v;
    }
    WM_T(5);
  }
#ifdef DCUE_KTRACE
  WM_T(6);
  if ((t == 0 || t == 64) && blockIdx.x < kKtraceBlocks)
    for (int q = 0; q < 8; ++q) dcue_ktrace_buf[2 + (t >> 6)][blockIdx.x][q] = kt[q];
#endif
}

template <int NB>
static int launch_wrmf_mfma(float* solve, long n_rows, const float* fixed, int dim, const wacc_t* G,
                            const int64_t* indptr, const int32_t* indices, const float* values, float alpha,
                            float lambda, const wacc_t* M, hipStream_t s) {
  // rows with at most 32 pairs by the Woodbury identity (M = (G + lambda I)^{-1}; DCUE_WRMF_LOWRANK=0:
  // every row by the Cholesky)
  constexpr int kLowNR = 2;
  const int min_pairs = M ? 16 * kLowNR : 0;
  if (M) {
    const size_t llds = wl_lds_bytes<NB, kLowNR>();
    auto lk = k_wrmf_solve_lowrank<NB, kLowNR>;
    DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)lk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)llds));
    const long lgrid = n_rows < 8192 ? n_rows : 8192;
    DCUE_LAUNCH(lk, dim3((unsigned)lgrid), dim3(256), llds, s, solve, n_rows, fixed, dim, M, indptr, indices,
                values, alpha);
    DCUE_LAUNCH_CHECK();
  }
  static const int phases = [] {  // (DCUE_WRMF_PHASES: see dcue_wrmf_half_step; + 64: the inverse)
    const char* e = getenv("DCUE_WRMF_PHASES");
    return e ? atoi(e) : 127;
  }();
  const size_t lds = wm_lds_bytes<NB>();
  auto kern = k_wrmf_solve_mfma<NB>;
  DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const long grid = n_rows < 4096 ? n_rows : 4096;
  DCUE_LAUNCH(kern, dim3((unsigned)grid), dim3(256), lds, s, solve, n_rows, fixed, dim, G, indptr, indices, values,
              alpha, lambda, phases, min_pairs);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

size_t wrmf_solve_lds_bytes() {
  return sizeof(wacc_t) * ((size_t)kWrmfTri + kWrmfMaxDim) + sizeof(float) * ((size_t)kWrmfStage * kWrmfMaxDim + kWrmfStage);
}

// gram workgroups (= partial sets): one per 512-row chunk, at most kWrmfGramMaxBlocks
long wrmf_gram_chunks(long n_fixed) {
  const long c = (n_fixed + kWrmfGramChunk - 1) / kWrmfGramChunk;
  return c < kWrmfGramMaxBlocks ? c : kWrmfGramMaxBlocks;
}

}  // namespace dcue

extern "C" {

int dcue_wrmf_workspace_bytes(int32_t dim, int64_t n_fixed, size_t* bytes_host) {
  if (!bytes_host || dim <= 0 || dim > dcue::kWrmfMaxDim || n_fixed < 0) return DCUE_ERR_INVALID;
  const long nch = dcue::wrmf_gram_chunks(n_fixed < 1 ? 1 : n_fixed);
  const size_t d16 = (size_t)((dim + 15) & ~15);
  // partials, G, and the Woodbury path's inverse M
  *bytes_host = sizeof(dcue::wacc_t) * ((size_t)nch * dim * dim + 2 * d16 * d16) + 256;
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
  static const bool scalar_gram = [] {  // DCUE_WRMF_GRAM=scalar: k_wrmf_gram (fp64 FMAs), A/B and check
    const char* e = getenv("DCUE_WRMF_GRAM");
    return e && e[0] == 's';
  }();
  if (scalar_gram)
    DCUE_LAUNCH(k_wrmf_gram, dim3((unsigned)nch), dim3(256), 0, s, fixed, (long)n_fixed, (int)dim, part);
  else
    DCUE_LAUNCH(k_wrmf_gram_mfma, dim3((unsigned)nch), dim3(256), 0, s, fixed, (long)n_fixed, (int)dim, part);
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
  // the fp64-MFMA block Cholesky (k_wrmf_solve_mfma) by default: 45 ms per ALS iteration against
  // 90 for the register-tile solve (DCUE_WRMF_SOLVE=tile) at the bench's shape
  static const bool tile_solve = [] {
    const char* e = getenv("DCUE_WRMF_SOLVE");
    return e && e[0] == 't';
  }();
  if (!tile_solve) {
    static const bool lowrank = [] {
      const char* e = getenv("DCUE_WRMF_LOWRANK");
      return !(e && e[0] == '0');
    }();
    wacc_t* M = nullptr;
    if (lowrank) {
      const size_t d16 = (size_t)((dim + 15) & ~15);
      M = G + d16 * d16;
      const size_t glds = sizeof(wacc_t) * d16 * d16;
      DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)k_wrmf_ginv, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)glds));
      DCUE_LAUNCH(k_wrmf_ginv, dim3(1), dim3(1024), glds, s, G, (int)dim, lambda, M);
      DCUE_LAUNCH_CHECK();
    }
    switch ((dim + 15) / 16) {
      case 1: return launch_wrmf_mfma<1>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 2: return launch_wrmf_mfma<2>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 3: return launch_wrmf_mfma<3>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 4: return launch_wrmf_mfma<4>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 5: return launch_wrmf_mfma<5>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 6: return launch_wrmf_mfma<6>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      case 7: return launch_wrmf_mfma<7>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
      default: return launch_wrmf_mfma<8>(solve, (long)n_rows, fixed, dim, G, indptr, indices, values, alpha, lambda, M, s);
    }
  }
  // DCUE_WRMF_PHASES (timing diagnostic, wrong results): bit 1 the accumulation, 2 the Cholesky,
  // 4 the back substitution, 8 / 16 / 32 the Cholesky's diagonal blocks / panels / trailing
  // updates (default 63: all)
  static const int phases = [] {
    const char* e = getenv("DCUE_WRMF_PHASES");
    return e ? atoi(e) : 63;
  }();
  DCUE_LAUNCH(k_wrmf_solve, dim3((unsigned)grid), dim3(256), lds, s, solve, (long)n_rows, fixed, (int)dim, G,
              indptr, indices, values, alpha, lambda, phases);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // extern "C"
