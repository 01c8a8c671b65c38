// Text branch of the mixed audio + text item tower (BASELINE config 4: "DCUE + language-model-pretrained
// text tower (bio/lyrics), d=256, mixed audio+text item encoder") -- gfx950.
//
// The reference never published this path: its text item set imports a `WordEmbeddings` module
// that does not exist (reference datasets/dcuelmitemset.py:8), so only the data contract is pinned
// by the reference: one sentence of token ids per track, BOS + sentence + EOS, cut to
// max_sentence_length + 1 and right-padded with PAD (dcuelmitemset.py:40-56). The encoder is this
// build's choice, parity-unpinned against the reference and pinned against
// oracle/text_oracle.py (torch-CPU):
//
//   e[i][t]   = words[tokens[track_i][t]]                    frozen word vectors [V][E] (the
//                                                            LM-pretrained part, caller supplied)
//   z[i][t]   = Conv1d(E -> C, k = 3, pad = 1)(e[i])[t]      text.conv.{weight [C][E][3], bias [C]}
//   s[i][o]   = relu(max over t with tokens[t] != PAD of z[i][t][o])
//   f[i]      = fc([s[i] ; bn5(y5[i])])                      conv.fc: Linear(C + d -> d)
//
// Kernels:
//   k_text_fwd     the conv as a row-GEMM on split-f16 MFMA (v_mfma_f32_16x16x32_f16, three per f32
//                  product as the audio forwards, conv_rows.h): a workgroup owns IPW items x 64 output
//                  channels, 4 waves x 16 channels over all of the items' T positions; the items' word
//                  vectors are gathered 32 channels at a time into LDS (hi/lo halves, register-
//                  prefetched one chunk ahead), the B operand (the packed split-f16 text weights) comes
//                  from L2. The epilogue adds the bias, takes the masked max over t in registers and
//                  across the wave's four row groups, applies the ReLU and writes s into the fc input
//                  xfc[:, :C] plus the argmax position (255: no gradient) for the backward.
//   k_text_wgrad   dW[o][c][k] = sum_i g[i][o] e[i][t*(i,o) + k - 1][c] -- the max routes each (item,
//                  channel) gradient to one position, so the weight gradient is a gathered sum, not a
//                  dense GEMM over positions (3 x C x E FMAs per item instead of 3 x C x E x T). A
//                  workgroup owns 8 output channels x 32 word channels over all of its chunk's items,
//                  3 fp32 accumulators per thread, exact fp32 FMAs in item order (deterministic);
//                  db[o] = sum_i g[i][o] in item order.
//   k_text_wreduce the chunk partials in chunk order (only when M needs more than one chunk).
#include <cstring>

#include "dcue_internal.h"

DCUE_KTRACE_READER(text)  // diagnostic builds only (dcue_common.h): kernel 0 = k_text_fwd_full

namespace dcue {

typedef _Float16 t16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 t16x4 __attribute__((ext_vector_type(4)));

constexpr int kTextKC = 32;        // word channels per K chunk (one MFMA k-step)
constexpr int kTextRowH = 72;      // LDS row: [hi x 32][lo x 32][pad x 8] halves = 144 B (conflict-free)
constexpr int kTextNoGrad = 255;   // argmax code: no gradient (ReLU off, or no valid position)

struct TextFwdArgs {
  const int32_t* tokens;      // [n_tracks][T]
  const int32_t* item_track;  // [M]
  const float* words;         // [V][E]
  float xscale, inv_xscale;   // 2^words_exp and its inverse (exact): the word values' split-f16 scale
  const uint4* wpack;         // [3 * EP/32][C][4][hi x 8, lo x 8] halves (uint4 = 8 halves)
  const float* bias;          // [C]
  int M, T, E, EP, C, Creal, pad;
  float* out;                 // s[i][o] at out[i * ld + o], o < Creal
  long ld;
  uint8_t* tidx;              // [M][C]
  int nxcd;                   // k_text_fwd_full: XCDs its work units run on (8 or 4)
  unsigned* ticket;           // k_text_fwd_full with position parts: [M][column blocks], zero
  unsigned long long* part;   // [M][parts][C]
};

// Split f32 -> (hi, lo) fp16 halves: hi = fp16(v), lo = fp16(v - hi) (v - hi is exact in f32).
__device__ __forceinline__ void split4(const float4& v, _Float16* hi, _Float16* lo) {
  const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const _Float16 h = (_Float16)a[q];
    hi[q] = h;
    lo[q] = (_Float16)(a[q] - (float)h);
  }
}

template <int TB, int IPW>
__global__ __launch_bounds__(256) void k_text_fwd(TextFwdArgs a) {
  constexpr int TP = TB * 16;       // conv positions computed per item (T rounded up)
  constexpr int RS = TP + 2;        // staged rows per item: token positions -1 .. TP
  constexpr int NROW = IPW * RS;
  constexpr int PASSES = (NROW * (kTextKC / 4) + 255) / 256;
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][NROW * kTextRowH];
  __shared__ int32_t tok[NROW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i0 = blockIdx.x * IPW;
  const int o0 = blockIdx.y * 64 + wv * 16;
  // the items' token rows (row r' = position r' - 1; -1 outside the sentence or the batch)
  for (int r = tid; r < NROW; r += 256) {
    const int s = r / RS, t = r - s * RS - 1;
    const int i = i0 + s;
    tok[r] = (i < a.M && t >= 0 && t < a.T) ? a.tokens[(long)a.item_track[i] * a.T + t] : -1;
  }
  __syncthreads();
  const int nchunk = a.EP / kTextKC;
  float4 pre[PASSES];
  auto load_chunk = [&](int cb) {
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      const int e = tid + 256 * p;
      const int r = e >> 3, q = e & 7;
      const int c = cb * kTextKC + 4 * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < NROW && c < a.E) {
        const int tk = tok[r];
        if (tk >= 0) v = *reinterpret_cast<const float4*>(a.words + (long)tk * a.E + c);
      }
      pre[p] = v;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      const int e = tid + 256 * p;
      const int r = e >> 3, q = e & 7;
      if (r < NROW) {
        float4 v = pre[p];
        v.x *= a.xscale; v.y *= a.xscale; v.z *= a.xscale; v.w *= a.xscale;  // exact (power of two)
        _Float16 hi[4], lo[4];
        split4(v, hi, lo);
        _Float16* row = &xs[buf][r * kTextRowH];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          row[4 * q + j] = hi[j];
          row[kTextKC + 4 * q + j] = lo[j];
        }
      }
    }
  };
  f32x4 acc[IPW][TB];
#pragma unroll
  for (int s = 0; s < IPW; ++s)
#pragma unroll
    for (int b = 0; b < TB; ++b) acc[s][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  const int col = o0 + (lane & 15), g = lane >> 4;
  for (int cb = 0; cb < nchunk; ++cb) {
    if (cb + 1 < nchunk) load_chunk(cb + 1);  // in flight under this chunk's MFMAs
    const _Float16* xb = xs[cb & 1];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const long q = (long)k * nchunk + cb;
      const uint4* wp = a.wpack + ((q * a.C + col) * 4 + g) * 2;
      const uint4 wh = wp[0], wl = wp[1];
      const t16x8 bh = *reinterpret_cast<const t16x8*>(&wh);
      const t16x8 bl = *reinterpret_cast<const t16x8*>(&wl);
#pragma unroll
      for (int s = 0; s < IPW; ++s)
#pragma unroll
        for (int b = 0; b < TB; ++b) {
          // conv row t = 16b + (lane & 15) reads token t + k - 1 = staged row t + k
          const _Float16* rp = xb + (s * RS + 16 * b + (lane & 15) + k) * kTextRowH + 8 * g;
          const t16x8 ah = *reinterpret_cast<const t16x8*>(rp);
          const t16x8 al = *reinterpret_cast<const t16x8*>(rp + kTextKC);
          acc[s][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[s][b], 0, 0, 0);
          acc[s][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[s][b], 0, 0, 0);
          acc[s][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[s][b], 0, 0, 0);
        }
    }
    if (cb + 1 < nchunk) store_chunk((cb + 1) & 1);
    __syncthreads();
  }
  // epilogue: bias, masked first-max over the positions, ReLU
  const float bo = a.bias[col];
#pragma unroll
  for (int s = 0; s < IPW; ++s) {
    const int i = i0 + s;
    float best = -INFINITY;
    int bi = kTextNoGrad;
#pragma unroll
    for (int b = 0; b < TB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = 16 * b + 4 * g + j;
        const int tk = tok[s * RS + t + 1];
        const float v = acc[s][b][j] * a.inv_xscale + bo;
        if (t < a.T && tk >= 0 && tk != a.pad && v > best) {
          best = v;
          bi = t;
        }
      }
    // the four row groups of this column: larger value, the earlier position on a tie
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ob = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (g == 0 && i < a.M) {
      const bool on = best > 0.f;
      if (col < a.Creal) a.out[(long)i * a.ld + col] = on ? best : 0.f;
      a.tidx[(long)i * a.C + col] = (uint8_t)(on ? bi : kTextNoGrad);
    }
  }
}

// The same conv with each workgroup's word vectors gathered once: a workgroup owns ONE item and 16*WV
// output channels (WV waves of 16), and stages the item's whole sentence -- every position's full
// word vector, all EP channels, split into hi/lo fp16 halves -- in LDS with one burst of loads
// before the MFMAs (k_text_fwd above refills one 32-channel chunk at a time, a dependent global
// round trip per chunk, and its four 64-channel column blocks each re-gather the same vectors). The
// column blocks of an item sit next to each other in XCD order, so the second reads the vectors from
// the first's L2. The B operand is prefetched 3 or 6 (chunk, tap) steps ahead, the A fragments one. Per accumulator the
// MFMA sequence (chunk-major, then tap, then lo*hi, hi*lo, hi*hi) and the epilogue are k_text_fwd's:
// bit-identical output (DCUE_TEXT_FWD=chunked runs the old kernel: A/B and tests/test_gpu_text.py).
__host__ __device__ constexpr int text_full_pitch(int EP) {  // halves per staged row: [chunk][hi 32, lo 32] + pad
  return 2 * EP + 2 * (((36 - EP % 64) % 64 + 64) % 64);  // row pitch = 36 (mod 64) dwords: conflict-free
}

template <int TB, int WV, int NCT, int BPD, int NCH, int SPL>
__global__ __launch_bounds__(64 * WV) void k_text_fwd_full(TextFwdArgs a) {
  constexpr int TP = TB * 16;  // conv positions computed by this workgroup (its part of T)
  constexpr int RS = TP + 2;   // staged rows: token positions p0 - 1 .. p0 + TP
  constexpr int NT = 64 * WV;
  extern __shared__ __attribute__((aligned(16))) _Float16 xf[];  // [RS][pitch]
  __shared__ int32_t tok[RS], tneed[RS];
  __shared__ unsigned s_arrived;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cb = a.C / (16 * WV * NCT);  // column blocks per item
  // work unit L: item i, position part h (SPL parts of TP positions), column block cbk. The units run
  // on a.nxcd of the 8 XCDs (blocks are dealt to XCDs round-robin: block b on XCD b % 8), each XCD a
  // contiguous range of units, so the column blocks and parts of an item share an L2; blocks of the
  // other XCDs exit at once. Every XCD that runs units reads the whole weight operand into its own
  // L2 (not coherent across XCDs): 4 XCDs halve those fills for the same 128 CUs of work.
  const int xb = blockIdx.x & 7;
  if (xb >= a.nxcd) return;
  const int nunit = a.M * cb * SPL, per = (nunit + a.nxcd - 1) / a.nxcd;
  const int L = xb * per + (int)(blockIdx.x >> 3);
  if (L >= nunit) return;
  const int i = L / (cb * SPL);
  const int h = (L - i * cb * SPL) / cb;
  const int cbk = L - i * cb * SPL - h * cb;
  const int p0 = h * TP;
  const int o0 = cbk * 16 * WV * NCT + wv * 16 * NCT;  // the wave's NCT column tiles
  const int pitch = text_full_pitch(a.EP);
  // NCH > 0: the chunk count at compile time (the step loop unrolls whole: loop-carried prefetch
  // registers would be waited for at the loop's latch)
  const int nchunk = NCH > 0 ? NCH : a.EP / kTextKC;
  DCUE_KTW(0, 6);
  DCUE_KT(0, 0);
  const long trk = a.item_track[i];
  for (int r = tid; r < RS; r += NT) {
    const int t = p0 + r - 1;
    tok[r] = (t >= 0 && t < a.T) ? a.tokens[trk * a.T + t] : -1;
  }
  __syncthreads();
  // the rows the unmasked positions read: staged row r feeds the positions of rows r - 1 .. r + 1;
  // a row no unmasked position reads (PAD beyond the sentence's end) stays zero and is never loaded
  // -- masked positions' values are never used, and every PAD row is one hot line of the table
  for (int r = tid; r < RS; r += NT) {
    bool need = false;
#pragma unroll
    for (int d = -1; d <= 1; ++d) {
      const int x = r + d;
      need |= x >= 1 && x <= TP && tok[x] >= 0 && tok[x] != a.pad;
    }
    tneed[r] = need ? tok[r] : -1;
  }
  __syncthreads();
  // B operand of (chunk ch, tap k) for this lane's columns: step q = ch * 3 + k, pack index k * nchunk + ch.
  // Every load below is unconditional (indices clamped in range, unused results dropped): a load
  // under a branch makes the compiler wait for every load in flight at the join.
  const int col = o0 + (lane & 15), g = lane >> 4;
  const int nq = 3 * nchunk;  // a multiple of BPD (launcher)
  auto bload = [&](int q, uint4* h, uint4* l) {
    const int ch = q / 3, k = q - 3 * ch;
#pragma unroll
    for (int n = 0; n < NCT; ++n) {
      const uint4* wp = a.wpack + (((long)(k * nchunk + ch) * a.C + col + 16 * n) * 4 + g) * 2;
      h[n] = wp[0];
      l[n] = wp[1];
    }
  };
  uint4 bh[BPD][NCT], bl[BPD][NCT];
#pragma unroll
  for (int q = 0; q < BPD; ++q) bload(q, bh[q], bl[q]);
  DCUE_KT(0, 1);
  float bo[NCT];  // (the epilogue's bias, loaded now: off its dependency chain)
#pragma unroll
  for (int n = 0; n < NCT; ++n) bo[n] = a.bias[col + 16 * n];
  // The sentence: every row's word channels [32 c0, 32 c1), float4 slots gathered kB per thread per
  // pass into v (loads unconditional: clamped addresses, invalid slots zeroed at the store), then split
  // into the hi/lo halves in LDS.
  constexpr int kB = 8;
  struct Gather {
    float4 v[kB];
    unsigned ok;
  };
  auto gather_issue = [&](int c0, int c1, int base, Gather& G) {
    const int qn = (c1 - c0) * (kTextKC / 4), n = RS * qn;
    int tkj[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) tkj[j] = tneed[min((base + NT * j) / qn, RS - 1)];
    __builtin_amdgcn_sched_barrier(0);  // (the token reads back to back, then the loads)
    G.ok = 0;
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int e = base + NT * j;
      const int c = 4 * (c0 * (kTextKC / 4) + e - (e / qn) * qn);
      const bool valid = e < n && tkj[j] >= 0 && c < a.E;
      G.ok |= (unsigned)valid << j;
      G.v[j] = *reinterpret_cast<const float4*>(a.words + (valid ? (long)tkj[j] * a.E + c : 0L));
    }
  };
  auto gather_store = [&](int c0, int c1, int base, const Gather& G) {
    const int qn = (c1 - c0) * (kTextKC / 4), n = RS * qn;
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int e = base + NT * j;
      if (e < n) {
        const int r = e / qn, c = 4 * (c0 * (kTextKC / 4) + e - r * qn);
        float4 x = (G.ok >> j) & 1u ? G.v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        x.x *= a.xscale; x.y *= a.xscale; x.z *= a.xscale; x.w *= a.xscale;  // exact (power of two)
        _Float16 hi[4], lo[4];
        split4(x, hi, lo);
        _Float16* row = xf + (long)r * pitch + (c / kTextKC) * 2 * kTextKC + (c % kTextKC);
        *reinterpret_cast<t16x4*>(row) = t16x4{hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<t16x4*>(row + kTextKC) = t16x4{lo[0], lo[1], lo[2], lo[3]};
      }
    }
  };
  f32x4 acc[NCT][TB];
#pragma unroll
  for (int n = 0; n < NCT; ++n)
#pragma unroll
    for (int b = 0; b < TB; ++b) acc[n][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A fragments of step q (conv row t = 16b + (lane & 15) reads token t + k - 1 = staged row t + k),
  // read one step ahead of their MFMAs
  auto aload = [&](int q, t16x8* ah, t16x8* al) {
    const int ch = q / 3, k = q - 3 * ch;
#pragma unroll
    for (int b = 0; b < TB; ++b) {
      const _Float16* rp = xf + (long)(16 * b + (lane & 15) + k) * pitch + ch * 2 * kTextKC + 8 * g;
      ah[b] = *reinterpret_cast<const t16x8*>(rp);
      al[b] = *reinterpret_cast<const t16x8*>(rp + kTextKC);
    }
  };
  t16x8 ah[TB], al[TB];
  // step q: B from ring slot j (refilled for step q + BPD), A of step q + 1 read ahead unless `last`
  auto step = [&](int q, int j, bool last) {
    t16x8 wh[NCT], wl[NCT];
#pragma unroll
    for (int n = 0; n < NCT; ++n) {
      wh[n] = *reinterpret_cast<const t16x8*>(&bh[j][n]);
      wl[n] = *reinterpret_cast<const t16x8*>(&bl[j][n]);
    }
    bload(min(q + BPD, nq - 1), bh[j], bl[j]);
    t16x8 nh[TB], nl[TB];
    if (!last) aload(q + 1, nh, nl);
    __builtin_amdgcn_sched_barrier(0);  // (the loads stay ahead of this step's MFMAs)
#pragma unroll
    for (int b = 0; b < TB; ++b)
#pragma unroll
      for (int n = 0; n < NCT; ++n) {
        acc[n][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[b], wh[n], acc[n][b], 0, 0, 0);
        acc[n][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], wl[n], acc[n][b], 0, 0, 0);
        acc[n][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], wh[n], acc[n][b], 0, 0, 0);
      }
    if (!last) {
#pragma unroll
      for (int b = 0; b < TB; ++b) {
        ah[b] = nh[b];
        al[b] = nl[b];
      }
    }
  };
  for (int base = tid; base < RS * (a.EP / 4); base += NT * kB) {
    Gather g0;
    gather_issue(0, nchunk, base, g0);
    gather_store(0, nchunk, base, g0);
  }
  __syncthreads();
  DCUE_KT(0, 2);
  aload(0, ah, al);
  constexpr int kUnroll = NCH > 0 ? 3 * NCH / BPD : 1;
#pragma unroll kUnroll
  for (int q0 = 0; q0 < nq; q0 += BPD) {
#pragma unroll
    for (int j = 0; j < BPD; ++j) step(q0 + j, j, q0 + j + 1 == nq);
  }
  DCUE_KT(0, 3);
  // epilogue (k_text_fwd's): bias, masked first-max over the positions, ReLU
  float best[NCT];
  int bi[NCT];
#pragma unroll
  for (int n = 0; n < NCT; ++n) {
    best[n] = -INFINITY;
    bi[n] = kTextNoGrad;
#pragma unroll
    for (int b = 0; b < TB; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * b + 4 * g + j, t = p0 + r;
        const int tk = tok[r + 1];
        const float v = acc[n][b][j] * a.inv_xscale + bo[n];
        if (t < a.T && tk >= 0 && tk != a.pad && v > best[n]) {
          best[n] = v;
          bi[n] = t;
        }
      }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {  // the four row groups: larger value, earlier position on a tie
      const float ob = __shfl_xor(best[n], off, 64);
      const int oi = __shfl_xor(bi[n], off, 64);
      if (ob > best[n] || (ob == best[n] && oi < bi[n])) {
        best[n] = ob;
        bi[n] = oi;
      }
    }
  }
  if constexpr (SPL > 1) {
    // The parts' maxima meet in a.part [M][SPL][C] ((value bits << 32) | position); the last part of
    // the (item, column block) to arrive (a.ticket, zero before the launch and left zero) merges them
    // in position order -- the same first maximum as one pass over all positions. Every access is a
    // device-coherent (agent-scope) atomic, performed past the XCD's L2, and the ticket is taken only
    // once the stores are acknowledged: no L2 write-back or invalidate fence is needed.
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < NCT; ++n)
        __hip_atomic_store(a.part + ((long)i * SPL + h) * a.C + col + 16 * n,
                           ((unsigned long long)__float_as_uint(best[n]) << 32) | (unsigned)bi[n],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_s_waitcnt(0);  // (vmcnt 0: on gfx9 it counts the stores too)
    __syncthreads();
    if (tid == 0)
      s_arrived = __hip_atomic_fetch_add(a.ticket + (long)i * cb + cbk, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_arrived != SPL - 1) return;
    if (tid == 0) __hip_atomic_store(a.ticket + (long)i * cb + cbk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int n = 0; n < NCT; ++n) {
      best[n] = -INFINITY;
      bi[n] = kTextNoGrad;
#pragma unroll
      for (int hh = 0; hh < SPL; ++hh) {
        const unsigned long long pv = __hip_atomic_load(a.part + ((long)i * SPL + hh) * a.C + col + 16 * n,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float v = __uint_as_float((unsigned)(pv >> 32));
        const int t = (int)(unsigned)(pv & 0xffffffffu);
        if (v > best[n]) {  // (parts in position order: a tie keeps the earlier)
          best[n] = v;
          bi[n] = t;
        }
      }
    }
  }
  if (g == 0) {
#pragma unroll
    for (int n = 0; n < NCT; ++n) {
      const int cn = col + 16 * n;
      const bool on = best[n] > 0.f;
      if (cn < a.Creal) a.out[(long)i * a.ld + cn] = on ? best[n] : 0.f;
      a.tidx[(long)i * a.C + cn] = (uint8_t)(on ? bi[n] : kTextNoGrad);
    }
  }
  DCUE_KT(0, 4);
  DCUE_KTW(0, 7);
}

// ------------------------------------------------------------------------------- weight gradient
struct TextWgradArgs {
  const int32_t* tokens;
  const int32_t* item_track;
  const float* words;
  const float* dt;       // [M][C] dL/ds (before the ReLU / max routing)
  const uint8_t* tidx;   // [M][C]
  int M, T, E, C;
  int items_per_chunk;
  float* dW;             // one chunk: [C][E][3] and db [C] written directly
  float* db;
  float* wpart;          // several: [nchunk][C * E * 3 + C], the chunk's dW and db partials
};

constexpr int kTwW = 32;       // word channels per workgroup (64: a wave per output channel -- as fast, 9.1 MB)
constexpr int kTwO = 256 / kTwW;  // output channels per workgroup (256 threads)
constexpr int kTwItems = 64;   // items whose tokens / routing are staged in LDS per pass
// items per load group: their 3 word loads each are in flight per thread together, and the next
// group's are issued before this group's FMAs (two register sets)
constexpr int kTwG = 16;

// Round 6: a workgroup owns 8 output channels x 32 word channels over ALL of its
// chunk's items (one chunk at the in-batch shape: no partials, no reduce launch), so the grid is
// (C / 8) x (E / 32) workgroups -- 320 at config 4 -- with 3 accumulators per thread. Per item a
// thread reads its channel of the three word rows around the item's argmax position for its output
// channel straight from L2 (the tokens and the routing staged in LDS once). Exact fp32 FMAs in item
// order (deterministic); the chunk partials, where M needs several chunks, are summed in chunk order
// by k_text_wreduce. (4 x 64 workgroups -- a wave per output channel -- and 16-64 items per chunk:
// each 22-24 us as well, the 4 x 64 form at 9.1 MB against 7.6; per-workgroup trace: staging 5 us,
// the 64 items 16.5 us -- profiles/r06_text_wgrad_ab.txt.)
struct TwGroup {
  float x[kTwG][3];
  float gv[kTwG];
  uint64_t ok;  // bit 3 j + k: position ti + k - 1 inside the sentence (kTwG <= 21)
  unsigned live;
};
static_assert(3 * kTwG <= 64, "TwGroup::ok bits");
__global__ __launch_bounds__(256) void k_text_wgrad(TextWgradArgs a) {
  __shared__ int32_t tok_s[kTwItems * 128];  // [item][T], T <= 128
  __shared__ float g_s[kTwItems][kTwO];
  __shared__ int32_t ti_s[kTwItems][kTwO];
  DCUE_KTW(1, 6);
  DCUE_KT(1, 0);
  const int tid = threadIdx.x, cl = tid & (kTwW - 1), ol = tid / kTwW;
  // XCD-aware (o block, word-channel block): consecutive logical blocks -- the o blocks of one
  // word-channel block, which read the same 128-B slices of the batch's word rows -- on one XCD, so
  // each XCD's L2 fetches about 1/8 of the rows' bytes instead of all of them
  const int nob = gridDim.x, nbl = gridDim.x * gridDim.y;
  const int Lg = xcd_swizzle(blockIdx.x + nob * blockIdx.y, nbl);
  const int ob = (Lg % nob) * kTwO;
  const int c = (Lg / nob) * kTwW + cl;
  const int cc = c < a.E ? c : a.E - 1;  // (loads unconditional: clamped column, value dropped past E)
  const int T = a.T;
  const int ib = blockIdx.z * a.items_per_chunk, ie = min(a.M, ib + a.items_per_chunk);
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, bacc = 0.f;
  // group [s0, s0 + kTwG) of the staged items: routing from LDS, the word loads issued
  auto issue = [&](int s0, int ni, TwGroup& G) {
    G.ok = G.live = 0;
#pragma unroll
    for (int j = 0; j < kTwG; ++j) {
      const int sl = min(s0 + j, ni - 1);
      const int ti = ti_s[sl][ol];
      const bool lv = s0 + j < ni && ti != kTextNoGrad;
      G.live |= (unsigned)lv << j;
      G.gv[j] = g_s[sl][ol];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int t = ti + k - 1;  // staged position ti + k - 1 (outside the sentence: a zero row)
        const bool in = lv && t >= 0 && t < T;
        G.ok |= (uint64_t)in << (3 * j + k);
        const int tk = tok_s[sl * T + (in ? t : 0)];
        G.x[j][k] = a.words[(long)(in ? tk : 0) * a.E + cc];
      }
    }
  };
  auto consume = [&](const TwGroup& G) {
#pragma unroll
    for (int j = 0; j < kTwG; ++j) {
      if (!((G.live >> j) & 1u)) continue;  // (uniform over the kTwW lanes of one output channel)
      bacc += G.gv[j];  // db's partial, in item order
      acc0 = fmaf(G.gv[j], (G.ok >> (3 * j)) & 1u ? G.x[j][0] : 0.f, acc0);
      acc1 = fmaf(G.gv[j], (G.ok >> (3 * j + 1)) & 1u ? G.x[j][1] : 0.f, acc1);
      acc2 = fmaf(G.gv[j], (G.ok >> (3 * j + 2)) & 1u ? G.x[j][2] : 0.f, acc2);  // (64-bit mask)
    }
  };
  for (int i0 = ib; i0 < ie; i0 += kTwItems) {
    const int ni = min(kTwItems, ie - i0);
    __syncthreads();  // (the previous pass's readers)
    for (int e = tid; e < ni * T; e += 256) {
      const int sl = e / T, t = e - sl * T;
      tok_s[e] = a.tokens[(long)a.item_track[i0 + sl] * T + t];
    }
    for (int e = tid; e < ni * kTwO; e += 256) {
      const int sl = e / kTwO, oo = e - sl * kTwO;
      const long off = (long)(i0 + sl) * a.C + ob + oo;
      const int ti = a.tidx[off];
      ti_s[sl][oo] = ti;
      g_s[sl][oo] = ti == kTextNoGrad ? 0.f : a.dt[off];
    }
    __syncthreads();
    if (i0 == ib) DCUE_KT(1, 1);
    TwGroup G0, G1;
    issue(0, ni, G0);
    for (int s0 = 0; s0 < ni; s0 += 2 * kTwG) {
      if (s0 + kTwG < ni) issue(s0 + kTwG, ni, G1);  // in flight under G0's FMAs
      consume(G0);
      if (s0 + kTwG >= ni) break;
      if (s0 + 2 * kTwG < ni) issue(s0 + 2 * kTwG, ni, G0);
      consume(G1);
    }
  }
  DCUE_KT(1, 2);
  const int o = ob + ol;
  const long n = (long)a.C * a.E * 3;
  float* dw = gridDim.z == 1 ? a.dW : a.wpart + (long)blockIdx.z * (n + a.C);
  float* dbp = gridDim.z == 1 ? a.db : dw + n;
  if (c < a.E) {
    float* d = dw + ((long)o * a.E + c) * 3;
    d[0] = acc0;
    d[1] = acc1;
    d[2] = acc2;
  }
  if (c == cl && cl == 0) dbp[o] = bacc;  // (the first word-channel block)
  DCUE_KT(1, 3);
  DCUE_KTW(1, 7);
}

// the chunk partials [nchunk][n + C] (dW then db per chunk) summed in chunk order
__global__ __launch_bounds__(256) void k_text_wreduce(const float* __restrict__ wpart, int nchunk, long n, int C,
                                                      float* __restrict__ dW, float* __restrict__ db) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n + C) return;
  float s = 0.f;
  for (int z = 0; z < nchunk; ++z) s += wpart[(long)z * (n + C) + e];
  if (e < n)
    dW[e] = s;
  else
    db[e - n] = s;
}

template <int TB, int IPW>
static int launch_text_fwd_t(const TextFwdArgs& a, hipStream_t s) {
  dim3 grid((unsigned)((a.M + IPW - 1) / IPW), (unsigned)(a.C / 64));
  DCUE_LAUNCH((k_text_fwd<TB, IPW>), grid, dim3(256), 0, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_text_fwd(const TextBranch& tb, const int32_t* item_track, int M, float* out, long ld, uint8_t* tidx,
                    hipStream_t s) {
  TextFwdArgs a;
  a.tokens = tb.tokens; a.item_track = item_track; a.words = tb.words;
  a.xscale = ldexpf(1.f, tb.words_exp); a.inv_xscale = ldexpf(1.f, -tb.words_exp);
  a.wpack = reinterpret_cast<const uint4*>(tb.wpack16);
  a.bias = tb.bias;
  a.M = M; a.T = tb.T; a.E = tb.E; a.EP = tb.EP; a.C = tb.C; a.Creal = tb.Creal; a.pad = tb.pad;
  a.out = out; a.ld = ld; a.tidx = tidx;
  a.ticket = tb.ticket; a.part = tb.part;
  if (tb.C % 64 || tb.T < 1 || tb.T > 128 || tb.E % 4 || tb.EP % kTextKC || tb.EP < tb.E) return DCUE_ERR_INVALID;
  static const bool chunked = [] {
    const char* e = getenv("DCUE_TEXT_FWD");
    return e && e[0] == 'c';
  }();
  // A/B: DCUE_TEXT_FWD=<waves>x<column tiles per wave> (default 8x1), DCUE_TEXT_PARTS=2 (two
  // workgroups per item and column block over halves of the positions, merged through tickets:
  // measured no faster -- the merge's three device-coherent round trips cost what the halves save)
  static const int shape = [] {
    const char* e = getenv("DCUE_TEXT_FWD");
    return e && e[0] >= '1' && e[0] <= '9' ? atoi(e) * 10 + (strchr(e, 'x') ? atoi(strchr(e, 'x') + 1) : 1) : 81;
  }();
  static const int parts_env = [] {
    const char* e = getenv("DCUE_TEXT_PARTS");
    return e ? atoi(e) : 1;
  }();
  static const int xcds_env = [] {
    const char* e = getenv("DCUE_TEXT_XCDS");
    return e ? atoi(e) : 4;
  }();
  static const int bpd_env = [] {  // (A/B: the config-4 kernel's weight-prefetch depth, 6 / 10 / 15 steps)
    const char* e = getenv("DCUE_TEXT_BPD");
    return e ? atoi(e) : 6;
  }();
  const int tb_ = tb.T <= 16 ? 1 : tb.T <= 32 ? 2 : tb.T <= 64 ? 4 : 8;
  // position parts (DCUE_TEXT_PARTS=2): two workgroups per (item, column block), given the merge buffers
  const int spl = parts_env == 2 && tb_ >= 2 && tb.ticket && tb.part ? 2 : 1;
  const int tbw = tb_ / spl;  // 16-position tiles per workgroup
  // the workgroup's staged rows must fit the LDS (config 4, two parts: 34 rows x 1,424 B = 48 KB)
  const size_t lds = (size_t)(16 * tbw + 2) * text_full_pitch(tb.EP) * sizeof(_Float16);
  if (!chunked && lds <= 150 * 1024) {
    int wv = shape / 10, nct = shape % 10;
    if (tb.C % (16 * wv * nct) || wv > 8) wv = tb.C % 128 == 0 ? 8 : 4, nct = 1;
    // work units on 4 XCDs while they fill at most 4 x 32 CUs at one workgroup per CU (the weight
    // operand's per-XCD L2 fills halve); DCUE_TEXT_XCDS=8 spreads them over all eight
    const long nunit = (long)M * (tb.C / (16 * wv * nct)) * spl;
    a.nxcd = xcds_env == 8 || nunit > 4 * 32 ? 8 : 4;
    const unsigned grid = (unsigned)((nunit + a.nxcd - 1) / a.nxcd * 8);
    auto pick = [&](auto kern) -> int {
      static bool attr = false;  // (one per instantiation)
      if (!attr) {
        DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
        attr = true;
      }
      DCUE_LAUNCH(kern, dim3(grid), dim3(64 * wv), lds, s, a);
      DCUE_LAUNCH_CHECK();
      return DCUE_OK;
    };
    // B steps in flight: a divisor of the 3 * nchunk steps (registers: 8 * NCT per step); the config-4
    // word width (EP = 320: 10 chunks) at compile time
    const bool b6 = nct == 1 && tbw <= 4 && (tb.EP / kTextKC) % 2 == 0;
#define DCUE_TEXT_PICK_S(TBW, W, N, P, S)                                             \
  if (tbw == TBW && spl == S) {                                                       \
    if (P == 6 && tb.EP == 320) {                                                     \
      if constexpr (TBW == 4 && W == 8 && N == 1 && S == 1) {                         \
        if (bpd_env == 10) return pick(k_text_fwd_full<TBW, W, N, 10, 10, S>);        \
        if (bpd_env == 15) return pick(k_text_fwd_full<TBW, W, N, 15, 10, S>);        \
      }                                                                               \
      return pick(k_text_fwd_full<TBW, W, N, P, 10, S>);                              \
    }                                                                                 \
    return pick(k_text_fwd_full<TBW, W, N, P, 0, S>);                                 \
  }
#define DCUE_TEXT_PICK_B(W, N, P)        \
  DCUE_TEXT_PICK_S(1, W, N, P, 2)        \
  DCUE_TEXT_PICK_S(2, W, N, P, 2)        \
  DCUE_TEXT_PICK_S(4, W, N, P, 2)        \
  DCUE_TEXT_PICK_S(1, W, N, P, 1)        \
  DCUE_TEXT_PICK_S(2, W, N, P, 1)        \
  DCUE_TEXT_PICK_S(4, W, N, P, 1)        \
  DCUE_TEXT_PICK_S(8, W, N, P, 1)
#define DCUE_TEXT_PICK(W, N)              \
  if (wv == W && nct == N) {              \
    if constexpr (N == 1)                 \
      if (b6) { DCUE_TEXT_PICK_B(W, N, 6) } \
    DCUE_TEXT_PICK_B(W, N, 3)             \
  }
    DCUE_TEXT_PICK(4, 1)
    DCUE_TEXT_PICK(8, 1)
    DCUE_TEXT_PICK(8, 2)
    DCUE_TEXT_PICK(4, 2)
#undef DCUE_TEXT_PICK
#undef DCUE_TEXT_PICK_B
#undef DCUE_TEXT_PICK_S
    return DCUE_ERR_INVALID;
  }
  if (tb.T <= 16) return launch_text_fwd_t<1, 8>(a, s);
  if (tb.T <= 32) return launch_text_fwd_t<2, 4>(a, s);
  if (tb.T <= 64) return launch_text_fwd_t<4, 2>(a, s);
  return launch_text_fwd_t<8, 1>(a, s);
}

// item chunks of the text weight gradient: one up to 128 items (the in-batch shapes: no partials),
// else about 128 items per chunk, at most 16 chunks
int text_wgrad_nchunk(int M) {
  // DCUE_TEXT_WGRAD_ITEMS: items per chunk (A/B diagnostic; default 128)
  static const int per = [] {
    const char* e = getenv("DCUE_TEXT_WGRAD_ITEMS");
    const int v = e ? atoi(e) : 0;
    return v >= 8 && v <= 4096 ? v : 128;
  }();
  const int n = (M + per - 1) / per;
  return n < 1 ? 1 : (n > 16 ? 16 : n);
}

int launch_text_wgrad(const TextBranch& tb, const int32_t* item_track, int M, const float* dt, const uint8_t* tidx,
                      float* wpart, float* dW, float* db, hipStream_t s) {
  if (tb.C % kTwO || tb.T < 1 || tb.T > 128 || M < 1) return DCUE_ERR_INVALID;
  TextWgradArgs a;
  a.tokens = tb.tokens; a.item_track = item_track; a.words = tb.words;
  a.dt = dt; a.tidx = tidx;
  a.M = M; a.T = tb.T; a.E = tb.E; a.C = tb.C;
  const int nchunk = text_wgrad_nchunk(M);
  a.items_per_chunk = (M + nchunk - 1) / nchunk;
  a.dW = dW; a.db = db; a.wpart = wpart;
  const dim3 grid((unsigned)(tb.C / kTwO), (unsigned)((tb.E + kTwW - 1) / kTwW), (unsigned)nchunk);
  TimerScope tsc;  // (live timing: DCUE_TIMED_TEXT_WGRAD)
  TRY(timer_begin(&tsc, DCUE_TIMED_TEXT_WGRAD, s));
  DCUE_LAUNCH(k_text_wgrad, grid, dim3(256), 0, s, a);
  DCUE_LAUNCH_CHECK();
  TRY(timer_end(&tsc));
  if (nchunk == 1) return DCUE_OK;
  const long n = (long)tb.C * tb.E * 3;
  DCUE_LAUNCH(k_text_wreduce, dim3((unsigned)((n + tb.C + 255) / 256)), dim3(256), 0, s, wpart, nchunk, n, tb.C,
              dW, db);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
