// Internal launch interfaces shared by the libdcue_hip translation units.
#pragma once

#include <atomic>
#include <vector>

#include <functional>

#include "dcue_common.h"
#include "bnacc.h"

// Host-time attribution of step issue (diagnostic; DCUE_HOST_PROFILE=1 prints the per-label mean
// host time between consecutive marks at exit)
namespace dcue {
bool host_profile_on();
void host_profile_mark(const char* label);
bool on_side_worker();  // side.hip: this thread is the side-issue worker
}  // namespace dcue
#define HPROF(label)                                          \
  do {                                                        \
    if (::dcue::host_profile_on() && !::dcue::on_side_worker()) ::dcue::host_profile_mark(label); \
  } while (0)

// propagate a non-zero dcue_status
#define TRY(x)                 \
  do {                         \
    int _st = (x);             \
    if (_st) return _st;       \
  } while (0)

namespace dcue {

// -------------------------------------------------------------- conv as row-GEMM (fwd / dgrad)
// One kernel shape serves the forward conv of every layer and the input-gradient (dgrad) of
// layers 2..5: rows = (item, position) pairs, columns = output channels, K = taps x slab channels.
// The A operand is an LDS "slab" of input positions (with zero halos) built from its source with
// the neighbouring elementwise op fused into the load (BatchNorm apply in forward; BatchNorm
// backward + ReLU mask + max-pool routing in dgrad).
enum SlabSrc { SRC_TRACK_F16 = 0, SRC_TRACK_F32 = 1, SRC_ACT = 2, SRC_DZ = 3 };

// One conv weight segment's packed copies (WpackLayout): W[o][c][k] at params + src; -1 = no such copy
struct PackSeg {
  long src, fwd, bwd, f16, f16b;  // floats: W in params; f32 forward pack (-1: none); dgrad pack (-1:
                                 // none); split-f16 forward and dgrad packs
  int cout, cin, ks;
  int cinp;  // the split-f16 forward pack's K per tap: cin rounded up to 32 (the text conv's word width)
};

__device__ __forceinline__ void pack_store(const PackSeg& sg, long e, float w, float* wpack) {
  const long ks = sg.ks;
  const long o = e / ((long)sg.cin * ks);
  const long rem = e - o * sg.cin * ks;
  const long cc = rem / ks, k = rem - cc * ks;
  if (sg.fwd >= 0) wpack[sg.fwd + (((k * (sg.cin / 4) + cc / 4) * sg.cout + o) * 4 + (cc & 3))] = w;
  if (sg.bwd >= 0) {
    const long kr = sg.ks - 1 - k;
    wpack[sg.bwd + (((kr * (sg.cout / 4) + o / 4) * sg.cin + cc) * 4 + (o & 3))] = w;
  }
  // split-f16 forward operand: hi = fp16(w), lo = fp16(w - hi) (w - hi is exact in f32)
  const _Float16 hi = (_Float16)w;
  const _Float16 lo = (_Float16)(w - (float)hi);
  if (sg.f16 >= 0) {
    _Float16* h16 = reinterpret_cast<_Float16*>(wpack + sg.f16);
    const long q = k * (sg.cinp / 32) + cc / 32;
    const long base = ((q * sg.cout + o) * 4 + (cc & 31) / 8) * 16 + (cc & 7);
    h16[base] = hi;
    h16[base + 8] = lo;
  }
  if (sg.f16b >= 0) {  // split-f16 dgrad operand: K = (reversed tap, o), columns cc
    _Float16* b16 = reinterpret_cast<_Float16*>(wpack + sg.f16b);
    const long qb = (sg.ks - 1 - k) * (sg.cout / 32) + o / 32;
    const long bb = ((qb * sg.cin + cc) * 4 + (o & 31) / 8) * 16 + (o & 7);
    b16[bb] = hi;
    b16[bb + 8] = lo;
  }
}

struct RowsArgs {
  const void* src;            // tracks [n_tracks][131][128] | y_{l-1} [M][Lin][KC] | g_l [M][Lp_l][KC]
  const int32_t* item_track;  // tracks only
  const float* in_mean;       // forward BN apply: (x - mean) * a + beta  (in_bn.acc == null)
  const float* in_a;
  const float* in_beta;
  BnPublish in_bn;            // forward, train: input BN finalized from its accumulators; block 0
                              // publishes it (mean/invstd/a buffers + running statistics)
  const float* y_l;           // dgrad: layer-l ReLU output (pre-BN) [M][Lp_l][KC]
  const uint8_t* idx_l;       // dgrad: layer-l max-pool argmax [M][Lp_l][KC]
  const float* mean_l;
  const float* invstd_l;
  const float* a_l;           // gamma_l * invstd_l
  const unsigned long long* dz_acc;  // dgrad: [sum g_l, sum g_l*xhat_l] accumulators of layer l
  float invN;                 // 1 / (copies * positions)
  const float* counts;        // [M] copies per item (nullable -> 1)
  const float* wpack;         // [KS][KC/4][nout][4]
  const uint4* wpack16;       // forward, split-f16 path: [KS*KC/32][nout][4][hi, lo] x 8 halves
  const float* bias;          // forward [nout]
  float* out;                 // forward y_l [M][Lp][nout]; dgrad g_{l-1} [M][R][nout]
  uint8_t* out_idx;           // forward argmax [M][Lp][nout]
  unsigned long long* out_acc;  // forward: BN_l stats of the output (null: eval); dgrad: the
                                // BN_{l-1} backward sums of the produced gradient
  const float* oy;            // dgrad: y_{l-1} [M][R][nout], mean/invstd of BN_{l-1} (xhat of out)
  const float* omean;
  const float* oinvstd;
  int M;
  int nout;
  // dgrad, res towers: out[i][t][o] += skip[i * skip_ld + o] * skip_scale (the time-pooled skip's
  // gradient, AvgPool1d backward), before BN_{l-1}'s backward sums
  const float* skip;
  int skip_ld;
  float skip_scale;
  int skip_n;  // channels o < skip_n carry a skip gradient (the reference's H; storage pads none)
  // forward, split-f16: the input layer's value range ([2][kRngC] ordered keys, dcue_common.h) --
  // the raw track values (layer 1) or the previous layer's ReLU output (min 0) -- from which every
  // workgroup derives the same power-of-two operand scale; out_range: this layer's output maximum,
  // merged by the epilogue (nullable)
  const unsigned* in_range;  // dgrad (SRC_DZ): max |g_l| per channel instead (ordered keys)
  unsigned* out_range;
  unsigned* out_grange;  // dgrad: max |g_{l-1}| per channel (ordered keys), for the split-f16 wgrad
  const unsigned* y_range;  // dgrad: y_l's range (its maximum), for the dz bound
  float kd_max;             // dgrad: the largest copies(item) * invN of the batch
  // forward, train, layer 2: conv 2's input-gradient operands (rp: bwd / f16b only) repacked from its
  // weights rp_src, spread over the grid -- the split plans' late Adam leaves them to this launch, the
  // first on the caller's stream after that Adam and before the next input gradient of conv 2
  // (launch_adam defer_dgrad2); rp_src null: none
  const float* rp_src;
  float* rp_wpack;  // the model's wpack
  PackSeg rp;
  DevWait wait;  // plans: a side stream's signal to wait for at the kernel's start (conv 2: the late Adam)
};

struct WgradArgs {
  DevWait wait;               // plans, layer 1 (k_conv_wgrad16t): the next step's prepared inputs
  int bn_world;               // SyncBN (> 1): dz sums are over the ranks; BN_l's dgamma/dbeta get 1/world
  const void* xsrc;           // layer input: tracks (l=1) or y_{l-1} [M][Lin][cin]
  const int32_t* item_track;
  const float* x_mean;        // x = (src - mean) * a + beta ; l=1 uses xhat0 (a = invstd0, beta = 0)
  const float* x_a;
  const float* x_beta;        // nullable
  const float* g_l;           // dz construction, as RowsArgs
  const float* y_l;
  const uint8_t* idx_l;
  const float* mean_l;
  const float* invstd_l;
  const float* a_l;
  const unsigned long long* dz_acc;  // [sum g_l, sum g_l*xhat_l] accumulators of layer l
  float* dgamma;              // block (0,0,0) publishes BN_l's gradients: sum g*xhat, sum g
  float* dbeta;
  float invN;
  const float* counts;
  int M, cout, cin;
  int rows_per_chunk;
  float* wpart;               // [nchunk][cout][KS*cin]  (kc = k*cin + c)
  float* bpart;               // [nchunk][NB][cout]
  // split-f16 kernels (conv_wgrad.hip wgrad16_body): the operand columns' magnitude bounds
  const unsigned* x_range;    // the x source's value range, [2][kRngC] ordered keys (+x, -x)
  const unsigned* y_range;    // y_l's range ([0][c]: its maximum; a ReLU output)
  const unsigned* g_range;    // max |g_l| per channel (ordered keys of |g|), from its producer
  float kd_max;               // the largest copies(item) * invN of the batch
};
// SyncBN: BN_l's dgamma / dbeta come from sums over every rank; DDP then averages them, so each rank
// contributes 1/world of the global sum (torch SyncBatchNorm: local sums, averaged by DDP). x1 otherwise.
__device__ __forceinline__ double bn_grad_scale(const WgradArgs& a) { return a.bn_world > 1 ? 1.0 / a.bn_world : 1.0; }

// weight gradients of n conv layers (of 2..5) in one launch, then their chunk sums in a second one
// (the host fills n, layer[], a[], nchunk[], dW[], db[]; the launcher derives the block ranges)
// slot layer 6 = the fc layer (dW = df^T bn5(y5), db = sum df; a 1x1 conv with dz = df, no BN)
constexpr int kWgradMultiMax = 5;
struct WgradMulti {
  int n;
  int layer[kWgradMultiMax];
  WgradArgs a[kWgradMultiMax];  // one per slot, each with its own wpart / bpart
  int nchunk[kWgradMultiMax];
  float *dW[kWgradMultiMax], *db[kWgradMultiMax];
  int kt[kWgradMultiMax], ot[kWgradMultiMax];  // kc / o tiles per layer
  int start[kWgradMultiMax + 1];      // wgrad block ranges
  int rstart[kWgradMultiMax + 1];     // reduce block ranges
};
int launch_conv_wgrad_multi(WgradMulti w, hipStream_t s);
// weight gradients on split-f16 MFMA (DCUE_WGRAD_F16=0: the f32-MFMA kernels)
bool wgrad_f16_on();

int launch_conv_fwd(int layer, int kc, int src, const RowsArgs& a, hipStream_t s);
int launch_conv_dgrad(int layer, int kc, const RowsArgs& a, hipStream_t s);
int launch_conv_wgrad(int layer, int src, const WgradArgs& a, int nchunk, hipStream_t s);
// xhat0[i][t + 2][c] = (x[track_i][t][c] - mean0[c]) * invstd0[c] in a [M][kXp][128] zero-padded
// layout, bn0's batch statistics finalized from its accumulators (layer 1's wgrad reads it from `xsrc`)
int launch_xhat0(int src, const void* tracks, const int32_t* item_track, int M, const unsigned long long* acc0,
                 double count, float* xhat0, hipStream_t s);
int wgrad_nchunk(int layer, int M, int cout, int cin);
// layer 1: the pooled BN1 backward dx1[M*33][cout] that k_conv1_wgrad reads from `g_l` (the
// WgradArgs of the same call, with g_l the pooled gradient)
int launch_conv1_dx(const WgradArgs& a, float* dx1, hipStream_t s);
int launch_wgrad_reduce(int layer, const float* wpart, const float* bpart, int nchunk, int cout,
                        int cin, float* dW, float* db, float* G_tmp, float* E_tmp, hipStream_t s);
// One channel's bn0 constants and one dW1 element (k_bn0_grads and the fused k_bn0_grads_adam share
// them, so the two compute identical bits: explicit fmaf, no reliance on contraction flags).
// E = the five layer-1 bias-partial sums [5][H]: sum dz1 and its parts at t = 0, 1, R-2, R-1. Tap k
// of conv row t reads input t+k-2 (zero padding at t+k-2 < 0 or > 130), so
//   S[0] = e0-e1-e2, S[1] = e0-e1, S[2] = e0-e4, S[3] = e0-e3-e4;  db1 = e0.
struct Bn0Chan {
  float ga, be, m0, i0;
  bool raw;
};
__device__ __forceinline__ Bn0Chan bn0_chan(const float* gamma0, const float* beta0, const float* mean0,
                                            const float* invstd0, int c) {
  Bn0Chan r;
  r.ga = gamma0[c];
  r.be = beta0[c];
  r.raw = mean0 != nullptr;
  r.m0 = r.raw ? mean0[c] : 0.f;
  r.i0 = r.raw ? invstd0[c] : 1.f;
  return r;
}
__device__ __forceinline__ float bn0_elem(const float* __restrict__ G, const float* __restrict__ E, int H,
                                          const Bn0Chan& ch, int o, int k, int c, float w, float& dg, float& db) {
  const float e0 = E[o], e1 = E[H + o], e2 = E[2 * H + o], e3 = E[3 * H + o], e4 = E[4 * H + o];
  const float sv = k == 0 ? (e0 - e1) - e2 : k == 1 ? e0 - e1 : k == 2 ? e0 - e4 : (e0 - e3) - e4;
  const float gr = G[(size_t)o * 4 * kMels + k * kMels + c];
  const float gv = ch.raw ? ch.i0 * fmaf(-ch.m0, sv, gr) : gr;
  dg = fmaf(w, gv, dg);
  db = fmaf(w, sv, db);
  return fmaf(ch.ga, gv, ch.be * sv);
}
// split plans (StepOpts::dense_split): bn0's gradients and, in the same launch, Adam over segments
// [0, DCUE_SEG_LATE) -- bn0, conv 1 (with its weight repack), bn1 -- every one of which this
// kernel's workgroups complete (workgroup c owns input channel c; workgroups 0 / 1 conv 1's bias and
// bn1). p == nullptr: gradients only (as k_bn0_grads).
struct Bn0Adam {
  const dcue_model* md;              // p / m / v / grads / wpack
  const int64_t* poff;               // segment offsets (reference order)
  dcue_adam_args args;               // the dense Adam step (host values; the launcher forms scalars)
  bool bn;                           // towers with BatchNorm: bn0 / bn1 segments exist
};
int launch_bn0_grads_adam(const float* G, const float* E, const float* gamma0, const float* beta0,
                          const float* mean0, const float* invstd0, int H, float* dgamma0, float* dbeta0,
                          const Bn0Adam& a, hipStream_t s);

// mean0 / invstd0 (nullable): G is the contraction with the raw input (split-f16 path, fp16 table)
int launch_bn0_grads(const float* G, const float* E, const float* W1, const float* gamma0,
                     const float* beta0, const float* mean0, const float* invstd0, int H, float* dW1,
                     float* dgamma0, float* dbeta0, float* db1, hipStream_t s);

// ------------------------------------------------------------------------------- BatchNorm
// bn0 statistics of the gathered spectrograms (count-weighted) into accumulators [2][128]
// (acc nullable: the range only) and the raw input's per-mel range into `range` (nullable)
int launch_input_stats(int src, const void* tracks, const int32_t* item_track, const float* counts,
                       int M, unsigned long long* acc, unsigned* range, hipStream_t s);
// eval mode: running statistics -> mean / invstd / gamma*invstd
int launch_bn_eval(int C, const float* gamma, const float* rmean, const float* rvar, float* mean,
                   float* invstd, float* a, hipStream_t s);

// ------------------------------------------------------------------ packed weight layout
// wpack = conv B operands (forward per layer, dgrad per layer >= 2). Dense weights are read in place.
// conv_f16[l]: the forward B operand split into fp16 pairs w = hi + lo (hi = fp16(w), lo =
// fp16(w - hi)) for the split-f16 MFMA forward (conv.hip), as halves
// [k * cin/32 + c/32][cout][(c % 32) / 8][hi, lo][c % 8] -- one float slot per weight;
// conv_f16b[l] (l >= 2): the dgrad B operand the same way, K = (reversed tap, layer-l channel o),
// columns = layer l-1's channels: [(ks-1-k) * cout/32 + o/32][cin][(o % 32) / 8][hi, lo][o % 8]
// text_f16: the text conv's split-f16 B operand (text.hip), K = (tap, word channel padded to st_word),
// [k * EWs/32 + c/32][C_s][(c % 32) / 8][hi, lo][c % 8] halves (zero past word_dim: the caller
// zero-fills wpack once); -1 outside the text tower
struct WpackLayout {
  long conv_fwd[6], conv_bwd[6], conv_f16[6], conv_f16b[6];
  long text_f16;
  long total;
};
inline WpackLayout wpack_layout(const dcue_dims* dm) {
  WpackLayout w = {};
  const long H = st_hidden(dm), D = st_feature(dm);
  long n = 0;
  for (int l = 1; l <= 5; ++l) {
    const long cin = l == 1 ? kMels : H, cout = l == 5 ? D : H;
    const long e = cin * cout * layer_geom(l).ks;
    w.conv_fwd[l] = n;
    n += e;
    w.conv_bwd[l] = l >= 2 ? n : -1;
    if (l >= 2) n += e;
    w.conv_f16[l] = n;  // cin is a multiple of 32 (128, or H in 32..256)
    n += e;
    w.conv_f16b[l] = l >= 2 ? n : -1;  // cout too (H or d_s)
    if (l >= 2) n += e;
  }
  w.text_f16 = -1;
  if (tower_text(dm)) {
    w.text_f16 = n;
    n += 3L * st_word(dm) * st_text(dm);
  }
  w.total = n;
  return w;
}

// --------------------------------------------------------------------- batch, tail, towers
// copies per item (BatchNorm weights); in-batch negatives are found by wave ballots over neg_item
int launch_item_counts(const dcue_batch* b, float* counts, hipStream_t s);

// gather-layout batches of at most this many items get per-item copy lists (StepPrologue)
constexpr int kCopyListMaxItems = 2048;
// step prologue of a plan (sampler.hip): batch copies, accumulator clear, in-batch draw, counts
struct StepPrologue {
  dcue_mt_state* mt;  // null: no draw (neg already given, or catalogue)
  int B, N, M;
  int gather;         // layout GATHER: counts from neg (else every item counts 1)
  int32_t* neg;
  int64_t* users_dst;
  const int64_t* users_src;  // nullable
  int32_t* items_dst;
  const int32_t* items_src;  // nullable
  unsigned long long* zero;  // words to clear
  long nzero;
  float* counts;             // [M] (nullable)
  dcue_mt_state* mt_out;     // where the advanced state goes (null: back to mt)
  dcue_mt_state* mt_commit;  // nullable: receives the state as loaded, before this draw
  const int32_t* copy_src;   // nullable: copy_dst[0..ncopy) = copy_src[..] (published negatives)
  int32_t* copy_dst;
  long ncopy;
  // nullable (gather layout): each item's copies as a CSR for the item-gradient sums -- copy_ptr[M+1],
  // copy_idx[B(N+1)] holding copy indices row*(N+1)+c, the positive first, then the negatives that
  // drew the item in (row, j) order
  int32_t* copy_ptr;
  int32_t* copy_idx;
};
int launch_step_prologue(const StepPrologue& p, hipStream_t s);

// small GEMM: C(m,n) = sum_k TA(A(m,k)) TB(B(k,n)) (+bias[n]) (*[cmask > 0]); TA: 0 none, 1 relu,
// 2 affine per k; TB: 0 none, 1 relu, 2 affine per n (affine = BatchNorm apply (x-mean)*a+beta)
struct TGemmArgs {
  int M, N, K;
  const float* A; long sam, sak; const int64_t* arow;
  const float* B; long sbk, sbn; const int64_t* brow;
  const float *amean, *aa, *abeta;
  BnPublish abn;  // TA == 2, train: the per-k BatchNorm comes from accumulators (block 0 publishes)
  const float *bmean, *ba, *bbeta;
  const float* bias;
  float* C; long scm, scn;
  const float* cmask; long smm, smn; const int64_t* cmrow;
  float* rowsum;  // nullable: sum_k TA(A(m,k)) per row m
  // nullable: per-column BN-backward sums of C into accumulators [2][N]: sum C, sum C * xhat with
  // xhat = (xy[m][n] - xmean[n]) * xinvstd[n]
  unsigned long long* colacc;
  const float *xy, *xmean, *xinvstd;
  unsigned* colmax;  // nullable: max |C| per column (ordered keys), the split-f16 wgrad's dz bound
};
int launch_tgemm(int ta, int tb, const TGemmArgs& g, hipStream_t s);
// the user tower's forward in one launch (adam.hip k_user_fwd): deferred mode's row sync, then g1
// (h1 = relu(E[users]) W1^T + b1) and g2 (uf = relu(h1) W2^T + b2) as launch_tgemm(1, 0, .) computes them
int launch_user_fwd(const dcue_model* md, const TGemmArgs& g1, const TGemmArgs& g2, const int64_t* users, int B,
                    hipStream_t s, unsigned* sig = nullptr);
int user_fwd_blocks(int B);  // k_user_fwd's workgroups (each adds 1 to sig)
// two independent GEMMs in one launch: g1 as launch_tgemm(0, 1, .) with a k-strided A, g2 as
// launch_tgemm(0, 0, .) with a k-contiguous A; both with n-contiguous B (the user tower's backward)
int launch_tgemm_pair(const TGemmArgs& g1, const TGemmArgs& g2, hipStream_t s);

int launch_score_fwd(const float* uf, const float* f, const dcue_batch* b, int d, float margin,
                     float* scores, float* cosv, float* norms, float* hinge, float* loss,
                     float* dhinge, hipStream_t s);
// forward + hinge backward in one pass (the loss gradient is known in the forward): also writes
// du / dfcopy and the per-row hinge sums; k_item_grad (given the row sums) takes the loss mean
int launch_score_fused(const float* uf, const float* f, const dcue_batch* b, int d, float margin,
                       float* scores, float* cosv, float* norms, float* rowsum, float* du,
                       float* dfcopy, hipStream_t s, DevWait uf_wait = DevWait{});
// k_signal: store `val` into the signal word `flag` once the stream's earlier work is done (DevWait)
int launch_signal(unsigned* flag, unsigned val, hipStream_t s);
// a plan's signal words (StepOpts::sig): the user tower's output, the late Adam, the prepared inputs
enum SigSlot { kSigUf = 0, kSigLate = 1, kSigInputs = 2, kSigText = 3, kSigSlots = 16 };
int launch_score_bwd(const float* uf, const float* f, const dcue_batch* b, int d,
                     const float* dscores, const float* cosv, const float* norms, float* du,
                     float* dfcopy, hipStream_t s);
// per-item feature gradients; with fcW also the fc input gradient g5 = df W and BN5's backward sums.
// copy_ptr / copy_idx (nullable): the gather layout's per-item copy lists from the step prologue
// g5max / dfmax (nullable): max |g5| / max |df| per column, ordered keys (split-f16 wgrad bounds)
int launch_item_grad(const float* dfcopy, const dcue_batch* b, int d, float* df, const float* fcW, float* g5,
                     unsigned long long* acc5, const float* y5, const float* mean5, const float* invstd5,
                     const float* rowsum, float* loss, const int32_t* copy_ptr, const int32_t* copy_idx,
                     unsigned* g5max, unsigned* dfmax, hipStream_t s);
int launch_emb_grad(const float* de, const int64_t* users, int B, int E, float scale,
                    float* emb_grad, int32_t* slot, int64_t* emb_rows, dcue_emb_log* log,
                    hipStream_t s);
// flush_slice = false: the user-table part leaves this step's rolling-flush slice to the caller
// (plans issue it during the next step, after that step's user tower: launch_emb_flush_rows)
// dense_lo / dense_hi: the dense part over [dense_lo, dense_hi) of the flat buffer only (-1: to the end)
// defer_dgrad2: leave conv 2's input-gradient operands (WpackLayout conv_bwd[2] / conv_f16b[2]) to
// the next training forward of conv 2 (RowsArgs::rp): the split plans' late Adam, which may run
// beside the caller stream's dgrad of conv 2 that reads them
int launch_adam(const dcue_model* m, const dcue_adam_args* a, const int64_t* poff, hipStream_t s,
                bool flush_slice = true, long dense_lo = 0, long dense_hi = -1, bool defer_dgrad2 = false,
                unsigned* sig = nullptr);
// workgroups of the dense Adam sweep over len floats (each adds 1 to launch_adam's sig)
long adam_dense_blocks(long len);
// conv layer l's packed copies (adam.hip pack_args)
PackSeg pack_seg(const dcue_model* m, const int64_t* poff, int l);
int launch_emb_flush_rows(const dcue_model* m, int step, hipStream_t s);
// deferred mode: launch_emb_grad + the user-table part of launch_adam (k_adam_touched) in one launch
// (k_emb_grad_adam, adam.hip): the same compact rows and the same per-element Adam arithmetic; the
// rolling-flush slice is left to the caller (plans issue it during the next step)
int launch_emb_grad_adam(const dcue_model* m, const dcue_adam_args* a, const float* de, const int64_t* users, int B,
                         float scale, hipStream_t s);
// BN-free towers: mean 0, invstd = a = 1 for the six BN layers, plus the ones / zeros arrays
int launch_bn_identity(float* const* mean, float* const* invstd, float* const* a, float* ones, float* zeros,
                       int cmax, int H, int D, hipStream_t s);
// res towers: xfc[i] = [mean_t bn_1(y_1), ..., mean_t bn_4(y_4), bn_5(y_5)] (truedcuemel1dres.py:93-97);
// p5 (train, BN): BN_5 finalized from its accumulators here (block 0 publishes it)
// H: storage width of y_1..y_4; HL: the reference's H, the column width of each block in xfc
// text tower (HL = 0): only bn5(y5), at columns [off5, off5 + D) of rows ld wide (res: off5 = 4 HL,
// ld = 4 HL + D)
int launch_timepool(float* const* y, float* const* mean, float* const* a, const float* beta1, const float* beta2,
                    const float* beta3, const float* beta4, const float* beta5, const BnPublish& p5, int M, int H,
                    int HL, int D, int off5, int ld, float* xfc, hipStream_t s);
// Text branch of the mixed item tower (text.hip): the token table, frozen word vectors, the text conv's
// split-f16 weight pack and bias, widths (C = storage channels, Creal = the reference's text_dim)
struct TextBranch {
  const int32_t* tokens;  // [n_tracks][T]
  const float* words;     // [V][E]
  int words_exp;
  const float* wpack16;   // WpackLayout::text_f16
  const float* bias;      // [C]
  int T, E, EP, C, Creal, pad;
  // the forward's position parts (text.hip k_text_fwd_full): per (item, column block) arrival
  // tickets, zero before the launch (the workspace's accumulator block), and the parts' maxima
  // [M][2][C]; null: one workgroup over all positions
  unsigned* ticket = nullptr;
  unsigned long long* part = nullptr;
};
// s[i][o] (o < Creal) -> out[i * ld + o] (the fc input's text columns), argmax -> tidx [M][C]
int launch_text_fwd(const TextBranch& tb, const int32_t* item_track, int M, float* out, long ld, uint8_t* tidx,
                    hipStream_t s);
// chunk partials of the text conv's weight / bias gradients (wpart: text_wgrad_nchunk(M) x (C E 3 + C)
// floats) and their chunk-ordered sums into dW [C][E][3], db [C]; dt [M][C] = dL/ds (read where
// tidx != 255)
int text_wgrad_nchunk(int M);
int launch_text_wgrad(const TextBranch& tb, const int32_t* item_track, int M, const float* dt, const uint8_t* tidx,
                      float* wpart, float* dW, float* db, hipStream_t s);
// SGD / Ranger over the dense buffer and the user table (optim.hip)
int launch_opt(const dcue_model* m, const dcue_opt_args* a, const dcue_opt_state* st, long n_dense,
               hipStream_t s);
int launch_emb_log_init(const dcue_model* m, int cap, int step, hipStream_t s);
int launch_emb_sync(const dcue_model* m, const int64_t* users, int n, hipStream_t s);
int launch_emb_flush(const dcue_model* m, hipStream_t s);
int launch_pack(const dcue_model* m, const int64_t* poff, hipStream_t s);

// ----------------------------------------------------------------- live kernel timing (timer.hip)
struct TimerScope {
  int cls = -1;
  hipStream_t s = nullptr;
  hipEvent_t a = nullptr, b = nullptr;  // bound to the timed launch (LaunchTag start / stop)
  LaunchTag saved;                      // the enclosing scope's tag, restored by timer_end
  bool capturing = false;
  std::vector<hipGraphNode_t> preds;  // under capture: the stream's dependency set before the launch
};
// A timed launch seen under stream capture: the plan adds event-record nodes around `kernel`.
struct CapturedTimer {
  int cls;
  std::vector<hipGraphNode_t> preds;
  hipGraphNode_t kernel;
};
int timer_begin(TimerScope* sc, int cls, hipStream_t s);
int timer_end(TimerScope* sc);
hipEvent_t timer_event();
void timer_release(hipEvent_t e);
void timer_add_recorded(int cls, hipEvent_t a, hipEvent_t b);
// RCCL exchange of a plan step (comm.hip): bucket grad[late:n) once `side_done`, then grad[0:late)
// after the caller's stream `s`; `s` then waits for both
int comm_exchange_step(dcue_comm* c, float* grad, long late, long n, hipEvent_t side_done, hipStream_t s);
// the split plans' exchange (StepOpts::comm): the comm stream waits for the side streams' points
// side[0..nside), all-reduces grad[late:n), runs Adam over it (dense, grad_div = world, conv 2's
// input-gradient operands deferred) and records *late_done; then, after the caller's stream `s`,
// all-reduces grad[0:late), and `s` waits for it.
// The caller then runs Adam over [0, late) on `s`.
int comm_exchange_split(dcue_comm* c, const dcue_model* m, const dcue_adam_args* dense, const int64_t* poff,
                        long late, long n, const hipEvent_t* side, int nside, hipEvent_t late_done, hipStream_t s);
int comm_world(const dcue_comm* c);
// SyncBN: n uint64 words (exact fixed-point BN accumulators, bnacc.h) summed over the ranks in place,
// ordered on `s` (through the comm's stream, so every collective of a rank runs in issue order)
int comm_allreduce_u64(dcue_comm* c, unsigned long long* buf, long n, hipStream_t s);
int comm_divide(const dcue_comm* c, float* grad, long n, hipStream_t s);
// whether this occurrence of a timed class is one to time (every stride-th; for intervals timed by
// event records rather than a bound launch, e.g. the RCCL exchange)
bool timer_take_turn(int cls);
std::vector<CapturedTimer> timer_take_captured();

// Flags of the library's stream-ordering events. They only order work between streams of one
// device, so they take a device-scope release: the default system-scope one writes back and
// invalidates the caches when the event completes, which measured 4-9 us of idle on the waiting and
// the recording stream after every event-bound kernel of a step (profiles/r03: the critical
// chain's gaps). DCUE_EVENT_SCOPE=system restores the default (A/B).
unsigned sync_event_flags();
// side streams (capi.hip): three per device, plus a ring of fork/join events
struct SidePool {
  // st[0]: user tower + user-table Adam; st[1], st[2]: weight gradients of layers 5..2
  // (alternating). Three side streams + the caller's = the box's 4 hardware queues: a fifth stream
  // would share a queue with another and serialize behind it.
  hipStream_t st[3] = {nullptr, nullptr, nullptr};
  static constexpr int kEvents = 512;
  hipEvent_t ev[kEvents] = {};
  std::atomic<unsigned> next{0};  // fork_point / ring_event: both host threads (side.hip) take events
};
SidePool* side_pool();
int stream_wait(SidePool* p, hipStream_t to, hipStream_t from);
int fork_point(SidePool* p, hipStream_t from, hipEvent_t* ev);
hipEvent_t ring_event(SidePool* p);

// Set while a plan captures its step (bound launch events are not captured; records are).
bool& capturing_step();

// A fork point at the end of the launches made inside the scope, without an event-record packet:
// the scope's ring event is bound to each launch (LaunchTag; the last binding is what a wait sees).
// If the scope launched nothing, or the step is being captured, done() records the event instead.
// Scopes nest: launches of an inner scope do not bind the outer event, so the outer one records.
class ForkAfter {
 public:
  ForkAfter(SidePool* p, hipStream_t s, hipEvent_t* ev);
  ~ForkAfter();
  int done();

 private:
  void restore();
  hipStream_t s_;
  hipEvent_t* out_;
  hipEvent_t e_;
  LaunchTag saved_;
  bool armed_ = false, finished_ = false;
};
int wait_point(hipStream_t to, hipEvent_t ev);
int join_user_stream(hipStream_t s);

// Side-stream issue on a second host thread (side.hip). run(fn) posts fn to the device's worker
// (FIFO) and returns its sequence number, or runs it here (returning 0, status in *inline_status)
// when the worker is off (DCUE_SIDE_THREAD=0), under stream capture, or on the worker itself.
// wait(seq): fn and everything posted before it have been issued; returns the first error a
// closure reported. The destructor waits for everything this queue posted.
class SideQueue {
 public:
  explicit SideQueue(bool enable = true);
  ~SideQueue();
  SideQueue(const SideQueue&) = delete;
  SideQueue& operator=(const SideQueue&) = delete;
  bool threaded() const { return impl_ != nullptr; }
  uint64_t run(std::function<int()> fn, int* inline_status);
  int wait(uint64_t seq);
  int drain();

 private:
  void* impl_ = nullptr;
  uint64_t last_ = 0;
};
bool on_side_worker();
// split plans: one wait before conv 1 for the previous step's late Adam, which covers the prepared
// inputs (capi.hip)
bool late_wait_at_conv1();

// ---------------------------------------------------------------- diagnostics (debug.hip)
// a spin kernel ahead of the work at `site` when a delay is set for it (dcue_debug_delay)
int debug_delay(int site, hipStream_t s);
// dcue_debug_probes: one record per probe id
struct ProbeRec {
  unsigned nonfinite, nonzero;
  unsigned long long first_bad;
};
enum ProbeId {
  PR_Y1 = 0,  // ... PR_Y1 + 4 = y5
  PR_H1 = 5, PR_UF, PR_F, PR_SCORES, PR_DU, PR_DFCOPY, PR_DF, PR_G5,
  PR_G4, PR_G3, PR_G2, PR_G1,  // dgrads 5..2
  PR_DE, PR_G_USER, PR_G_HI, PR_G_2, PR_G_FC, PR_G_1, PR_P_EARLY, PR_P_LATE,
  kNumProbes
};
bool probes_on();
int probe(int id, const float* x, long n, hipStream_t s);
bool poison_on();
unsigned* user_fwd_fail_flag();
// frozen-row epochs of a user-table Adam log (adam.hip): forget the host's epoch (the log re-initialised)
void frz_forget(const dcue_emb_log* hdr);
// DCUE_LEGACY_ORDERS=1: the round-4 cross-stream orders, without the waits that closed its races
//  -- only to show tests/test_gpu_races.py failing on them
bool legacy_orders();

// ------------------------------------------------------------- step implementation (capi.hip)
struct StepOpts {
  hipEvent_t wait_inputs = nullptr;  // plans: the next step's prepared inputs; the caller's stream
                                     // waits for it before the conv-1 weight gradient
  uint64_t wait_inputs_seq = 0;      // ... once the side-issue thread has recorded it (SideQueue)
  // plans: the next step's input preparation (lookahead), issued by the backward on the side path
  // once the dgrad chain's first fork point exists (its argument: that point, which orders it after
  // everything the caller enqueued before the step); the conv-1 weight gradient's wait for
  // wait_inputs then waits for it to be issued
  const std::function<int(hipEvent_t)>* ahead = nullptr;
  // plans: a point on the caller's stream at the launch's start (the user tower waits for it);
  // null: the forward records one
  hipEvent_t ev_in = nullptr;
  dcue_comm* sync_bn = nullptr;  // SyncBN: BatchNorm sums all-reduced over this communicator's ranks
  bool prologue_done = false;  // counts written + accumulators cleared by the prologue
  bool fuse_score = false;     // train forward also runs the hinge backward (k_score_fused)
  const dcue_adam_args* emb_adam = nullptr;  // backward: also step the user table (parts = EMBEDDING)
  hipEvent_t* score_done = nullptr;     // forward (fuse_score): a fork point after the score kernel
  // backward: where the step ends, for a caller that prepares the next one (plans): [0] the
  // caller's stream after its last kernel, [1] wgrad stream 0 once every side stream's part is in
  hipEvent_t* tails = nullptr;
  // prepared ahead (plans): the step's copy counts and its cleared accumulator block, in place of
  // the workspace's own
  const float* counts = nullptr;
  unsigned long long* acc = nullptr;
  // deferred rolling flush (plans): the backward's user-table Adam skips its flush slice, and the
  // next forward issues the slice of step flush_slice_step on the user stream right after the user
  // tower -- same stream order relative to every Adam step, but off the next step's user-tower path
  bool defer_flush_slice = false;
  int flush_slice_step = -1;
  // the slice issued off the user stream (DCUE_SLICE_STREAM): its end, which the backward's
  // user-table Adam waits for (written by the forward's user part, read by the backward's)
  hipEvent_t* slice_done = nullptr;
  // prepared one step ahead from the announced next batch (plans, dcue_plan_set_next): bn0's batch
  // sums already in `acc`, and the conv-1 weight gradient's X operand (k_xhat0) already built
  bool input_stats_done = false;
  const float* xhat0 = nullptr;
  bool clear_bn0 = false;  // the block holds bn0 sums of an announced batch this step did not use
  // split dense Adam (plans without a communicator): the caller's stream runs Adam over bn0 / conv 1 /
  // bn1 (segments [0, DCUE_SEG_LATE)) right after its conv-1 tail, and the user stream the rest once
  // the side streams' gradients are in -- the caller's stream never waits for the join. *late_done
  // receives the user stream's point after that part; the next forward waits for it before conv 2
  // (the first reader of a late segment on the caller's stream).
  const dcue_adam_args* dense_split = nullptr;
  hipEvent_t* late_done = nullptr;
  hipEvent_t wait_late = nullptr;  // forward: the previous split step's late_done
  // plans (round 6): device-side waits (DevWait) in place of the caller stream's event waits -- the
  // plan's signal words [kSigSlots] and its host counters of the values issued into them (null:
  // event waits); late_wait: the previous step's late Adam (conv 2 waits for it instead of wait_late),
  // *late_sig receives this step's; inputs_wait: the next step's prepared inputs (the conv-1 weight
  // gradient waits for it instead of wait_inputs)
  unsigned* sig = nullptr;
  unsigned* sig_issued = nullptr;
  DevWait late_wait{};
  DevWait* late_sig = nullptr;
  DevWait inputs_wait{};
  // the step's per-item copy lists (gather layout, built by the plan's prologue; StepPrologue)
  const int32_t* copy_ptr = nullptr;
  const int32_t* copy_idx = nullptr;
  // DCBR regression (dcue_dcbr_step): the item tower only -- dfcopy already holds dL/df, no score
  // backward, no user tower, no embedding gradient
  bool item_only = false;
  // split plans: conv 1's output y_1 per plan slot (step parity). The layer-2 weight gradient of step
  // t reads y_1 on a side stream that the caller's stream does not join before step t+1's conv 1
  // writes it; alternating buffers keep that write off the one being read (step t+2's conv 1 is
  // ordered after it: its stream waited for step t's late Adam before step t+1's conv 2)
  float* y1 = nullptr;
  // split plans with a communicator (data parallelism): the exchange runs inside the backward -- the
  // late bucket all-reduced on the comm stream once the side streams' gradients are in and Adam over
  // it right there (dense_split's grad_div = world), bn0 / conv 1 / bn1 after the early bucket on the
  // caller's stream -- so each Adam waits only for its own bucket (comm_exchange_split)
  dcue_comm* comm = nullptr;
};
// DCBR's MSE head: loss = sum over [M][d] of (f - y)^2 / (M d) (rows of width ld, the first d
// columns), df = 2 (f - y) / (M d) into dfcopy ([M][ld], zero past d); rowsq [M]: the per-row sums
// (scratch); deterministic
int launch_mse_grad(const float* f, const float* y, int M, int d, int ld, float* df, float* rowsq, float* loss,
                    hipStream_t s);
// A batch's model-independent item inputs, issued ahead of its step (plans): bn0's count-weighted
// batch sums into the accumulator block `acc` (cleared, counts written, on the same stream before)
// and bn0(x) zero-padded into xhat0 ([M+1][kXp][128] floats).
int ahead_item_inputs(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, const int32_t* items,
                      const float* counts, unsigned long long* acc, float* xhat0, hipStream_t s);
// words of the per-step accumulator block (BN sums) cleared before each step
long step_acc_words(const dcue_dims* d, int B, int N, int M);
int forward_impl(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
                 int train, float margin, const StepOpts& o, hipStream_t s);
int backward_impl(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
                  const float* dscores, float emb_grad_scale, const StepOpts& o, hipStream_t s);
int step_prologue(const dcue_model* m, const dcue_batch* b, void* ws, size_t ws_bytes, dcue_mt_state* mt,
                  const int64_t* users_src, const int32_t* items_src, hipStream_t s);

}  // namespace dcue
