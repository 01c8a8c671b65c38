// libdcue_hip C ABI: layouts, workspace carving and the per-step kernel schedule.
//
// The schedule mirrors the reference step (nn/dcue.py:202-210):
//   forward   bn0 stats -> [conv_l (BN_{l-1} fused in its load) -> BN_l stats] x5 -> fc ->
//             user tower -> cosine scores + hinge loss                (dcue/dcue.py:70-108)
//   backward  score grads -> item grads -> fc -> [BN_l bwd sums -> wgrad_l, dgrad_l] l=5..2 ->
//             BN1 -> wgrad_1 (+ bn0 grads without conv1 dgrad) -> user tower -> embedding rows
//   adam      dense params + user table, then weight repack
#include <math.h>
#include <atomic>
#include <functional>
#include <string.h>

#include "dcue_internal.h"

using namespace dcue;

namespace dcue {
// Side streams. A training step is a chain of small kernels, each far from filling 256 CUs; the
// independent branches run concurrently: the user tower beside the item tower (forward and
// backward), and each conv layer's weight gradient beside the dgrad chain of the layers below
// (alternating between two streams, each with its own partial-sum buffers). Forks and joins are
// event-ordered against the caller's stream, so the calls stay stream-ordered (and capturable).

unsigned sync_event_flags() {
  static const unsigned f = [] {
    const char* e = getenv("DCUE_EVENT_SCOPE");
    return (e && e[0] == 's') ? (unsigned)hipEventDisableTiming
                              : (unsigned)(hipEventDisableTiming | hipEventReleaseToDevice);
  }();
  return f;
}

SidePool* side_pool() {
  static SidePool pools[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SidePool& p = pools[dev];
  if (!p.st[0]) {
    // DCUE_SIDE_PRIO=low: the side streams at the device's least stream priority, so the command
    // processor favours the caller's (critical-path) queue when both have workgroups to dispatch
    static const bool low = [] {
      const char* e = getenv("DCUE_SIDE_PRIO");
      return e && e[0] == 'l';
    }();
    // DCUE_USER_PRIO=high: the user stream (st[0]) at the device's greatest priority, so its short
    // user-tower GEMMs are dispatched between the item tower's conv workgroups (A/B knob)
    static const bool user_high = [] {
      const char* e = getenv("DCUE_USER_PRIO");
      return e && e[0] == 'h';
    }();
    int least = 0, greatest = 0;
    if ((low || user_high) && hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
    for (int i = 0; i < 3; ++i) {
      hipStream_t& s = p.st[i];
      const bool prio = low || (user_high && i == 0);
      const int pr = (user_high && i == 0) ? greatest : least;
      if ((prio ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pr)
                : hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess)
        return nullptr;
    }
    for (auto& e : p.ev)
      if (hipEventCreateWithFlags(&e, sync_event_flags()) != hipSuccess) return nullptr;
  }
  return &p;
}

// A point on `from` that other streams can wait for later (wait_point): a ring event is recorded
// now. The ring is long enough that no event is re-recorded before its waits are enqueued
// (a step records fewer than 16 points).
int fork_point(SidePool* p, hipStream_t from, hipEvent_t* ev) {
  hipEvent_t e = ring_event(p);
  DCUE_HIP_CHECK(hipEventRecord(e, from));
  *ev = e;
  return DCUE_OK;
}

hipEvent_t ring_event(SidePool* p) {
  return p->ev[p->next.fetch_add(1, std::memory_order_relaxed) % SidePool::kEvents];
}

LaunchTag& launch_tag() {
  thread_local LaunchTag t;
  return t;
}

static std::atomic<int64_t> g_launches{0};
void count_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }

bool& capturing_step() {
  thread_local bool c = false;
  return c;
}

ForkAfter::ForkAfter(SidePool* p, hipStream_t s, hipEvent_t* ev) : s_(s), out_(ev), e_(ring_event(p)) {
  saved_ = launch_tag();
  if (!capturing_step()) {
    launch_tag() = LaunchTag{nullptr, e_, 0, false};
    armed_ = true;
  }
}

void ForkAfter::restore() {
  if (!armed_) return;
  const int n = launch_tag().launches;
  launch_tag() = saved_;
  if (n && saved_.stop) launch_tag().missed = true;
  armed_ = false;
}

int ForkAfter::done() {
  if (finished_) return DCUE_OK;
  finished_ = true;
  const bool bound = armed_ && launch_tag().launches > 0 && !launch_tag().missed;
  restore();
  if (!bound) DCUE_HIP_CHECK(hipEventRecord(e_, s_));
  *out_ = e_;
  return DCUE_OK;
}

ForkAfter::~ForkAfter() { restore(); }

// Plans leave the user table's Adam step (and its rolling flush slice) running on the user stream
// past the end of a step; entry points that touch the table from the caller's stream join it first.
int join_user_stream(hipStream_t s) {
  SidePool* sp = side_pool();
  if (!sp) return DCUE_ERR_HIP;
  return stream_wait(sp, s, sp->st[0]);
}

int wait_point(hipStream_t to, hipEvent_t ev) {
  DCUE_HIP_CHECK(hipStreamWaitEvent(to, ev, 0));
  return DCUE_OK;
}

// `to` waits for everything enqueued on `from` so far. An event is re-recorded only after the
// wait on its previous record has been enqueued, so a small ring of events suffices.
int stream_wait(SidePool* p, hipStream_t to, hipStream_t from) {
  hipEvent_t e = ring_event(p);
  DCUE_HIP_CHECK(hipEventRecord(e, from));
  DCUE_HIP_CHECK(hipStreamWaitEvent(to, e, 0));
  return DCUE_OK;
}

}  // namespace dcue

namespace {

constexpr int kSeg = DCUE_N_DENSE_SEGMENTS;

int check_dims(const dcue_dims* d) {
  if (!d) return DCUE_ERR_INVALID;
  if (d->conv_hidden <= 0 || d->feature_dim <= 0 || d->user_embdim <= 0 || d->n_users < 0)
    return DCUE_ERR_INVALID;
  // any width up to 256 (run at its storage width, dcue_common.h); the user tower's E up to 1024
  if (d->conv_hidden > 256 || d->feature_dim > 256 || d->user_embdim > 1024) return DCUE_ERR_UNSUPPORTED;
  if (d->tower < DCUE_TOWER_BN || d->tower > DCUE_TOWER_TEXT) return DCUE_ERR_INVALID;
  if (d->tower == DCUE_TOWER_TEXT) {  // text.hip's limits: uint8 argmax positions, float4 word rows
    if (d->text_dim <= 0 || d->word_dim <= 0 || d->text_len < 2 || d->text_pad < 0) return DCUE_ERR_INVALID;
    if (d->text_dim > 256 || d->word_dim > 1024 || d->word_dim % 4 || d->text_len > 128) return DCUE_ERR_UNSUPPORTED;
  }
  return DCUE_OK;
}

long al4(long v) { return (v + 3) & ~3L; }

void param_sizes(const dcue_dims* d, long* sz) {
  const long H = st_hidden(d), D = st_feature(d), E = d->user_embdim;
  const long cin[5] = {kMels, H, H, H, H}, cout[5] = {H, H, H, H, D};
  const long bn = tower_has_bn(d) ? 1 : 0;  // the BN parameters' segments are empty without BN
  int s = 0;
  sz[s++] = bn * kMels;  // bn0.weight
  sz[s++] = bn * kMels;  // bn0.bias
  for (int l = 1; l <= 5; ++l) {
    sz[s++] = cout[l - 1] * cin[l - 1] * layer_geom(l).ks;  // conv.layer{l}.weight
    sz[s++] = cout[l - 1];                                  // conv.layer{l}.bias
    sz[s++] = bn * cout[l - 1];                             // conv.bn{l}.weight
    sz[s++] = bn * cout[l - 1];                             // conv.bn{l}.bias
  }
  sz[s++] = D * fc_in(d);  // conv.fc.weight [d][d] or, res towers, [d][4H + d]
  sz[s++] = D;      // conv.fc.bias
  sz[s++] = E * E;  // user_embd.linear1.weight
  sz[s++] = E;
  sz[s++] = D * E;  // user_embd.linear2.weight
  sz[s++] = D;
  const long CT = st_text(d);  // 0 outside the text tower: empty segments
  sz[s++] = CT * d->word_dim * 3;  // text.conv.weight [C_s][E_w][3]
  sz[s++] = CT;                    // text.conv.bias
}

void param_offsets(const dcue_dims* d, int64_t* off) {
  long sz[kSeg];
  param_sizes(d, sz);
  long o = 0;
  for (int s = 0; s < kSeg; ++s) {
    off[s] = o;
    o = al4(o + sz[s]);
  }
  off[kSeg] = o;
}

int bn_channels(const dcue_dims* d, int l) {
  return l == 0 ? kMels : l == 5 ? st_feature(d) : st_hidden(d);
}

void bn_offsets(const dcue_dims* d, int64_t* off) {
  long o = 0;
  for (int l = 0; l < DCUE_N_BN; ++l) {
    off[2 * l] = o;
    o = al4(o + bn_channels(d, l));
    off[2 * l + 1] = o;
    o = al4(o + bn_channels(d, l));
  }
  off[2 * DCUE_N_BN] = o;
}

long wpack_offset(const dcue_dims* d, int l, bool bwd) {
  const WpackLayout wl = wpack_layout(d);
  return bwd ? wl.conv_bwd[l] : wl.conv_fwd[l];
}

// pointers into the caller's workspace
struct Ws {
  float* counts;
  int32_t *copy_ptr, *copy_idx;  // gather layout: per-item copy lists (StepPrologue), M <= kCopyListMaxItems
  float *mean[6], *invstd[6], *a[6];
  float* bcp[6];  // the step's BN betas as the forward used them (BnPublish::beta_out)
  // exact BN sums (bnacc.h), [6 layers][2 sums][Cmax][2 words]: forward stats, backward sums
  unsigned long long *bnacc, *bnbacc;
  // the forward's value ranges (split-f16 operand scales, conv_rows.h / conv_wgrad.hip): [6 layers]
  // [2][kRngC] ordered keys, between the forward and backward sums of the block (cleared with the
  // forward sums); the backward's gradient maxima [7][kRngC] (max |g_l| for l = 1..5, max |df| at 6)
  // after the backward sums (cleared with them)
  unsigned* rng;
  unsigned* grng;
  long nzero;            // words of the accumulator block (one clear per step)
  long nfwd;             // its forward part: the sums and the ranges
  float* rowsum;         // [B] per-row hinge sums (score_fused)
  int cmax;
  float* y[6];
  uint8_t* idx[6];
  float *f, *uf, *h1;
  float *cosv, *norms, *hinge, *scores, *loss, *dhinge;
  float *du, *dfcopy, *df;
  float* g[6];
  float *dh1, *de;
  float *wpart[3], *bpart[3], *G, *S;  // wgrad partials: one set per wgrad stream
  float *wpm[5], *bpm[5];                // k_conv_wgrad_multi's partials, layers 2..5 and the fc
  float* xhat0;          // [M][kXp][128] bn0-normalised, zero-padded input: conv-1 wgrad's X operand
  float* dx1;            // [M][33][H] BN1 backward at the pooled positions: conv-1 wgrad's dz operand
  // towers without BN: the BN operands every kernel reads become the identity (mean 0, a = invstd
  // = 1, beta 0) and the BN parameter gradients go to a scratch sink
  float *ones, *zeros, *sink;
  // res towers: the fc input [M][4H + d] (time-pooled blocks 1-4, then block 5) and the gradient
  // of the four time-pooled outputs [M][4H]; text tower: the fc input [M][text_dim + d] (text
  // features, then block 5) and the text features' gradient [M][C_s]
  float *xfc, *dtp;
  uint8_t* tidx;  // text tower: [M][C_s] the max-over-positions argmax (255: no gradient)
  // text tower: the forward's position-part merge (TextBranch::ticket / part): tickets in the
  // accumulator block's forward part (ntick 64-bit words, cleared with it), maxima [M][2][C_s]
  unsigned* tticket;
  unsigned long long* tpart;
  long ntick;
  float* twpart;  // text tower: the text conv's weight-gradient chunk partials
};

// the accumulator block's parts: [6][2][Cmax][2] forward sums, then the same for the backward
constexpr long kRngWords = 6L * 2 * kRngC / 2;   // the ranges' 64-bit words
constexpr long kGrngWords = 7L * kRngC / 2 + 64;  // the gradient maxima's (+ padding to keep 16-B alignment)

void rebase_acc(Ws* w, unsigned long long* acc) {
  w->bnacc = acc;
  w->rng = reinterpret_cast<unsigned*>(acc + 6L * 2 * w->cmax * 2);
  w->tticket = w->ntick ? reinterpret_cast<unsigned*>(acc + 6L * 2 * w->cmax * 2 + kRngWords) : nullptr;
  w->bnbacc = acc + 6L * 2 * w->cmax * 2 + kRngWords + w->ntick;
  w->grng = reinterpret_cast<unsigned*>(w->bnbacc + 6L * 2 * w->cmax * 2);
}

// layer l's range (l = 0: the raw input of conv 1; l = 1..5: the ReLU output of conv l)
unsigned* rng_at(const Ws& w, int l) { return w.rng + (size_t)l * 2 * kRngC; }
// max |g_l| per channel (l = 1..5), max |df| (l = 6)
unsigned* grng_at(const Ws& w, int l) { return w.grng + (size_t)l * kRngC; }

size_t carve(const dcue_dims* d, int B, int N, int M, void* base, Ws* w) {
  Arena ar{(char*)base, 0, 0};
  const int H = st_hidden(d), D = st_feature(d), E = d->user_embdim;
  const int Cmax = H > kMels ? H : kMels;
  w->counts = ar.take<float>(M);
  w->copy_ptr = ar.take<int32_t>(M + 1);
  w->copy_idx = ar.take<int32_t>((long)B * (N + 1));
  for (int l = 0; l < 6; ++l) {
    const int C = bn_channels(d, l);
    w->mean[l] = ar.take<float>(C);
    w->invstd[l] = ar.take<float>(C);
    w->a[l] = ar.take<float>(C);
    w->bcp[l] = ar.take<float>(C);
  }
  w->cmax = Cmax > D ? Cmax : D;
  // text tower: one 32-bit ticket per (item, column block of >= 64 columns), in 16-B units
  w->ntick = tower_text(d) ? ((long)M * (st_text(d) / 64) + 3) / 4 * 2 : 0;
  w->nfwd = 6L * 2 * w->cmax * 2 + kRngWords + w->ntick;
  w->nzero = w->nfwd + 6L * 2 * w->cmax * 2 + kGrngWords;
  w->bnacc = ar.take<unsigned long long>(w->nzero);
  rebase_acc(w, w->bnacc);
  w->rowsum = ar.take<float>(B);
  w->y[0] = nullptr;
  w->idx[0] = nullptr;
  for (int l = 1; l <= 5; ++l) {
    const long n = (long)M * layer_geom(l).lp * (l == 5 ? D : H);
    w->y[l] = ar.take<float>(n);
    w->idx[l] = ar.take<uint8_t>(n);
  }
  w->f = ar.take<float>((long)M * D);
  w->uf = ar.take<float>((long)B * D);
  w->h1 = ar.take<float>((long)B * E);
  w->cosv = ar.take<float>((long)B * (N + 1));
  w->norms = ar.take<float>((long)B * (N + 2));
  w->hinge = ar.take<float>((long)B * (N > 0 ? N : 1));
  w->scores = ar.take<float>((long)B * (N > 0 ? N : 1));
  w->loss = ar.take<float>(4);
  w->dhinge = ar.take<float>((long)B * (N > 0 ? N : 1));
  w->du = ar.take<float>((long)B * D);
  w->dfcopy = ar.take<float>((long)B * (N + 1) * D);
  w->df = ar.take<float>((long)M * D);
  w->g[0] = nullptr;
  for (int l = 1; l <= 5; ++l) w->g[l] = ar.take<float>((long)M * layer_geom(l).lp * (l == 5 ? D : H));
  w->dh1 = ar.take<float>((long)B * E);
  w->de = ar.take<float>((long)B * E);
  long wp = 0, bp = 0;
  for (int l = 1; l <= 5; ++l) {
    const int cin = l == 1 ? kMels : H, cout = l == 5 ? D : H;
    const long nch = wgrad_nchunk(l, M, cout, cin);
    const long e = nch * cout * cin * layer_geom(l).ks;
    if (e > wp) wp = e;
    if (nch * 5 * cout > bp) bp = nch * 5 * cout;
  }
  for (int i = 0; i < 3; ++i) {
    w->wpart[i] = ar.take<float>(wp);
    w->bpart[i] = ar.take<float>(bp);
  }
  for (int l = 2; l <= 6; ++l) {  // 6: the fc layer (a 1x1 conv over bn5(y5), D -> D)
    const int cin = l == 6 ? D : H, cout = l >= 5 ? D : H;
    const long nch = wgrad_nchunk(l, M, cout, cin);
    w->wpm[l - 2] = ar.take<float>(nch * cout * cin * layer_geom(l == 6 ? 5 : l).ks);
    w->bpm[l - 2] = ar.take<float>(nch * cout);
  }
  w->G = ar.take<float>((long)H * 4 * kMels);
  w->S = ar.take<float>(5L * H);  // the five layer-1 bias partial sums E[5][H]
  w->xhat0 = ar.take<float>((long)(M + 1) * kXp * kMels);  // + a zero item
  w->dx1 = ar.take<float>((long)M * layer_geom(1).lp * H);
  w->ones = w->zeros = w->sink = w->xfc = w->dtp = w->twpart = nullptr;
  w->tidx = nullptr;
  w->tpart = nullptr;
  if (!tower_has_bn(d)) {
    w->ones = ar.take<float>(w->cmax);
    w->zeros = ar.take<float>(w->cmax);
    w->sink = ar.take<float>(2L * w->cmax);
  }
  if (tower_res(d)) {
    w->xfc = ar.take<float>((long)M * fc_in(d));
    w->dtp = ar.take<float>((long)M * 4 * d->conv_hidden);  // the fc input's block columns: reference H
  }
  if (tower_text(d)) {
    const long CT = st_text(d);
    w->xfc = ar.take<float>((long)M * fc_in(d));
    w->dtp = ar.take<float>((long)M * CT);
    w->tidx = ar.take<uint8_t>((long)M * CT);
    w->tpart = ar.take<unsigned long long>((long)M * 2 * CT);
    w->twpart = ar.take<float>((long)text_wgrad_nchunk(M) * (CT * d->word_dim * 3 + CT));
  }
  return ar.used + 256;
}

inline unsigned long long* bn_acc(unsigned long long* base, int cmax, int l) {
  return base + (size_t)l * 2 * cmax * 2;
}

struct Ctx {
  const dcue_model* m;
  int64_t poff[kSeg + 1];
  int64_t boff[2 * DCUE_N_BN + 1];
  int H, D, E;   // storage widths (H, d padded to 32/64/128/256) and E
  int HL;        // the reference's conv_hidden: column width of the res towers' time-pooled blocks
  bool bn, res;  // tower variant (dcue_dims.tower)
  bool text;     // the mixed audio + text tower (text.hip)
  int FI;        // fc input width: D, 4H + D in the res towers, text_dim + D in the text tower
  int off5;      // first fc-input column of bn5(y5)
  int CT;        // text tower: storage channels of the text branch
  const float* P(int seg) const { return m->params + poff[seg]; }
  float* Gd(int seg) const { return m->grads + poff[seg]; }
  float* rmean(int l) const { return m->bn_stats + boff[2 * l]; }
  float* rvar(int l) const { return m->bn_stats + boff[2 * l + 1]; }
  // BN_l's gamma / beta as the kernels read them, and where their gradients go; the identity and a
  // scratch sink in the towers without BN
  const float* gamma(const Ws& w, int l) const;
  const float* beta(const Ws& w, int l) const;
  // the backward's view of BN l's beta: the forward's snapshot (the parameter itself may already be
  // stepping: split plans run Adam over bn1 beside the layer-2 weight gradient that reads it)
  const float* beta_bwd(const Ws& w, int l) const { return bn ? w.bcp[l] : w.zeros; }
  float* dgamma(const Ws& w, int l) const;
  float* dbeta(const Ws& w, int l) const;
};
// segment indices
int seg_bn_w(int l) { return l == 0 ? 0 : 4 + 4 * (l - 1); }
int seg_bn_b(int l) { return l == 0 ? 1 : 5 + 4 * (l - 1); }
const float* Ctx::gamma(const Ws& w, int l) const { return bn ? P(seg_bn_w(l)) : w.ones; }
const float* Ctx::beta(const Ws& w, int l) const { return bn ? P(seg_bn_b(l)) : w.zeros; }
float* Ctx::dgamma(const Ws& w, int l) const { return bn ? Gd(seg_bn_w(l)) : w.sink; }
float* Ctx::dbeta(const Ws& w, int l) const { return bn ? Gd(seg_bn_b(l)) : w.sink + w.cmax; }
int seg_conv_w(int l) { return 2 + 4 * (l - 1); }
int seg_conv_b(int l) { return 3 + 4 * (l - 1); }
constexpr int SEG_FC_W = 22, SEG_FC_B = 23, SEG_L1_W = 24, SEG_L1_B = 25, SEG_L2_W = 26, SEG_L2_B = 27;
constexpr int SEG_TX_W = 28, SEG_TX_B = 29;

int init_ctx(Ctx* c, const dcue_model* m) {
  int st = check_dims(&m->dims);
  if (st) return st;
  if (!m->params || !m->bn_stats || !m->bn_batches || !m->wpack) return DCUE_ERR_INVALID;
  // deferred user-table Adam needs its log, the moments it replays and a valid history capacity
  if (m->emb_step && (!m->emb_log || !m->emb || !m->emb_exp_avg || !m->emb_exp_avg_sq ||
                      m->emb_log_cap < 1 || m->emb_log_cap > DCUE_MAX_LOG_CAP))
    return DCUE_ERR_INVALID;
  c->m = m;
  param_offsets(&m->dims, c->poff);
  bn_offsets(&m->dims, c->boff);
  c->H = st_hidden(&m->dims);
  c->D = st_feature(&m->dims);
  c->HL = m->dims.conv_hidden;
  c->E = m->dims.user_embdim;
  c->bn = tower_has_bn(&m->dims);
  c->res = tower_res(&m->dims);
  c->text = tower_text(&m->dims);
  c->FI = fc_in(&m->dims);
  c->off5 = fc_off5(&m->dims);
  c->CT = st_text(&m->dims);
  if (c->text && (!m->words || m->n_words <= 0)) return DCUE_ERR_INVALID;
  return DCUE_OK;
}

// the text branch's operands (text tower); t->tokens must be set
TextBranch text_branch(const Ctx& c, const dcue_tracks* t) {
  const dcue_dims* d = &c.m->dims;
  TextBranch tb;
  tb.tokens = t->tokens;
  tb.words = c.m->words;
  tb.words_exp = c.m->words_exp;
  tb.wpack16 = c.m->wpack + wpack_layout(d).text_f16;
  tb.bias = c.P(SEG_TX_B);
  tb.T = d->text_len; tb.E = d->word_dim; tb.EP = st_word(d); tb.C = c.CT; tb.Creal = d->text_dim;
  tb.pad = d->text_pad;
  return tb;
}

// ... with the workspace's position-part merge buffers (k_text_fwd_full, DCUE_TEXT_PARTS=2)
TextBranch text_branch_ws(const Ctx& c, const dcue_tracks* t, const Ws& w) {
  TextBranch tb = text_branch(c, t);
  tb.ticket = w.tticket;
  tb.part = w.tpart;
  return tb;
}

// DCUE_SLICE_STREAM: the side stream of the rolling flush slice (0: the user stream; w0 / w1: the
// weight-gradient streams st[1] / st[2])
int slice_stream() {
  static const int v = [] {
    const char* e = getenv("DCUE_SLICE_STREAM");
    return !e ? 0 : (e[0] == 'w' && e[1] == '0') ? 1 : (e[0] == 'w' && e[1] == '1') ? 2 : 0;
  }();
  return v;
}

// DCUE_TEXT_SIDE=0: the training forward's text branch on the caller's stream after conv 5 instead
// of on the user stream beside the audio convs (A/B)
bool text_side_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_TEXT_SIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Item tower forward. train: batch statistics (weighted by counts, accumulated exactly by the
// producing kernels) + running-stat update by each BN's first consumer; eval: running statistics.
int item_forward(const Ctx& c, const Ws& w, const dcue_tracks* t, const int32_t* item_track, int M,
                 double copies, bool train, const float* counts, float* f_out, hipStream_t s,
                 bool acc_cleared = false, bool stats_done = false, bool clear_bn0 = false,
                 hipEvent_t before_l2 = nullptr, const std::function<int()>* after_l1 = nullptr,
                 dcue_comm* sync_bn = nullptr, const std::function<int()>* text_join = nullptr,
                 const DevWait* l2_wait = nullptr) {
  const dcue_model* m = c.m;
  if (c.text && !t->tokens) return DCUE_ERR_INVALID;
  const int src = t->dtype == 0 ? SRC_TRACK_F16 : SRC_TRACK_F32;
  // one BN's finalize/publish record for its first consumer (train) -- bnacc.h
  auto bn_of = [&](int l) {
    BnPublish p = {};
    if (!train || !c.bn) return p;  // eval / no BatchNorm: consumers read the mean / a arrays
    p.acc = bn_acc(w.bnacc, w.cmax, l);
    p.count = copies * (l == 0 ? kFrames : layer_geom(l).lp);
    p.inv_count = 1.0 / p.count;
    p.gamma = c.gamma(w, l);
    p.beta = c.beta(w, l);
    p.mean = w.mean[l]; p.invstd = w.invstd[l]; p.a = w.a[l];
    p.beta_out = w.bcp[l];
    p.rmean = c.rmean(l); p.rvar = c.rvar(l); p.nbt = m->bn_batches + l;
    p.C = bn_channels(&m->dims, l);
    return p;
  };
  // the forward sums and value ranges start cleared (train: by the step prologue, or here). The text
  // branch's position-merge tickets sit at the end of that part; when the branch runs on a side
  // stream (text_join) that stream clears them itself, in its own order (forward_impl), so this
  // clear cannot land between its parts' arrivals
  if (!train || !acc_cleared)
    DCUE_HIP_CHECK(hipMemsetAsync(w.bnacc, 0, sizeof(unsigned long long) * (w.nfwd - (text_join ? w.ntick : 0)), s));
  if (!c.bn) {  // mean 0, invstd = a = 1, beta 0 for every layer: the BN-free towers
    TRY(launch_bn_identity(w.mean, w.invstd, w.a, w.ones, w.zeros, w.cmax, c.H, c.D, s));
    // (the epilogues still add their unused BN sums) the raw input's range, for conv 1's split
    TRY(launch_input_stats(src, t->data, item_track, nullptr, M, nullptr, rng_at(w, 0), s));
  } else if (train) {
    if (clear_bn0 && !stats_done) {  // sums of a batch announced ahead but not the one launched
      DCUE_HIP_CHECK(hipMemsetAsync(bn_acc(w.bnacc, w.cmax, 0), 0, sizeof(unsigned long long) * 2 * w.cmax * 2, s));
      DCUE_HIP_CHECK(hipMemsetAsync(rng_at(w, 0), 0, sizeof(unsigned) * 2 * kRngC, s));
    }
    if (!stats_done)  // else computed one step ahead into this accumulator block (plans)
      TRY(launch_input_stats(src, t->data, item_track, counts, M, bn_acc(w.bnacc, w.cmax, 0), rng_at(w, 0), s));
  } else {
    for (int l = 0; l < 6; ++l)
      TRY(launch_bn_eval(bn_channels(&m->dims, l), c.P(seg_bn_w(l)), c.rmean(l), c.rvar(l), w.mean[l],
                         w.invstd[l], w.a[l], s));
    TRY(launch_input_stats(src, t->data, item_track, nullptr, M, nullptr, rng_at(w, 0), s));
  }
  // SyncBN: each layer's batch sums over every rank before their first consumer (the next launch on
  // this stream finalizes them); the counts are already the global ones (forward_impl)
  const bool sync = train && c.bn && sync_bn;
  if (sync) TRY(comm_allreduce_u64(sync_bn, bn_acc(w.bnacc, w.cmax, 0), 4L * w.cmax, s));
  auto rows_args = [&](int l) {
    RowsArgs a = {};
    a.src = l == 1 ? t->data : (const void*)w.y[l - 1];
    a.item_track = item_track;
    a.in_mean = w.mean[l - 1];
    a.in_a = w.a[l - 1];
    a.in_beta = c.beta(w, l - 1);
    a.in_bn = bn_of(l - 1);
    a.counts = counts;
    a.wpack = m->wpack + wpack_offset(&m->dims, l, false);
    a.wpack16 = reinterpret_cast<const uint4*>(m->wpack + wpack_layout(&m->dims).conv_f16[l]);
    a.bias = c.P(seg_conv_b(l));
    a.out = w.y[l];
    a.out_idx = w.idx[l];
    a.out_acc = train ? bn_acc(w.bnacc, w.cmax, l) : nullptr;
    a.in_range = rng_at(w, l - 1);
    a.out_range = rng_at(w, l);
    a.M = M;
    a.nout = l == 5 ? c.D : c.H;
    if (l == 2 && l2_wait) a.wait = *l2_wait;  // (plans: the previous step's late Adam, on the device)
    if (l == 2 && train) {  // conv 2's input-gradient operands, left by the split plans' late Adam
      a.rp = pack_seg(m, c.poff, 2);
      a.rp.fwd = a.rp.f16 = -1;
      a.rp_src = c.P(seg_conv_w(2));
      a.rp_wpack = m->wpack;
    }
    return a;
  };
  // the fc of the BN tower: f = bn5(y5) W^T + b   (truedcuemel1dbn.py:65,101)
  auto fc_args = [&]() {
    TGemmArgs g = {};
    g.M = M; g.N = c.D; g.K = c.D;
    g.A = w.y[5]; g.sam = c.D; g.sak = 1;
    g.amean = w.mean[5]; g.aa = w.a[5]; g.abeta = c.beta(w, 5);
    g.abn = bn_of(5);
    g.B = c.P(SEG_FC_W); g.sbk = 1; g.sbn = c.D;
    g.bias = c.P(SEG_FC_B);
    g.C = f_out ? f_out : w.f; g.scm = c.D; g.scn = 1;
    return g;
  };
  for (int l = 1; l <= 5; ++l) {
    // the previous step's late-segment Adam (split plans, StepOpts::dense_split) ran on the user
    // stream: conv 2 is the first kernel on this stream to read those parameters
    if (l == 2 && before_l2) TRY(wait_point(s, before_l2));
    if (l == 2 && train) TRY(debug_delay(DCUE_SITE_CONV2, s));
    const RowsArgs a = rows_args(l);
    TimerScope tsc;
    TRY(timer_begin(&tsc, l == 1 ? DCUE_TIMED_CONV1_FWD : -1, s));
    TRY(launch_conv_fwd(l, l == 1 ? kMels : c.H, l == 1 ? src : SRC_ACT, a, s));
    TRY(timer_end(&tsc));
    TRY(probe(PR_Y1 + l - 1, w.y[l], (long)M * layer_geom(l).lp * a.nout, s));
    if (sync) TRY(comm_allreduce_u64(sync_bn, bn_acc(w.bnacc, w.cmax, l), 4L * w.cmax, s));
    if (l == 1 && after_l1) TRY((*after_l1)());
  }
  if (c.res || c.text) {  // fc on [tp1, tp2, tp3, tp4, bn5(y5)] (truedcuemel1dres.py:93-97) or [s, bn5(y5)]
    TRY(launch_timepool(w.y, w.mean, w.a, c.bn ? c.P(seg_bn_b(1)) : nullptr, c.bn ? c.P(seg_bn_b(2)) : nullptr,
                        c.bn ? c.P(seg_bn_b(3)) : nullptr, c.bn ? c.P(seg_bn_b(4)) : nullptr,
                        c.bn ? c.P(seg_bn_b(5)) : nullptr, bn_of(5), M, c.H, c.res ? c.HL : 0, c.D, c.off5,
                        c.FI, w.xfc, s));
    if (c.text && text_join) {  // the text branch ran on a side stream (forward_impl): join it
      TRY((*text_join)());
    } else if (c.text) {
      TimerScope tsc;
      TRY(timer_begin(&tsc, DCUE_TIMED_TEXT_FWD, s));
      TRY(launch_text_fwd(text_branch_ws(c, t, w), item_track, M, w.xfc, c.FI, w.tidx, s));
      TRY(timer_end(&tsc));
    }
    TGemmArgs g = {};
    g.M = M; g.N = c.D; g.K = c.FI;
    g.A = w.xfc; g.sam = c.FI; g.sak = 1;
    g.B = c.P(SEG_FC_W); g.sbk = 1; g.sbn = c.FI;
    g.bias = c.P(SEG_FC_B);
    g.C = f_out ? f_out : w.f; g.scm = c.D; g.scn = 1;
    TRY(launch_tgemm(0, 0, g, s));
    return probe(PR_F, g.C, (long)M * c.D, s);
  }
  // fc on BN5(y5): f = bn5(y5) W^T + b   (truedcuemel1dbn.py:65,101)
  const TGemmArgs g = fc_args();
  TRY(launch_tgemm(2, 0, g, s));
  return probe(PR_F, g.C, (long)M * c.D, s);
}

// user tower (userembedding.py:33-44): h1 = relu(E[u]) W1^T + b1; uf = relu(h1) W2^T + b2
int user_forward(const Ctx& c, const Ws& w, const int64_t* users, int B, float* uf_out, hipStream_t s) {
  const dcue_model* m = c.m;
  TGemmArgs g = {};
  g.M = B; g.N = c.E; g.K = c.E;
  g.A = m->emb; g.sam = c.E; g.sak = 1; g.arow = users;
  g.B = c.P(SEG_L1_W); g.sbk = 1; g.sbn = c.E;
  g.bias = c.P(SEG_L1_B);
  g.C = w.h1; g.scm = c.E; g.scn = 1;
  TRY(launch_tgemm(1, 0, g, s));
  g = TGemmArgs{};
  g.M = B; g.N = c.D; g.K = c.E;
  g.A = w.h1; g.sam = c.E; g.sak = 1;
  g.B = c.P(SEG_L2_W); g.sbk = 1; g.sbn = c.E;
  g.bias = c.P(SEG_L2_B);
  g.C = uf_out ? uf_out : w.uf; g.scm = c.D; g.scn = 1;
  return launch_tgemm(1, 0, g, s);
}

// the same, with the deferred rows' sync in one launch (k_user_fwd): the train forward's user tower;
// sig: the plan's signal word its workgroups add to once uf is stored (DevWait)
int user_forward_fused(const Ctx& c, const Ws& w, const int64_t* users, int B, hipStream_t s,
                       unsigned* sig = nullptr) {
  const dcue_model* m = c.m;
  TGemmArgs g1 = {}, g2 = {};
  g1.M = B; g1.N = c.E; g1.K = c.E;
  g1.A = m->emb; g1.sam = c.E; g1.sak = 1; g1.arow = users;
  g1.B = c.P(SEG_L1_W); g1.sbk = 1; g1.sbn = c.E;
  g1.bias = c.P(SEG_L1_B);
  g1.C = w.h1; g1.scm = c.E; g1.scn = 1;
  g2.M = B; g2.N = c.D; g2.K = c.E;
  g2.A = w.h1; g2.sam = c.E; g2.sak = 1;
  g2.B = c.P(SEG_L2_W); g2.sbk = 1; g2.sbn = c.E;
  g2.bias = c.P(SEG_L2_B);
  g2.C = w.uf; g2.scm = c.D; g2.scn = 1;
  return launch_user_fwd(m, g1, g2, users, B, s, sig);
}

// whether a gather batch gets per-item copy lists (the prologue's histogram path)
bool copy_lists(const dcue_batch* b) {
  return b->layout == DCUE_LAYOUT_GATHER && b->n_items <= kCopyListMaxItems;
}

// counts (+ copy lists) of a batch issued outside a plan: the prologue kernel without draws, so
// eager steps and plan replays sum the item gradients in the same order
int batch_counts(const dcue_batch* b, const Ws& w, hipStream_t s) {
  if (!copy_lists(b)) return launch_item_counts(b, w.counts, s);
  StepPrologue p = {};
  p.B = b->n_rows; p.N = b->n_neg; p.M = b->n_items;
  p.gather = 1;
  p.neg = const_cast<int32_t*>(b->neg_item);
  p.counts = w.counts;
  p.copy_ptr = w.copy_ptr;
  p.copy_idx = w.copy_idx;
  return launch_step_prologue(p, s);
}

int check_batch(const dcue_batch* b) {
  if (!b || !b->users || !b->item_track || b->n_rows <= 0 || b->n_neg < 0 || b->n_items <= 0)
    return DCUE_ERR_INVALID;
  if (b->layout == DCUE_LAYOUT_CATALOGUE) {
    if ((long)b->n_items != (long)b->n_rows * (1 + b->n_neg)) return DCUE_ERR_INVALID;
  } else if (b->layout == DCUE_LAYOUT_GATHER) {
    if (b->n_neg > 0 && !b->neg_item) return DCUE_ERR_INVALID;
    if (b->n_items < b->n_rows) return DCUE_ERR_INVALID;
  } else {
    return DCUE_ERR_INVALID;
  }
  return DCUE_OK;
}

}  // namespace

extern "C" {

int dcue_abi_version(void) { return DCUE_ABI_VERSION; }

int64_t dcue_launch_count(void) { return dcue::g_launches.load(std::memory_order_relaxed); }

int dcue_storage_dims(const dcue_dims* dims, dcue_dims* storage_host) {
  TRY(check_dims(dims));
  if (!storage_host) return DCUE_ERR_INVALID;
  *storage_host = *dims;
  storage_host->conv_hidden = st_hidden(dims);
  storage_host->feature_dim = st_feature(dims);
  return DCUE_OK;
}

int dcue_param_layout(const dcue_dims* dims, int64_t* offsets_host) {
  TRY(check_dims(dims));
  if (!offsets_host) return DCUE_ERR_INVALID;
  param_offsets(dims, offsets_host);
  return DCUE_OK;
}

int dcue_bn_layout(const dcue_dims* dims, int64_t* offsets_host) {
  TRY(check_dims(dims));
  if (!offsets_host) return DCUE_ERR_INVALID;
  bn_offsets(dims, offsets_host);
  return DCUE_OK;
}

int dcue_wpack_floats(const dcue_dims* dims, int64_t* n) {
  TRY(check_dims(dims));
  if (!n) return DCUE_ERR_INVALID;
  *n = wpack_layout(dims).total;
  return DCUE_OK;
}

int dcue_workspace_bytes(const dcue_dims* dims, int32_t max_rows, int32_t max_neg,
                         int32_t max_items, size_t* bytes) {
  TRY(check_dims(dims));
  if (!bytes || max_rows <= 0 || max_neg < 0 || max_items <= 0) return DCUE_ERR_INVALID;
  Ws w;
  *bytes = carve(dims, max_rows, max_neg, max_items, nullptr, &w);
  return DCUE_OK;
}

int dcue_workspace_outputs(const dcue_dims* dims, int32_t B, int32_t N, int32_t M,
                           size_t* offsets_host) {
  TRY(check_dims(dims));
  if (!offsets_host || B <= 0 || N < 0 || M <= 0) return DCUE_ERR_INVALID;
  Ws w;
  carve(dims, B, N, M, nullptr, &w);
  offsets_host[0] = (size_t)w.scores;
  offsets_host[1] = (size_t)w.uf;
  offsets_host[2] = (size_t)w.f;
  offsets_host[3] = (size_t)w.loss;
  return DCUE_OK;
}

int dcue_workspace_activations(const dcue_dims* dims, int32_t B, int32_t N, int32_t M,
                               size_t* offsets_host) {
  TRY(check_dims(dims));
  if (!offsets_host || B <= 0 || N < 0 || M <= 0) return DCUE_ERR_INVALID;
  Ws w;
  carve(dims, B, N, M, nullptr, &w);
  for (int l = 1; l <= 5; ++l) {
    offsets_host[2 * (l - 1)] = (size_t)w.y[l];
    offsets_host[2 * (l - 1) + 1] = (size_t)w.idx[l];
  }
  return DCUE_OK;
}

int dcue_pack_weights(const dcue_model* m, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  TRY(join_user_stream((hipStream_t)stream));
  return launch_pack(m, c.poff, (hipStream_t)stream);
}

int dcue_forward(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                 size_t ws_bytes, int32_t train, float margin, float* scores, float* user_feat,
                 float* item_feat, float* loss, void* stream) {
  // a plan step may leave Adam work on the user stream (its late dense segments, the user table)
  TRY(join_user_stream((hipStream_t)stream));
  TRY(dcue::forward_impl(m, b, t, ws, ws_bytes, train, margin, StepOpts{}, (hipStream_t)stream));
  // the outputs live in the workspace (dcue_workspace_outputs gives their offsets); copies are
  // made only for callers that ask for their own buffers
  Ws w;
  carve(&m->dims, b->n_rows, b->n_neg, b->n_items, ws, &w);
  hipStream_t s = (hipStream_t)stream;
  const int B = b->n_rows, N = b->n_neg, M = b->n_items, D = st_feature(&m->dims);
  if (scores && N > 0) DCUE_HIP_CHECK(hipMemcpyAsync(scores, w.scores, sizeof(float) * B * N, hipMemcpyDeviceToDevice, s));
  if (user_feat) DCUE_HIP_CHECK(hipMemcpyAsync(user_feat, w.uf, sizeof(float) * B * D, hipMemcpyDeviceToDevice, s));
  if (item_feat) DCUE_HIP_CHECK(hipMemcpyAsync(item_feat, w.f, sizeof(float) * (size_t)M * D, hipMemcpyDeviceToDevice, s));
  if (loss) DCUE_HIP_CHECK(hipMemcpyAsync(loss, w.loss, sizeof(float), hipMemcpyDeviceToDevice, s));
  return DCUE_OK;
}

int dcue_train_backward(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                        size_t ws_bytes, const float* dscores, float emb_grad_scale, void* stream) {
  TRY(join_user_stream((hipStream_t)stream));
  return dcue::backward_impl(m, b, t, ws, ws_bytes, dscores, emb_grad_scale, StepOpts{},
                             (hipStream_t)stream);
}

int dcue_dcbr_step(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, const float* target,
                   float* loss, void* ws, size_t ws_bytes, void* stream) {
  // the item tower's train forward, the MSE head and the item tower's backward (dcue.h)
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!b || !t || !t->data || !target || !ws || !m->grads || !b->item_track) return DCUE_ERR_INVALID;
  if (b->layout != DCUE_LAYOUT_CATALOGUE || b->n_neg != 0 || b->n_rows <= 0 || b->n_items != b->n_rows)
    return DCUE_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  TRY(join_user_stream(s));
  Ws w;
  const int M = b->n_items;
  if (carve(&m->dims, M, 0, M, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, M, 0, M, ws, &w);
  TRY(launch_item_counts(b, w.counts, s));
  TRY(item_forward(c, w, t, b->item_track, M, (double)M, true, w.counts, nullptr, s, false, false, false,
                   nullptr));
  TRY(launch_mse_grad(w.f, target, M, m->dims.feature_dim, c.D, w.dfcopy, w.rowsum, w.loss, s));
  if (loss) DCUE_HIP_CHECK(hipMemcpyAsync(loss, w.loss, sizeof(float), hipMemcpyDeviceToDevice, s));
  StepOpts o;
  o.item_only = true;
  return dcue::backward_impl(m, b, t, ws, ws_bytes, nullptr, 1.f, o, s);
}

}  // extern "C"

namespace dcue {

int forward_impl(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
                 int train, float margin, const StepOpts& o, hipStream_t s) {
  Ctx c;
  TRY(init_ctx(&c, m));
  HPROF("capi:1");
  TRY(check_batch(b));
  HPROF("capi:2");
  if (!t || !t->data || !ws || !m->emb) return DCUE_ERR_INVALID;
  if (o.fuse_score && !train) return DCUE_ERR_INVALID;
  Ws w;
  if (carve(&m->dims, b->n_rows, b->n_neg, b->n_items, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, b->n_rows, b->n_neg, b->n_items, ws, &w);
  if (o.acc) rebase_acc(&w, o.acc);
  if (o.counts) w.counts = const_cast<float*>(o.counts);
  if (o.y1) w.y[1] = o.y1;
  // SyncBN: BatchNorm normalises over every rank's copies (same B, N on each rank)
  const double copies = (double)b->n_rows * (1 + b->n_neg) * (o.sync_bn ? comm_world(o.sync_bn) : 1);
  SidePool* sp = side_pool();
  if (!sp) return DCUE_ERR_HIP;
  hipStream_t su = sp->st[0];
  // the user tower runs beside the item tower; the item tower's chain is issued first
  hipEvent_t ev_in = o.ev_in;
  if (!ev_in) TRY(fork_point(sp, s, &ev_in));
  HPROF("capi:3");
  if (!o.prologue_done) TRY(batch_counts(b, w, s));
  HPROF("capi:4");
  hipEvent_t ev_uf = nullptr, ev_tx = nullptr;
  const bool text_side = c.text && text_side_on();
  // plans: the score kernel waits for the user tower on the device (DevWait), not by a stream wait
  const bool uf_sig = o.sig != nullptr && !capturing_step();
  static const bool split_fwd = [] {  // DCUE_USER_FWD=split: k_emb_sync + two k_tgemm (A/B)
    const char* e = getenv("DCUE_USER_FWD");
    return e && e[0] == 's';
  }();
  DevWait uf_wait{};
  // the fused launch signals from its own workgroups; the three-launch form through k_signal
  if (uf_sig)
    uf_wait = DevWait{o.sig + kSigUf, o.sig_issued[kSigUf] += split_fwd ? 1u : (unsigned)user_fwd_blocks(b->n_rows),
                      user_fwd_fail_flag()};
  // the user tower on su: emb rows brought up to date, then the two GEMMs (+ the text branch, the
  // rolling flush slice)
  const std::function<int()> user_part = [&]() -> int {
    TRY(wait_point(su, ev_in));
    HPROF("capi:5");
    TRY(debug_delay(DCUE_SITE_USER_FWD, su));
    // The rows' sync and the two GEMMs in one launch (k_user_fwd); DCUE_USER_FWD=split issues them
    // as three (k_emb_sync, one workgroup per row, then two k_tgemm) -- A/B and the schedule test.
    // (Round 4 made the fused form opt-in after non-finite runs; their cause was the plan's
    // cross-stream races, DESIGN.md §4.7 round 5, tests/test_gpu_races.py.)
    unsigned* const ufs = uf_sig && !split_fwd ? o.sig + kSigUf : nullptr;
    TimerScope tsu;  // (the fused launch is timed live: DCUE_TIMED_USER_FWD)
    TRY(timer_begin(&tsu, split_fwd ? -1 : DCUE_TIMED_USER_FWD, su));
    if (tsu.b && !tsu.capturing) {  // a timed launch: the timer's stop event is its end
      TRY(user_forward_fused(c, w, b->users, b->n_rows, su, ufs));
      ev_uf = tsu.b;
      TRY(timer_end(&tsu));
    } else {  // (untimed, or a captured plan: its timer node follows the launch)
      ForkAfter fk(sp, su, &ev_uf);
      if (split_fwd) {
        if (m->emb_step) TRY(launch_emb_sync(m, b->users, b->n_rows, su));
        TRY(user_forward(c, w, b->users, b->n_rows, nullptr, su));
      } else {
        TRY(user_forward_fused(c, w, b->users, b->n_rows, su, ufs));
      }
      HPROF("capi:7");
      TRY(fk.done());
      HPROF("capi:8");
      TRY(timer_end(&tsu));
    }
    if (uf_sig && split_fwd) TRY(launch_signal(o.sig + kSigUf, uf_wait.val, su));
    TRY(probe(PR_H1, w.h1, (long)b->n_rows * c.E, su));
    TRY(probe(PR_UF, w.uf, (long)b->n_rows * c.D, su));
    if (text_side) {  // the text branch: the item tower's fc input columns [0, C_s), beside its convs
      // on wgrad stream 1 (the user stream holds the user tower's ≈65 µs): after the launch's start
      // point (the items) and the previous step's late Adam (its weights); the previous step's text
      // weight gradient, which read xfc / tidx, ran on this same stream
      hipStream_t stx = sp->st[2];
      TRY(wait_point(stx, ev_in));
      if (o.wait_late) TRY(wait_point(stx, o.wait_late));
      // the position-merge tickets: cleared by the step prologue (plans, before ev_in), else here --
      // item_forward's clear on the caller's stream leaves them out
      if (!(train && o.prologue_done) && w.ntick)
        DCUE_HIP_CHECK(hipMemsetAsync(w.tticket, 0, sizeof(unsigned long long) * w.ntick, stx));
      TRY(debug_delay(DCUE_SITE_TEXT_FWD, stx));
      TimerScope tsc;
      TRY(timer_begin(&tsc, DCUE_TIMED_TEXT_FWD, stx));
      if (tsc.b && !tsc.capturing) {  // a timed launch: the timer's stop event is its end
        TRY(launch_text_fwd(text_branch_ws(c, t, w), b->item_track, b->n_items, w.xfc, c.FI, w.tidx, stx));
        ev_tx = tsc.b;
      } else {
        ForkAfter fk(sp, stx, &ev_tx);
        TRY(launch_text_fwd(text_branch_ws(c, t, w), b->item_track, b->n_items, w.xfc, c.FI, w.tidx, stx));
        TRY(fk.done());
      }
      TRY(timer_end(&tsc));
    }
    static const bool skip_slice = [] {  // DCUE_SLICE_SKIP=1: timing diagnostic only (wrong table)
      const char* e = getenv("DCUE_SLICE_SKIP");
      return e && e[0] == '1';
    }();
    if (o.flush_slice_step >= 0 && m->emb_step && !skip_slice) {
      // DCUE_SLICE_STREAM=w1 / w0: the slice on a weight-gradient stream, after this user tower (its
      // rows' claims) and before the step's user-table Adam (which waits for *slice_done): a long
      // slice then holds no user-stream work behind it (A/B)
      const int ss = slice_stream();
      if (ss > 0 && o.slice_done) {
        hipEvent_t e_u = nullptr;
        TRY(fork_point(sp, su, &e_u));
        TRY(wait_point(sp->st[ss], e_u));
        ForkAfter fk(sp, sp->st[ss], o.slice_done);
        TRY(launch_emb_flush_rows(m, o.flush_slice_step, sp->st[ss]));
        TRY(fk.done());
      } else {
        TRY(launch_emb_flush_rows(m, o.flush_slice_step, su));
      }
    }
    return DCUE_OK;
  };
  // DCUE_USER_EARLY=1: the user tower is issued right after conv 1 instead of after the whole item
  // tower, so the host's issue order does not hold it behind four conv launches (A/B knob)
  static const bool early = [] {
    const char* e = getenv("DCUE_USER_EARLY");
    return e && e[0] == '1';
  }();
  // with the side-issue thread (side.hip) the user tower is issued there, beside the item tower's issue
  SideQueue side;
  int ust = DCUE_OK;
  const uint64_t useq = side.threaded() ? side.run(user_part, &ust) : 0;
  // (under an exchange the late Adam follows the all-reduce: it keeps its wait before conv 2)
  const bool late_first = o.wait_late && late_wait_at_conv1() && !o.comm;
  if (late_first) TRY(wait_point(s, o.wait_late));
  // the fc waits for the text branch: its launch issued (the side thread's part done), then its end
  const std::function<int()> text_join = [&]() -> int {
    if (!early && !side.threaded()) TRY(user_part());
    TRY(side.wait(useq));
    return wait_point(s, ev_tx);
  };
  bool user_done = false;
  if (text_side) user_done = !early || side.threaded();  // (text_join issues the user part)
  // conv 2's wait for the previous step's late Adam: on the device when the plan signals it
  const bool l2_dev = o.late_wait.flag != nullptr && !late_first && !capturing_step();
  TRY(item_forward(c, w, t, b->item_track, b->n_items, copies, train != 0, w.counts, nullptr, s,
                   o.prologue_done, o.input_stats_done && o.prologue_done, o.clear_bn0,
                   late_first || l2_dev ? nullptr : o.wait_late,
                   early && !side.threaded() ? &user_part : nullptr, o.sync_bn,
                   text_side ? &text_join : nullptr, l2_dev ? &o.late_wait : nullptr));
  if (!early && !side.threaded() && !user_done) TRY(user_part());
  TRY(side.wait(useq));
  if (!uf_sig) TRY(wait_point(s, ev_uf));
  HPROF("capi:9");
  if (o.fuse_score) {
    // a fork point after the score kernel only for a caller that asks for one: a launch-bound event
    // costs the chain a ≈6 µs gap before its next kernel (the backward's side work waits for the
    // dgrad chain's first fork point instead)
    const int B = b->n_rows, N = b->n_neg;
    auto probes = [&]() -> int {
      TRY(probe(PR_SCORES, w.scores, (long)B * N, s));
      TRY(probe(PR_DU, w.du, (long)B * c.D, s));
      return probe(PR_DFCOPY, w.dfcopy, (long)B * (N + 1) * c.D, s);
    };
    if (!o.score_done) {
      TRY(launch_score_fused(w.uf, w.f, b, c.D, margin, w.scores, w.cosv, w.norms, w.rowsum, w.du,
                             w.dfcopy, s, uf_wait));
      return probes();
    }
    hipEvent_t ev = nullptr;
    ForkAfter fk(sp, s, &ev);
    TRY(launch_score_fused(w.uf, w.f, b, c.D, margin, w.scores, w.cosv, w.norms, w.rowsum, w.du,
                           w.dfcopy, s, uf_wait));
    TRY(fk.done());
    HPROF("capi:10");
    *o.score_done = ev;
    return probes();
  }
  if (uf_sig) return DCUE_ERR_INVALID;  // (device waits: plans, which fuse the score backward)
  return launch_score_fwd(w.uf, w.f, b, c.D, margin, w.scores, w.cosv, w.norms, w.hinge, w.loss,
                          w.dhinge, s);
}

int ahead_item_inputs(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, const int32_t* items,
                      const float* counts, unsigned long long* acc, float* xhat0, hipStream_t s) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!c.bn) return DCUE_ERR_UNSUPPORTED;  // bn0-free towers have no input statistics to prepare
  Ws w;
  carve(&m->dims, b->n_rows, b->n_neg, b->n_items, nullptr, &w);
  rebase_acc(&w, acc);
  const int src = t->dtype == 0 ? SRC_TRACK_F16 : SRC_TRACK_F32;
  const int M = b->n_items;
  const double copies = (double)b->n_rows * (1 + b->n_neg);
  TRY(launch_input_stats(src, t->data, items, counts, M, bn_acc(w.bnacc, w.cmax, 0), rng_at(w, 0), s));
  if (wgrad_f16_on()) return DCUE_OK;  // the split-f16 conv-1 weight gradient reads the table itself
  return launch_xhat0(src, t->data, items, M, bn_acc(w.bnacc, w.cmax, 0), copies * kFrames, xhat0, s);
}

long step_acc_words(const dcue_dims* d, int B, int N, int M) {
  Ws w;
  carve(d, B, N, M, nullptr, &w);
  return w.nzero;
}

int step_prologue(const dcue_model* m, const dcue_batch* b, void* ws, size_t ws_bytes, dcue_mt_state* mt,
                  const int64_t* users_src, const int32_t* items_src, hipStream_t s) {
  Ws w;
  if (carve(&m->dims, b->n_rows, b->n_neg, b->n_items, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, b->n_rows, b->n_neg, b->n_items, ws, &w);
  StepPrologue p = {};
  p.mt = mt;
  p.B = b->n_rows; p.N = b->n_neg; p.M = b->n_items;
  p.gather = b->layout == DCUE_LAYOUT_GATHER;
  p.neg = const_cast<int32_t*>(b->neg_item);
  p.users_dst = const_cast<int64_t*>(b->users); p.users_src = users_src;
  p.items_dst = const_cast<int32_t*>(b->item_track); p.items_src = items_src;
  p.zero = w.bnacc; p.nzero = w.nzero;
  p.counts = w.counts;
  if (copy_lists(b)) {
    p.copy_ptr = w.copy_ptr;
    p.copy_idx = w.copy_idx;
  }
  return launch_step_prologue(p, s);
}

// Split plans: where the caller's stream waits for the previous step's late Adam (StepOpts::
// wait_late). Default: before conv 2, and for the next step's prepared inputs (StepOpts::
// wait_inputs) before the conv-1 weight gradient. DCUE_LATE_WAIT=conv1: one wait before conv 1, the
// late Adam itself waiting for the inputs on the user stream first -- one barrier gap fewer on the
// chain, but conv 1 then starts behind the previous step's late Adam: 4-5 µs slower per step
// (GPU-only A/B, profiles/r04_ab_late_wait.txt).
bool late_wait_at_conv1() {
  static const bool on = [] {
    const char* e = getenv("DCUE_LATE_WAIT");
    return e && e[0] == 'c' && e[4] == '1';
  }();
  return on;
}

static bool fuse_late_adam_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_FUSE_LATE_ADAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// DCUE_FORK_ONCE=1: one fork point on the dgrad chain (after dgrad 3) for both weight-gradient
// launches instead of two (A/B diagnostic: each launch-bound event costs the chain a gap)
static bool fork_once() {
  static const bool on = [] {
    const char* e = getenv("DCUE_FORK_ONCE");
    return e && e[0] == '1';
  }();
  return on;
}

int backward_impl(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
                  const float* dscores, float emb_grad_scale, const StepOpts& o, hipStream_t s) {
  Ctx c;
  TRY(init_ctx(&c, m));
  HPROF("capi:11");
  if (!o.item_only) TRY(check_batch(b));
  HPROF("capi:12");
  if (!t || !t->data || !ws || !m->grads) return DCUE_ERR_INVALID;
  if (!o.item_only && (!m->emb_grad || !m->emb_slot)) return DCUE_ERR_INVALID;
  Ws w;
  if (carve(&m->dims, b->n_rows, b->n_neg, b->n_items, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, b->n_rows, b->n_neg, b->n_items, ws, &w);
  if (o.acc) rebase_acc(&w, o.acc);
  if (o.counts) w.counts = const_cast<float*>(o.counts);
  if (o.y1) w.y[1] = o.y1;
  const int B = b->n_rows, N = b->n_neg, M = b->n_items;
  const int H = c.H, D = c.D, E = c.E;
  const double copies = (double)B * (1 + N) * (o.sync_bn ? comm_world(o.sync_bn) : 1);  // (SyncBN: global)
  const bool sync = o.sync_bn && c.bn;
  const int bn_world = sync ? comm_world(o.sync_bn) : 0;
  const int src = t->dtype == 0 ? SRC_TRACK_F16 : SRC_TRACK_F32;
  if (o.fuse_score && dscores) return DCUE_ERR_INVALID;
  // the item gradients' copy lists: the plan's (current slot), else the workspace's (eager steps and
  // graph plans built them in the forward / prologue)
  const int32_t* cptr = o.copy_ptr ? o.copy_ptr : (copy_lists(b) ? w.copy_ptr : nullptr);
  const int32_t* cidx = o.copy_ptr ? o.copy_idx : (copy_lists(b) ? w.copy_idx : nullptr);
  if (o.emb_adam && (o.emb_adam->parts & ~DCUE_ADAM_EMBEDDING)) return DCUE_ERR_INVALID;
  SidePool* sp = side_pool();
  if (!sp) return DCUE_ERR_HIP;
  hipStream_t su = sp->st[0], sw[2] = {sp->st[1], sp->st[2]};

  // Host issue order follows the critical path: the main stream's chain (item grads -> fc -> the
  // dgrad chain) is enqueued first, recording a fork point before each layer; the side streams'
  // work (user tower, fc weight gradient, per-layer weight gradients) is enqueued afterwards
  // against those recorded points, so issuing it never delays the chain.
  if (!o.prologue_done)  // the backward sums and the gradient maxima
    DCUE_HIP_CHECK(hipMemsetAsync(w.bnbacc, 0, sizeof(unsigned long long) * (6 * 2 * w.cmax * 2 + kGrngWords), s));
    HPROF("capi:13");
  if (!o.fuse_score && !o.item_only)  // else the fused score kernel (or the MSE head) produced dfcopy
    TRY(launch_score_bwd(w.uf, w.f, b, D, dscores ? dscores : w.dhinge, w.cosv, w.norms, w.du,
                         w.dfcopy, s));
  // fork points on the chain are bound to its launches (ForkAfter): no record packets between them
  // ev_score: after the score backward, for the xhat0 build of the f32 weight-gradient path only
  // (the user tower's backward waits for the dgrad chain's first fork point, ev_layer[3])
  hipEvent_t ev_score = nullptr, ev_layer[6] = {};
  if (o.fuse_score && o.score_done && *o.score_done)
    ev_score = *o.score_done;
  else if (!o.xhat0 && !wgrad_f16_on())
    TRY(fork_point(sp, s, &ev_score));
    HPROF("capi:14");
  // the conv-1 weight gradient's X operand, bn0(x) without gamma/beta, materialised once beside the
  // backward chain (it needs only the forward's input statistics); waited for just before that kernel
  hipEvent_t ev_x0 = nullptr;
  const bool f16w = wgrad_f16_on();  // split-f16 weight gradients (conv_wgrad.hip)
  // split plans: Adam over bn0 / conv 1 / bn1 rides in the bn0-gradient launch (adam.hip
  // k_bn0_grads_adam) instead of a launch of its own behind it (DCUE_FUSE_LATE_ADAM=0: separate);
  // not under an exchange, whose Adam must wait for the all-reduced gradient
  const bool fuse_late = o.dense_split && !o.comm && o.dense_split->grad_div <= 1.0 && fuse_late_adam_on();
  // the largest copy count of an item (in-batch: a positive drawn by every other row), the
  // split-f16 dz bounds' kD factor
  const double kd_max = b->layout == DCUE_LAYOUT_GATHER ? 1.0 + (double)B * N : 1.0;
  const float* xhat0 = o.xhat0 ? o.xhat0 : w.xhat0;  // prepared one step ahead (plans), or built here
  if (!o.xhat0 && !f16w) {
    TRY(wait_point(sw[1], ev_score));
    ForkAfter fk(sp, sw[1], &ev_x0);
    TRY(launch_xhat0(src, t->data, b->item_track, M, c.bn ? bn_acc(w.bnacc, w.cmax, 0) : nullptr,
                     copies * kFrames, w.xhat0, sw[1]));
    TRY(fk.done());
  }
  if (c.text && !t->tokens) return DCUE_ERR_INVALID;
  hipEvent_t tail[4] = {};  // caller's stream, user stream, wgrad streams 0 and 1
  // user tower (userembedding.py:33-44 backward), the compact embedding rows, and -- when the step
  // carries it -- the user table's Adam step (it needs nothing from the item tower)
  auto user_bwd = [&]() -> int {
    TRY(wait_point(su, ev_score ? ev_score : ev_layer[3]));
    HPROF("capi:26");
    TRY(debug_delay(DCUE_SITE_USER_BWD, su));
    {
      // two launches of two independent GEMMs each (launch_tgemm_pair; the same blocks as four
      // launch_tgemm calls, so the same bits): (dW2, dh1) from du, then (dW1, de) from dh1
      TGemmArgs g = {}, h = {};
      // dW2[n][k] = sum_b du[b][n] relu(h1)[b][k]; db2[n] = sum_b du[b][n]
      g.M = D; g.N = E; g.K = B;
      g.A = w.du; g.sam = 1; g.sak = D;
      g.B = w.h1; g.sbk = E; g.sbn = 1;
      g.C = c.Gd(SEG_L2_W); g.scm = E; g.scn = 1;
      g.rowsum = c.Gd(SEG_L2_B);
      // dh1 = (du W2) * (h1 > 0)
      h.M = B; h.N = E; h.K = D;
      h.A = w.du; h.sam = D; h.sak = 1;
      h.B = c.P(SEG_L2_W); h.sbk = E; h.sbn = 1;
      h.C = w.dh1; h.scm = E; h.scn = 1;
      h.cmask = w.h1; h.smm = E; h.smn = 1;
      TRY(launch_tgemm_pair(g, h, su));
      HPROF("capi:28");
      // dW1[n][k] = sum_b dh1[b][n] relu(E[u_b])[k]; db1[n] = sum_b dh1[b][n]
      g = TGemmArgs{};
      g.M = E; g.N = E; g.K = B;
      g.A = w.dh1; g.sam = 1; g.sak = E;
      g.B = m->emb; g.sbk = E; g.sbn = 1; g.brow = b->users;
      g.C = c.Gd(SEG_L1_W); g.scm = E; g.scn = 1;
      g.rowsum = c.Gd(SEG_L1_B);
      // de = (dh1 W1) * (E[u_b] > 0)
      h = TGemmArgs{};
      h.M = B; h.N = E; h.K = E;
      h.A = w.dh1; h.sam = E; h.sak = 1;
      h.B = c.P(SEG_L1_W); h.sbk = E; h.sbn = 1;
      h.C = w.de; h.scm = E; h.scn = 1;
      h.cmask = m->emb; h.smm = E; h.smn = 1; h.cmrow = b->users;
      TRY(launch_tgemm_pair(g, h, su));
      HPROF("capi:30");
    }
    // the step's end joins the user stream here: its Adam part (and the rolling flush slice) below
    // needs nothing more from this step and runs on into the next one, ordered on this stream
    // deferred user-table Adam with the step (plans): the compact rows and their Adam step in one
    // launch (k_emb_grad_adam: each distinct user's workgroup sums its rows, then steps them)
    const bool emb_fused = o.emb_adam && m->emb_step && o.defer_flush_slice;
    if (o.slice_done && *o.slice_done) TRY(wait_point(su, *o.slice_done));  // (a slice off this stream)
    {
      ForkAfter fk(sp, su, &tail[1]);
      if (emb_fused)
        TRY(launch_emb_grad_adam(m, o.emb_adam, w.de, b->users, B, emb_grad_scale, su));
      else
        TRY(launch_emb_grad(w.de, b->users, B, E, emb_grad_scale, m->emb_grad, m->emb_slot, m->emb_rows,
                            m->emb_step ? m->emb_log : nullptr, su));
      TRY(fk.done());
      HPROF("capi:31");
    }
    if (probes_on()) {
      TRY(probe(PR_DE, w.de, (long)B * E, su));
      TRY(probe(PR_G_USER, c.Gd(SEG_L1_W), c.poff[SEG_L2_B + 1] - c.poff[SEG_L1_W], su));
    }
    if (o.emb_adam && !emb_fused) TRY(launch_adam(m, o.emb_adam, c.poff, su, !o.defer_flush_slice));
    HPROF("capi:32");
    return DCUE_OK;
  };

  // fc weight gradient of the res / text towers: dW[n][k] = sum_m df[m][n] xfc[m][k], db = sum df over the
  // concatenated fc input (the other towers' fc rides in the layer 3-5 launch, below)
  auto fc_text_wgrad = [&]() -> int {
    TRY(wait_point(sw[1], ev_layer[5]));
    HPROF("capi:23");
    TRY(debug_delay(DCUE_SITE_FC_WGRAD, sw[1]));
    TGemmArgs g = {};
    g.M = D; g.N = c.FI; g.K = M;
    g.A = w.df; g.sam = 1; g.sak = D;
    g.C = c.Gd(SEG_FC_W); g.scm = c.FI; g.scn = 1;
    g.rowsum = c.Gd(SEG_FC_B);
    g.B = w.xfc; g.sbk = c.FI; g.sbn = 1;
    TRY(launch_tgemm(0, 0, g, sw[1]));
    HPROF("capi:24");
    // the text conv's weight and bias gradients (the max routes each gradient to one position)
    if (c.text)
      TRY(launch_text_wgrad(text_branch(c, t), b->item_track, M, w.dtp, w.tidx, w.twpart, c.Gd(SEG_TX_W),
                            c.Gd(SEG_TX_B), sw[1]));
    if (probes_on()) {
      TRY(probe(PR_G_FC, c.Gd(SEG_FC_W), c.poff[SEG_FC_B + 1] - c.poff[SEG_FC_W], sw[1]));
      if (c.text) TRY(probe(PR_G_FC, c.Gd(SEG_TX_W), c.poff[SEG_TX_B + 1] - c.poff[SEG_TX_W], sw[1]));
    }
    return DCUE_OK;
  };

  // (wgrad of layer l reads g_l, which dgrad l+1 produced: ev_layer[l]) layers 5..3 in one launch
  // on wgrad stream 0 once dgrad 4 is done (beside dgrad 3-2); layer 2 on wgrad stream 1 (behind
  // xhat0 and the fc weight gradient) once dgrad 3 is (beside dgrad 2 and the conv-1 tail); each
  // + one reduce launch.
  auto issue_multi = [&](int lo, int hi, bool with_fc, hipStream_t so, hipEvent_t after, hipEvent_t* tl) -> int {
    TRY(wait_point(so, after));
    TRY(debug_delay(lo == 2 ? DCUE_SITE_WGRAD_2 : DCUE_SITE_WGRAD_HI, so));
    WgradMulti mw = {};
    if (with_fc) {  // fc: dW[n][k] = sum_m df[m][n] bn5(y5)[m][k], db = sum_m df (df final since item_grad)
      const int j = mw.n++;
      mw.layer[j] = 6;
      WgradArgs& wa = mw.a[j];
      wa.xsrc = w.y[5];
      wa.x_mean = w.mean[5]; wa.x_a = w.a[5]; wa.x_beta = c.beta_bwd(w, 5);
      wa.g_l = w.df;
      wa.M = M; wa.cout = D; wa.cin = D;
      wa.wpart = w.wpm[4]; wa.bpart = w.bpm[4];
      if (f16w) {
        wa.x_range = rng_at(w, 5); wa.g_range = grng_at(w, 6);
      }
      mw.nchunk[j] = wgrad_nchunk(6, M, D, D);
      mw.dW[j] = c.Gd(SEG_FC_W);
      mw.db[j] = c.Gd(SEG_FC_B);
    }
    for (int l = hi; l >= lo; --l) {
      const LayerGeom gm = layer_geom(l);
      const int j = mw.n++;
      mw.layer[j] = l;
      WgradArgs& wa = mw.a[j];
      wa.xsrc = w.y[l - 1];
      wa.item_track = b->item_track;
      wa.x_mean = w.mean[l - 1]; wa.x_a = w.a[l - 1]; wa.x_beta = c.beta_bwd(w, l - 1);
      wa.g_l = w.g[l]; wa.y_l = w.y[l]; wa.idx_l = w.idx[l];
      wa.mean_l = w.mean[l]; wa.invstd_l = w.invstd[l]; wa.a_l = w.a[l];
      wa.dz_acc = bn_acc(w.bnbacc, w.cmax, l); wa.dgamma = c.dgamma(w, l); wa.dbeta = c.dbeta(w, l);
      wa.invN = c.bn ? (float)(1.0 / (copies * gm.lp)) : 0.f;
      wa.bn_world = bn_world;
      wa.counts = w.counts;
      wa.M = M; wa.cout = l == 5 ? D : H; wa.cin = H;
      wa.wpart = w.wpm[l - 2]; wa.bpart = w.bpm[l - 2];
      if (f16w) {
        wa.x_range = rng_at(w, l - 1); wa.y_range = rng_at(w, l); wa.g_range = grng_at(w, l);
        wa.kd_max = (float)kd_max * wa.invN;
      }
      mw.nchunk[j] = wgrad_nchunk(l, M, wa.cout, wa.cin);
      mw.dW[j] = c.Gd(seg_conv_w(l));
      mw.db[j] = c.Gd(seg_conv_b(l));
    }
    {
      ForkAfter fk(sp, so, tl);
      TRY(launch_conv_wgrad_multi(mw, so));
      TRY(fk.done());
    }
    if (!probes_on()) return DCUE_OK;
    const int s1 = with_fc ? SEG_FC_B : seg_bn_b(hi);
    return probe(lo == 2 ? PR_G_2 : PR_G_HI, c.Gd(seg_conv_w(lo)), c.poff[s1 + 1] - c.poff[seg_conv_w(lo)], so);
  };

  // the step's end. Split plans: the late segments' Adam (every gradient the side streams made) on the
  // user stream once the two weight-gradient streams' tails are in -- the user stream's own tail is in
  // stream order -- and bn0 / conv 1 / bn1 on this stream behind its conv-1 tail (unless it rode in
  // the bn0-gradient launch); this stream does not wait for the late part (the next forward waits
  // for *late_done before conv 2). Other steps: the join -- wgrad stream 0 collects the user
  // stream's and wgrad stream 1's tails, and the caller's stream waits for it once (each
  // cross-queue wait on a pending event costs the waiting queue ≈4 µs, measured; on the side
  // stream that time is slack, on the caller's it is the step's). DCUE_LATE_JOIN=hop keeps the join
  // in split plans too, for the A/B.
  static const bool hop = [] {
    const char* e = getenv("DCUE_LATE_JOIN");
    return e && e[0] == 'h';
  }();
  // split plans without an exchange: the late Adam on the user stream waits for the prepared inputs
  // and the next launch waits for it before conv 1 (late_wait_at_conv1)
  const bool inputs_via_late = o.dense_split && !o.comm && o.late_done && late_wait_at_conv1();
  hipEvent_t joined = nullptr;
  // plans (split, no exchange): the late Adam also signals the next step's conv 2 (DevWait)
  DevWait late_sig{};
  // The late Adam's signal is a one-lane k_signal after the sweep: every workgroup of the sweep
  // releasing its stores itself (dev_signal_wg, DCUE_LATE_SIG=kernel) costs an L2 writeback each on
  // gfx950 -- 440 of them -- and measured 2-4 us slower per step (profiles/r06_ab_late_signal.txt)
  static const bool late_sig_launch = [] {
    const char* e = getenv("DCUE_LATE_SIG");
    return !(e && e[0] == 'k');
  }();
  if (o.dense_split && !o.comm && o.late_sig && o.sig && !capturing_step()) {
    // (DCUE_LATE_SIG=kernel: the sweep's workgroups signal themselves, k_adam_dense_pack)
    const unsigned nwg = late_sig_launch ? 1u : (unsigned)adam_dense_blocks(c.poff[kSeg] - c.poff[DCUE_SEG_LATE]);
    late_sig = DevWait{o.sig + kSigLate, o.sig_issued[kSigLate] += nwg, user_fwd_fail_flag()};
    *o.late_sig = late_sig;
  }
  dcue_adam_args dense = {};
  if (o.dense_split) {
    dense = *o.dense_split;
    dense.parts = DCUE_ADAM_DENSE;
  }
  const long late = c.poff[DCUE_SEG_LATE];
  auto late_part = [&]() -> int {
    if (!o.dense_split || hop) {
      if (tail[1]) TRY(wait_point(sw[0], tail[1]));
      TRY(wait_point(sw[0], tail[3]));
      TRY(fork_point(sp, sw[0], &joined));
    }
    if (o.dense_split) {
      if (hop) {
        TRY(wait_point(su, joined));
      } else {
        TRY(wait_point(su, tail[2]));
        TRY(wait_point(su, tail[3]));
      }
      // (the dgrad of conv 2 on the caller's stream may still run: this Adam leaves its packed
      // operands to the next forward of conv 2 -- launch_adam defer_dgrad2; DCUE_LEGACY_ORDERS=1
      // restores the round-4 order, the repack here and no wait: the race tests/test_gpu_races.py shows)
      // (recorded by the plan's prologue closure, posted before this one: FIFO on the side thread)
      if (inputs_via_late && o.wait_inputs) TRY(wait_point(su, o.wait_inputs));
      TRY(debug_delay(DCUE_SITE_LATE_ADAM, su));
      {
        ForkAfter fk(sp, su, o.late_done);
        TRY(launch_adam(m, &dense, c.poff, su, true, late, -1, !legacy_orders(),
                        late_sig.flag && !late_sig_launch ? o.sig + kSigLate : nullptr));
        TRY(fk.done());
      }
      if (late_sig.flag && late_sig_launch) TRY(launch_signal(o.sig + kSigLate, late_sig.val, su));
      TRY(probe(PR_P_LATE, m->params + late, c.poff[kSeg] - late, su));
    }
    return DCUE_OK;
  };

  // Side-stream work on the side-issue thread (side.hip) when it runs: each part is posted as soon as
  // the events it waits on are recorded on this thread, and runs beside the chain's issue below.
  // Without it the parts are issued here after the chain, in critical-path order.
  SideQueue side;
  const bool thr = side.threaded();
  int ist = DCUE_OK;
  auto post = [&](std::function<int()> f) -> int {
    side.run(std::move(f), &ist);
    return ist;
  };
  auto multi_hi = [&]() { return issue_multi(3, 5, !c.res && !c.text, sw[0], ev_layer[3], &tail[2]); };
  auto multi_2 = [&]() { return issue_multi(2, 2, false, sw[1], ev_layer[2], &tail[3]); };
  // the user tower's backward needs only the score kernel's du; it and a plan's lookahead are issued
  // at the dgrad chain's first fork point (ev_layer[3]), which the layer 3-5 weight gradients wait
  // for anyway: no extra fork event on the chain
  uint64_t ahead_seq = 0;
  auto after_fork3 = [&]() -> int {
    if (thr && !o.item_only) TRY(post(user_bwd));
    if (o.ahead) {
      const std::function<int(hipEvent_t)>* ah = o.ahead;
      const hipEvent_t e3 = ev_layer[3];
      ahead_seq = side.run([ah, e3]() { return (*ah)(e3); }, &ist);
      TRY(ist);
    }
    return DCUE_OK;
  };
  if (c.res || c.text) {  // df; then the fc input gradient split: g5 = df W[:, off5:] (+ BN5's sums) and
                          // the time-pooled blocks' dtp = df W[:, :4H] (text: the text features' df W[:, :C])
    TRY(launch_item_grad(w.dfcopy, b, D, w.df, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                         o.fuse_score ? w.rowsum : nullptr, w.loss, cptr, cidx, nullptr, grng_at(w, 6), s));
    TGemmArgs g = {};
    g.M = M; g.N = D; g.K = D;
    g.A = w.df; g.sam = D; g.sak = 1;
    g.B = c.P(SEG_FC_W) + c.off5; g.sbk = c.FI; g.sbn = 1;
    g.C = w.g[5]; g.scm = D; g.scn = 1;
    g.colacc = bn_acc(w.bnbacc, w.cmax, 5); g.xy = w.y[5]; g.xmean = w.mean[5]; g.xinvstd = w.invstd[5];
    g.colmax = grng_at(w, 5);
    TRY(launch_tgemm(0, 0, g, s));
    g = TGemmArgs{};
    g.M = M; g.N = c.off5; g.K = D;
    g.A = w.df; g.sam = D; g.sak = 1;
    g.B = c.P(SEG_FC_W); g.sbk = c.FI; g.sbn = 1;
    g.C = w.dtp; g.scm = c.text ? c.CT : 4 * c.HL; g.scn = 1;
    ForkAfter fk(sp, s, &ev_layer[5]);
    TRY(launch_tgemm(0, 0, g, s));
    TRY(fk.done());
    if (thr) TRY(post(fc_text_wgrad));
  } else {  // per-item feature gradients df, then (same kernel) the fc input gradient g5 = df W and BN5's sums
    // (no fork point here: the fc weight gradient waits with the layer 3-5 weight gradients, below)
    TRY(launch_item_grad(w.dfcopy, b, D, w.df, c.P(SEG_FC_W), w.g[5], bn_acc(w.bnbacc, w.cmax, 5),
                         w.y[5], w.mean[5], w.invstd[5], o.fuse_score ? w.rowsum : nullptr, w.loss,
                         cptr, cidx, grng_at(w, 5), grng_at(w, 6), s));
    HPROF("capi:15");
  }
  if (probes_on()) {
    TRY(probe(PR_DF, w.df, (long)M * D, s));
    TRY(probe(PR_G5, w.g[5], (long)M * D, s));
  }
  if (sync) TRY(comm_allreduce_u64(o.sync_bn, bn_acc(w.bnbacc, w.cmax, 5), 4L * w.cmax, s));
  auto dgrad_args = [&](int l) {
    const LayerGeom gm = layer_geom(l);
    RowsArgs ra = {};
    ra.src = w.g[l]; ra.y_l = w.y[l]; ra.idx_l = w.idx[l];
    ra.mean_l = w.mean[l]; ra.invstd_l = w.invstd[l]; ra.a_l = w.a[l];
    ra.dz_acc = bn_acc(w.bnbacc, w.cmax, l);
    ra.invN = c.bn ? (float)(1.0 / (copies * gm.lp)) : 0.f;  // 0: BN backward is the identity
    ra.counts = w.counts;
    if (c.res) {  // + d tp_{l-1} / Lp_{l-1} at every position of block l-1 (AvgPool1d backward)
      ra.skip = w.dtp + (l - 2) * c.HL;
      ra.skip_ld = 4 * c.HL;
      ra.skip_n = c.HL;  // storage channels past the reference's H get no skip gradient
      ra.skip_scale = 1.0f / (float)layer_geom(l - 1).lp;
    }
    ra.wpack = m->wpack + wpack_offset(&m->dims, l, true);
    ra.wpack16 = reinterpret_cast<const uint4*>(m->wpack + wpack_layout(&m->dims).conv_f16b[l]);
    // the split-f16 dgrad's dz bound: max |g_l| (the previous dgrad / item gradient), y_l's range
    ra.in_range = grng_at(w, l); ra.y_range = rng_at(w, l);
    ra.kd_max = (float)kd_max * ra.invN;
    ra.out = w.g[l - 1];
    ra.out_acc = bn_acc(w.bnbacc, w.cmax, l - 1);
    ra.oy = w.y[l - 1]; ra.omean = w.mean[l - 1]; ra.oinvstd = w.invstd[l - 1];
    ra.out_grange = grng_at(w, l - 1);  // max |g_{l-1}|: the split-f16 weight gradient's dz bound
    ra.M = M;
    ra.nout = H;
    return ra;
  };
  for (int l = 5; l >= 2; --l) {  // dgrad chain: g_l (+ BN_l sums) -> g_{l-1} (+ BN_{l-1} sums)
    const RowsArgs ra = dgrad_args(l);
    // a fork point only where a side stream waits (wgrads of layers 3-5 after g_3, of layer 2
    // after g_2): every event bound to a launch costs the chain a gap before its next kernel
    if ((l - 1 == 3 && !fork_once()) || l - 1 == 2) {
      ForkAfter fk(sp, s, &ev_layer[l - 1]);
      TRY(launch_conv_dgrad(l, l == 5 ? D : H, ra, s));
      if (sync) {  // the weight gradients forked here read the summed BN_{l-1} sums: the fork point
                   // is recorded after the exchange instead of bound to the launch
        TRY(comm_allreduce_u64(o.sync_bn, bn_acc(w.bnbacc, w.cmax, l - 1), 4L * w.cmax, s));
        launch_tag().missed = true;
      }
      TRY(fk.done());
      if (l - 1 == 3 && !fork_once()) {
        if (thr) TRY(post(multi_hi));
        TRY(after_fork3());
      }
      if (l - 1 == 2) {
        if (fork_once()) {
          ev_layer[3] = ev_layer[2];
          if (thr) TRY(post(multi_hi));
          TRY(after_fork3());
        }
        if (thr) TRY(post(multi_2));
      }
    } else {
      if (l == 2) TRY(debug_delay(DCUE_SITE_DGRAD_2, s));
      TRY(launch_conv_dgrad(l, l == 5 ? D : H, ra, s));
      if (sync) TRY(comm_allreduce_u64(o.sync_bn, bn_acc(w.bnbacc, w.cmax, l - 1), 4L * w.cmax, s));
    }
    TRY(probe(PR_G4 + (5 - l), w.g[l - 1], (long)M * layer_geom(l - 1).lp * H, s));
    HPROF("capi:16");
  }
  // plans: the next step's prepared inputs ordered by the conv-1 weight gradient's device-side wait
  // (k_conv_wgrad16t, DevWait) instead of a stream wait before it
  const bool inputs_dev = o.inputs_wait.flag != nullptr && f16w && !inputs_via_late && !capturing_step();
  // conv weight gradient of layer l on stream `so` (its own split-K partial set `ps`); `tail`:
  // a fork point after its last kernel
  auto issue_wgrad = [&](int l, hipStream_t so, int ps, hipEvent_t* tail) -> int {
    const LayerGeom gm = layer_geom(l);
    const int C = l == 5 ? D : H;
    const int cin = l == 1 ? kMels : H;
    if (so != s) TRY(wait_point(so, ev_layer[l]));
    HPROF("capi:18");
    WgradArgs wa = {};
    // split-f16 kernels: layer 1 reads the track table itself (bn0 applied at the fill), not xhat0
    wa.xsrc = l == 1 ? (f16w ? t->data : (const void*)xhat0) : (const void*)w.y[l - 1];
    wa.item_track = b->item_track;
    wa.x_mean = w.mean[l - 1];
    wa.x_a = l == 1 ? w.invstd[0] : w.a[l - 1];
    wa.x_beta = l == 1 ? nullptr : c.beta_bwd(w, l - 1);
    wa.g_l = w.g[l]; wa.y_l = w.y[l]; wa.idx_l = w.idx[l];
    wa.mean_l = w.mean[l]; wa.invstd_l = w.invstd[l]; wa.a_l = w.a[l];
    wa.dz_acc = bn_acc(w.bnbacc, w.cmax, l); wa.dgamma = c.dgamma(w, l); wa.dbeta = c.dbeta(w, l);
    wa.invN = c.bn ? (float)(1.0 / (copies * gm.lp)) : 0.f;
    wa.bn_world = bn_world;
    wa.counts = w.counts;
    wa.M = M; wa.cout = C; wa.cin = cin;
    wa.wpart = w.wpart[ps]; wa.bpart = w.bpart[ps];
    if (f16w) {
      wa.x_range = rng_at(w, l - 1); wa.y_range = rng_at(w, l); wa.g_range = grng_at(w, l);
      wa.kd_max = kd_max * wa.invN;
    }
    if (l == 1 && inputs_dev) wa.wait = o.inputs_wait;
    const int nch = wgrad_nchunk(l, M, C, cin);
    if (l == 1 && !f16w) {  // the GEMM reads the pooled BN1 backward, expanded to rows at MFMA time
      TRY(launch_conv1_dx(wa, w.dx1, so));
      wa.g_l = w.dx1;
    }
    TimerScope tsc;
    TRY(timer_begin(&tsc, l == 1 ? DCUE_TIMED_CONV1_WGRAD : -1, so));
    HPROF("capi:19");
    TRY(launch_conv_wgrad(l, l == 1 ? src : SRC_ACT, wa, nch, so));
    HPROF("capi:20");
    TRY(timer_end(&tsc));
    HPROF("capi:21");
    if (l != 1) {
      ForkAfter fk(sp, so, tail);
      TRY(launch_wgrad_reduce(l, wa.wpart, wa.bpart, nch, C, cin, c.Gd(seg_conv_w(l)),
                              c.Gd(seg_conv_b(l)), w.G, w.S, so));
      return fk.done();
    }
    TRY(launch_wgrad_reduce(l, wa.wpart, wa.bpart, nch, C, cin, c.Gd(seg_conv_w(l)),
                            c.Gd(seg_conv_b(l)), w.G, w.S, so));
    ForkAfter fk(sp, so, tail);
    const bool graw = f16w && src == SRC_TRACK_F16;  // G over the raw fp16 input (conv_wgrad.hip)
    if (fuse_late) {  // split plans: bn0's gradients and Adam over [0, DCUE_SEG_LATE) in one launch
      Bn0Adam ba;
      ba.md = m; ba.poff = c.poff; ba.args = *o.dense_split; ba.bn = c.bn;
      TRY(launch_bn0_grads_adam(w.G, w.S, c.gamma(w, 0), c.beta(w, 0), graw ? w.mean[0] : nullptr,
                                graw ? w.invstd[0] : nullptr, H, c.dgamma(w, 0), c.dbeta(w, 0), ba, so));
      TRY(fk.done());
      if (!probes_on()) return DCUE_OK;
      TRY(probe(PR_G_1, m->grads, late, so));
      return probe(PR_P_EARLY, m->params, late, so);
    }
    TRY(launch_bn0_grads(w.G, w.S, c.P(seg_conv_w(1)), c.gamma(w, 0), c.beta(w, 0),
                         graw ? w.mean[0] : nullptr, graw ? w.invstd[0] : nullptr, H,
                         c.Gd(seg_conv_w(1)), c.dgamma(w, 0), c.dbeta(w, 0),
                         c.Gd(seg_conv_b(1)), so));
    TRY(fk.done());
    return probe(PR_G_1, m->grads, late, so);
  };
  // layer 1 (the step's tail) follows the chain on the caller's stream, issued right away
  if (ev_x0) TRY(wait_point(s, ev_x0));
  if (o.wait_inputs && !inputs_via_late && !inputs_dev) {
    TRY(side.wait(o.ahead ? ahead_seq : o.wait_inputs_seq));
    TRY(wait_point(s, o.wait_inputs));
  }
  TRY(debug_delay(DCUE_SITE_WGRAD_1, s));
  TRY(issue_wgrad(1, s, 2, &tail[0]));
  HPROF("capi:22");

  if (!thr) {
    if (c.res || c.text) TRY(fc_text_wgrad());
    if (fork_once()) ev_layer[3] = ev_layer[2];
    TRY(multi_hi());
    TRY(multi_2());
    HPROF("capi:25");
    if (!o.item_only) TRY(user_bwd());
    HPROF("capi:32");
  }
  if (o.dense_split && o.comm) {
    // data parallelism, split: each bucket's Adam waits only for its all-reduce (comm_exchange_split):
    // the late segments' (every side stream's gradient) on the comm stream, then bn0 / conv 1 / bn1 on
    // this stream after the early bucket; *late_done (the late Adam) is what the next forward's conv 2
    // waits for, as without an exchange
    TRY(side.drain());
    const long n = c.poff[kSeg];
    const hipEvent_t sides[3] = {tail[1], tail[2], tail[3]};
    hipEvent_t ld = ring_event(sp);
    TRY(comm_exchange_split(o.comm, m, &dense, c.poff, late, n, sides, 3, ld, s));
    if (o.late_done) *o.late_done = ld;
    TRY(launch_adam(m, &dense, c.poff, s, true, 0, late));
    TRY(probe(PR_P_EARLY, m->params, late, s));
    if (o.tails) {  // [1]: the comm stream after the late Adam, which waited for every side stream
      o.tails[0] = tail[0];
      o.tails[1] = ld;
    }
    return DCUE_OK;
  }
  TRY(post(late_part));
  if (o.dense_split) {
    if (!fuse_late) {
      TRY(launch_adam(m, &dense, c.poff, s, true, 0, late));
      TRY(probe(PR_P_EARLY, m->params, late, s));
    }
  } else {
    TRY(side.drain());
    TRY(wait_point(s, joined));
  }
  TRY(side.drain());
  HPROF("capi:36");
  if (o.tails) {  // [1], split steps: the user stream after the late Adam (it waited for the others)
    o.tails[0] = tail[0];
    o.tails[1] = o.dense_split && o.late_done ? *o.late_done : joined;
  }
  return DCUE_OK;
}

}  // namespace dcue

extern "C" {

int dcue_adam_step(const dcue_model* m, const dcue_adam_args* a, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!a || a->step < 1 || (a->parts & ~(DCUE_ADAM_DENSE | DCUE_ADAM_EMBEDDING))) return DCUE_ERR_INVALID;
  const int parts = a->parts ? a->parts : (DCUE_ADAM_DENSE | DCUE_ADAM_EMBEDDING);
  if ((parts & DCUE_ADAM_DENSE) && (!m->grads || !m->exp_avg || !m->exp_avg_sq)) return DCUE_ERR_INVALID;
  if ((parts & DCUE_ADAM_EMBEDDING) &&
      (!m->emb || !m->emb_exp_avg || !m->emb_exp_avg_sq || !m->emb_slot || !m->emb_grad))
    return DCUE_ERR_INVALID;
  if ((parts & DCUE_ADAM_EMBEDDING) && m->emb_step && !m->emb_rows) return DCUE_ERR_INVALID;
  TRY(join_user_stream((hipStream_t)stream));
  TRY(launch_adam(m, a, c.poff, (hipStream_t)stream));
  // the dense sweep repacked the conv weights as it went (k_adam_dense_pack)
  return DCUE_OK;
}

int dcue_optimizer_step(const dcue_model* m, const dcue_opt_args* a, const dcue_opt_state* st, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!a || !st || a->step < 1 || !m->grads || !m->emb || !m->emb_slot) return DCUE_ERR_INVALID;
  if (m->dims.n_users > 0 && !m->emb_grad) return DCUE_ERR_INVALID;
  if (a->kind == DCUE_OPT_SGD) {
    if (!st->dense_a || !st->emb_a) return DCUE_ERR_INVALID;
  } else if (a->kind == DCUE_OPT_RANGER) {
    if (!st->dense_a || !st->dense_b || !st->dense_c || !st->emb_a || !st->emb_b || !st->emb_c || a->k < 1)
      return DCUE_ERR_INVALID;
  } else {
    return DCUE_ERR_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  TRY(join_user_stream(s));
  TRY(launch_opt(m, a, st, c.poff[kSeg], s));
  return launch_pack(m, c.poff, s);
}

int dcue_item_tower_eval(const dcue_model* m, const dcue_tracks* t, const int32_t* item_track,
                         int32_t n_items, void* ws, size_t ws_bytes, float* item_feat,
                         void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!t || !t->data || !item_track || !ws || !item_feat || n_items <= 0) return DCUE_ERR_INVALID;
  Ws w;
  if (carve(&m->dims, 1, 0, n_items, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, 1, 0, n_items, ws, &w);
  TRY(join_user_stream((hipStream_t)stream));
  return item_forward(c, w, t, item_track, n_items, (double)n_items, false, nullptr, item_feat,
                      (hipStream_t)stream);
}

int dcue_user_tower(const dcue_model* m, const int64_t* users, int32_t n, void* ws, size_t ws_bytes,
                    float* user_feat, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!users || !ws || !user_feat || n <= 0 || !m->emb) return DCUE_ERR_INVALID;
  Ws w;
  if (carve(&m->dims, n, 0, 1, nullptr, &w) > ws_bytes) return DCUE_ERR_WORKSPACE;
  carve(&m->dims, n, 0, 1, ws, &w);
  TRY(join_user_stream((hipStream_t)stream));
  if (m->emb_step) TRY(launch_emb_sync(m, users, n, (hipStream_t)stream));
  return user_forward(c, w, users, n, user_feat, (hipStream_t)stream);
}

int dcue_emb_log_bytes(int32_t cap, size_t* bytes_host) {
  if (!bytes_host || cap < 1 || cap > DCUE_MAX_LOG_CAP) return DCUE_ERR_INVALID;
  *bytes_host = sizeof(dcue_emb_log) + (size_t)cap * 8 * sizeof(float);
  return DCUE_OK;
}

int dcue_emb_log_init(const dcue_model* m, int32_t cap, int32_t step, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!m->emb_step || !m->emb_log || cap < 1 || cap > DCUE_MAX_LOG_CAP || cap != m->emb_log_cap ||
      step < 0)
    return DCUE_ERR_INVALID;
  TRY(join_user_stream((hipStream_t)stream));
  return launch_emb_log_init(m, cap, step, (hipStream_t)stream);
}

int dcue_embedding_sync(const dcue_model* m, const int64_t* users, int32_t n, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!users || n < 0) return DCUE_ERR_INVALID;
  if (!m->emb_step) return DCUE_OK;  // dense mode: rows are always current
  TRY(join_user_stream((hipStream_t)stream));
  return launch_emb_sync(m, users, n, (hipStream_t)stream);
}

int dcue_embedding_flush(const dcue_model* m, void* stream) {
  Ctx c;
  TRY(init_ctx(&c, m));
  if (!m->emb_step) return DCUE_OK;
  TRY(join_user_stream((hipStream_t)stream));
  return launch_emb_flush(m, (hipStream_t)stream);
}

}  // extern "C"
