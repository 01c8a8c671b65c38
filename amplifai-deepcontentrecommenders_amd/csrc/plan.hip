// Step plans (dcue_plan_*): one training step's sample + forward + backward bound once to its
// buffers and issued by one host call.
//
// The reference's per-batch loop (nn/dcue.py:202-210) runs the same ~60 small kernels every step.
// A plan binds model, batch, tracks and workspace at creation and replays the step either eagerly
// (default: the kernels issued from C++ onto the caller's stream and the side streams, no Python
// between them) or, with DCUE_PLAN_GRAPH, as a HIP graph captured once on a private stream.
// Measured on MI355X / ROCm 7.2 the graph replay is the slower of the two: hipGraphLaunch costs
// about as much host time as the individual launches and executes the captured side-stream
// branches one after another on one queue, losing their overlap. Timed kernel classes
// (dcue_timer_*) get event-record nodes added around their graph nodes, re-pointed at fresh events
// on every replay.
#include <vector>

#include "dcue_internal.h"

struct dcue_plan {
  dcue_model model = {};
  dcue_tracks tracks = {};
  dcue_plan_config cfg = {};
  void* ws = nullptr;
  size_t ws_bytes = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  dcue_batch batch = {};
  struct TimerNodes {
    int cls;
    hipGraphNode_t a, b;
  };
  std::vector<TimerNodes> timers;
  std::vector<hipEvent_t> placeholders;  // events the record nodes were built with
  // eager plans prepare each step's inputs one step ahead (issue_eager): double-buffered draws,
  // copy counts and cleared accumulator blocks, and the draw stream's state after the last prepared
  // step
  void* ahead = nullptr;
  int32_t* neg[2] = {};
  float* counts[2] = {};
  int32_t* copy_ptr[2] = {};  // per-item copy lists (gather layout, StepPrologue)
  int32_t* copy_idx[2] = {};
  unsigned long long* acc[2] = {};
  long nacc = 0;
  dcue_mt_state* mt_ahead = nullptr;
  // lookahead (dcue_plan_set_next): each slot's conv-1 wgrad X operand, the items its bn0 sums and
  // xhat0 were prepared from (nullptr: not prepared), and the announced next batch
  float* xh[2] = {};
  float* y1[2] = {};  // conv 1's output per slot (split plans, StepOpts::y1)
  const int32_t* ahead_items[2] = {};
  const int32_t* next_items = nullptr;
  long launches = 0;
  hipEvent_t tails[2] = {};       // the last launched step's end (StepOpts::tails)
  hipEvent_t late_done = nullptr; // the last split step's late-segment Adam (StepOpts::dense_split)
  hipEvent_t inputs_ready = nullptr;  // the next step's inputs (prologue + lookahead) on wgrad stream 0
  int pending_flush = -1;         // step whose rolling-flush slice the next launch issues
  hipStream_t last_stream = nullptr;  // the caller's stream of the last launch
  dcue_comm* comm = nullptr;      // data-parallel exchange between backward and Adam (plan_step)
  bool sync_bn = false;           // SyncBN over `comm` (dcue_plan_set_sync_bn)
  long late = 0, n_dense = 0;     // flat-gradient floats: end of bn0/conv1/bn1, total
  int comm_world = 1;
  // device-side waits (StepOpts::sig, DevWait): the plan's signal words, the values issued into
  // them, and the last split step's late-Adam signal (what the next step's conv 2 waits for)
  unsigned* sig = nullptr;
  unsigned sig_issued[dcue::kSigSlots] = {};
  dcue::DevWait late_sig{};
};

// DCUE_XQ_WAIT=event: the plan's caller-stream waits as HIP event waits (rounds 1-5; A/B). Also off
// under rocprofv3 counter collection (ROCPROF_COUNTER_COLLECTION): it runs one dispatch at a time, so
// a consumer kernel polling for a producer on another queue would hold the GPU until its wait gave up
// (DevWait's bound; measured: the fail word's bit 1 set, 1.4 ms steps)
static bool dev_waits_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_XQ_WAIT");
    const char* pmc = getenv("ROCPROF_COUNTER_COLLECTION");
    const bool counters = pmc && pmc[0] && pmc[0] != '0' && pmc[0] != 'f' && pmc[0] != 'F';
    return !(e && e[0] == 'e') && !counters;
  }();
  return on;
}

namespace {

// The step as the plan issues it: one prologue block (batch copies, accumulator clear, in-batch
// draw, copy counts), the train forward with the hinge backward fused into its score kernel, and
// the rest of the backward.
int issue_step(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
               const dcue_plan_config* cfg, const int64_t* users_src, const int32_t* items_src,
               hipStream_t s, const dcue_adam_args* emb_adam = nullptr, bool captured = false) {
  dcue::StepOpts o;
  o.prologue_done = true;
  o.fuse_score = true;
  o.emb_adam = emb_adam;
  hipEvent_t score_done = nullptr;
  o.score_done = &score_done;
  (void)captured;
  int st = dcue::step_prologue(m, b, ws, ws_bytes,
                               (cfg->flags & DCUE_PLAN_SAMPLE_INBATCH) ? cfg->mt : nullptr, users_src,
                               items_src, s);
  if (!st) st = dcue::forward_impl(m, b, t, ws, ws_bytes, 1, cfg->margin, o, s);
  if (!st) st = dcue::backward_impl(m, b, t, ws, ws_bytes, nullptr, cfg->emb_grad_scale, o, s);
  return st;
}

// Eager replay with the step's inputs prepared one step ahead. Step t's draw, copy counts and
// accumulator clear are made by launch t-1 on a weight-gradient stream while step t-1 computes (one
// 1024-thread block beside the step's kernels), so step t's first kernel on the caller's stream is
// already the item tower's input statistics. Buffers alternate by step parity; launch t prepares
// slot t+1 once step t-1 -- the last reader of that slot -- has ended, and publishes what the
// caller can see of step t: the negatives into the bound neg_item buffer, the batch indices into
// the bound batch buffers and, into cfg.mt, the draw stream's state after step t's draw (the
// plan's own copy runs one step ahead).
int issue_eager(dcue_plan* p, const int64_t* users_src, const int32_t* items_src, hipStream_t s,
                const dcue_adam_args* emb_adam, const dcue_adam_args* dense_split = nullptr) {
  using namespace dcue;
  SidePool* sp = side_pool();
  if (!sp) return DCUE_ERR_HIP;
  const dcue_batch& b0 = p->batch;
  const bool inbatch = (p->cfg.flags & DCUE_PLAN_SAMPLE_INBATCH) != 0;
  const int cur = (int)(p->launches & 1), nxt = cur ^ 1;
  hipStream_t sa = sp->st[1];
  auto inputs = [&](int slot) {
    StepPrologue q = {};
    q.B = b0.n_rows; q.N = b0.n_neg; q.M = b0.n_items;
    q.gather = b0.layout == DCUE_LAYOUT_GATHER;
    q.neg = inbatch ? p->neg[slot] : const_cast<int32_t*>(b0.neg_item);
    q.zero = p->acc[slot]; q.nzero = p->nacc;
    q.counts = p->counts[slot];
    q.copy_ptr = p->copy_ptr[slot];
    q.copy_idx = p->copy_idx[slot];
    return q;
  };
  if (p->launches == 0) {  // the first step's inputs, on the caller's stream
    StepPrologue q = inputs(cur);
    q.mt = inbatch ? p->cfg.mt : nullptr;
    q.mt_out = p->mt_ahead;
    TRY(launch_step_prologue(q, s));
    HPROF("plan:1");
    TRY(fork_point(sp, s, &p->tails[0]));
    HPROF("plan:2");
  }
  // A point on the caller's stream at this launch's start: the user tower, this launch's prologue
  // for the next step and the lookahead wait for it (it orders them after everything the caller
  // enqueued before the launch -- the batch indices, the announced next items -- and after the last
  // step, which ended on this stream).
  hipEvent_t ev_in = nullptr;
  TRY(fork_point(sp, s, &ev_in));
  dcue_batch b = b0;
  if (users_src) b.users = users_src;
  if (items_src) b.item_track = items_src;
  if (inbatch) b.neg_item = p->neg[cur];
  // this step's inputs were prepared ahead from exactly these items
  const bool prepared = p->ahead_items[cur] != nullptr;
  const bool ahead = prepared && items_src == p->ahead_items[cur];
  p->ahead_items[cur] = nullptr;
  // The next step's inputs (slot nxt) are made on wgrad stream 0, which split plans never join back
  // into the caller's stream: the prologue (draws, copy counts, cleared accumulators, published
  // batch) and the lookahead (the announced next batch's bn0 sums and, on the f32 path, its xhat0),
  // issued on the side-issue thread (side.hip) when it runs. The caller's stream waits for them
  // (inputs_ready) inside this step's backward, just before the conv-1 weight gradient -- long after
  // they finished -- so the next launch's conv 1 is ordered after them.
  // DCUE_INPUTS_WAIT=start waits at the next launch's start instead, =0 not at all (A/B only).
  // DCUE_AHEAD_AT=fork: the lookahead at the backward's first dgrad fork point instead of right
  // behind the prologue (A/B).
  static const int inputs_wait = [] {
    const char* e = getenv("DCUE_INPUTS_WAIT");
    return !e ? 1 : e[0] == '0' ? 0 : e[0] == 's' ? 2 : 1;
  }();
  static const bool ahead_at_fork = [] {
    const char* e = getenv("DCUE_AHEAD_AT");
    return e && e[0] == 'f';
  }();
  if (p->inputs_ready && inputs_wait == 2) TRY(wait_point(s, p->inputs_ready));
  p->ahead_items[nxt] = nullptr;
  const bool look = p->next_items && p->xh[nxt];
  if (look) p->ahead_items[nxt] = p->next_items;
  p->next_items = nullptr;
  p->inputs_ready = ring_event(sp);  // slot nxt's inputs, for the next launch (recorded below)
  // the lookahead, then the inputs_ready record, on wgrad stream 0 after `after`
  // device-side waits (no communicator: its exchange keeps the event orders)
  const bool dev = p->sig && !p->comm && dev_waits_on();
  DevWait in_sig{};
  if (dev && inputs_wait == 1) in_sig = DevWait{p->sig + kSigInputs, ++p->sig_issued[kSigInputs], user_fwd_fail_flag()};
  const std::function<int(hipEvent_t)> lookahead = [p, sa, nxt, look, ir = p->inputs_ready, in_sig](hipEvent_t after) -> int {
    if (look) {
      if (after) TRY(wait_point(sa, after));
      TRY(debug_delay(DCUE_SITE_LOOKAHEAD, sa));
      TRY(ahead_item_inputs(&p->model, &p->batch, &p->tracks, p->ahead_items[nxt], p->counts[nxt], p->acc[nxt],
                            p->xh[nxt], sa));
    }
    DCUE_HIP_CHECK(hipEventRecord(ir, sa));
    if (in_sig.flag) TRY(launch_signal(const_cast<unsigned*>(in_sig.flag), in_sig.val, sa));
    return DCUE_OK;
  };
  SideQueue side;
  int sst = DCUE_OK;
  uint64_t iseq = 0;
  StepOpts o;
  o.ev_in = ev_in;
  o.sync_bn = p->sync_bn ? p->comm : nullptr;
  o.prologue_done = true;
  o.fuse_score = true;
  o.emb_adam = emb_adam;
  o.counts = p->counts[cur];
  o.copy_ptr = p->copy_ptr[cur];
  o.copy_idx = p->copy_idx[cur];
  o.acc = p->acc[cur];
  o.input_stats_done = ahead;
  o.xhat0 = ahead ? p->xh[cur] : nullptr;
  o.clear_bn0 = prepared && !ahead;
  o.tails = p->tails;
  o.wait_late = p->late_done;  // the previous split step's late Adam (before conv 1 or 2, late_wait_at_conv1)
  o.dense_split = dense_split;
  if (dense_split) o.y1 = p->y1[cur];
  o.comm = dense_split ? p->comm : nullptr;  // the exchange inside the backward (comm_exchange_split)
  hipEvent_t late_done = nullptr;
  o.late_done = &late_done;
  DevWait late_sig{};
  if (dev) {
    o.sig = p->sig;
    o.sig_issued = p->sig_issued;
    o.late_wait = p->late_sig;
    o.late_sig = &late_sig;
    o.inputs_wait = in_sig;
  }
  // the previous step's rolling-flush slice runs after this step's user tower (StepOpts)
  const bool deferred = p->model.emb_step != nullptr;
  o.flush_slice_step = deferred ? p->pending_flush : -1;
  o.defer_flush_slice = deferred && emb_adam != nullptr;
  hipEvent_t slice_done = nullptr;
  o.slice_done = &slice_done;
  // DCUE_SCORE_FORK=1: the score kernel binds a fork point that the user tower's backward waits for
  // (A/B; default: it waits for the dgrad chain's first fork point, one bound event fewer)
  static const bool score_fork = [] {
    const char* e = getenv("DCUE_SCORE_FORK");
    return e && e[0] == '1';
  }();
  hipEvent_t score_done = nullptr;
  if (score_fork) o.score_done = &score_done;
  // DCUE_PROLOGUE_FIRST=1: the prologue closure is posted before the forward (A/B)
  static const bool prologue_first = [] {
    const char* e = getenv("DCUE_PROLOGUE_FIRST");
    return e && e[0] == '1';
  }();
  auto post_prologue = [&]() -> int {
    StepPrologue q = inputs(nxt);
    if (inbatch) {
      q.mt = p->mt_ahead;
      q.mt_commit = p->cfg.mt;
      q.copy_src = p->neg[cur];
      q.copy_dst = const_cast<int32_t*>(b0.neg_item);
      q.ncopy = (long)b0.n_rows * b0.n_neg;
    }
    q.users_dst = const_cast<int64_t*>(b0.users); q.users_src = users_src;
    q.items_dst = const_cast<int32_t*>(b0.item_track); q.items_src = items_src;
    // Slot nxt was last read by the previous step, partly on side streams that the caller's stream
    // does not join (split plans): the layer-2 weight gradient on wgrad stream 1 reads its copy
    // counts, BN sums and value ranges, which this prologue clears and rewrites. The previous step's
    // late Adam waited for every side stream, so its point (late_done, also what this step's conv 2
    // waits for) orders the prologue after all of them. Without this wait a delayed layer-2 weight
    // gradient read a cleared range -- a NaN operand scale -- and the step's conv-2 gradient went
    // non-finite (tests/test_gpu_races.py).
    const hipEvent_t prev_late = legacy_orders() ? nullptr : p->late_done;
    iseq = side.run([q, sa, ev_in, prev_late, &lookahead]() -> int {
      TRY(wait_point(sa, ev_in));
      if (prev_late) TRY(wait_point(sa, prev_late));
      TRY(debug_delay(DCUE_SITE_PROLOGUE, sa));
      TRY(launch_step_prologue(q, sa));
      return ahead_at_fork ? DCUE_OK : lookahead(nullptr);  // (the prologue on sa orders it)
    }, &sst);
    return sst;
  };
  if (prologue_first) TRY(post_prologue());
  TRY(forward_impl(&p->model, &b, &p->tracks, p->ws, p->ws_bytes, 1, p->cfg.margin, o, s));
  HPROF("plan:4");
  // posted after the forward, whose user tower (on the critical path's first fork) the side thread
  // then issues first
  if (!prologue_first) TRY(post_prologue());
  if (ahead_at_fork) o.ahead = &lookahead;
  if (inputs_wait == 1) {
    o.wait_inputs = p->inputs_ready;
    o.wait_inputs_seq = iseq;
    p->inputs_ready = nullptr;
  } else if (!ahead_at_fork) {
    TRY(side.wait(iseq));
  }
  TRY(backward_impl(&p->model, &b, &p->tracks, p->ws, p->ws_bytes, nullptr, p->cfg.emb_grad_scale, o, s));
  HPROF("plan:5");
  p->pending_flush = o.defer_flush_slice ? emb_adam->step : -1;
  p->late_done = dense_split ? late_done : nullptr;
  p->late_sig = dense_split ? late_sig : DevWait{};
  p->last_stream = s;
  ++p->launches;
  return DCUE_OK;
}

// DCUE_SPLIT_COMM=0: data-parallel plan steps keep the unsplit exchange (both buckets, then the whole
// dense Adam on the caller's stream) -- the A/B of comm_exchange_split
bool split_comm_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_SPLIT_COMM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// DCUE_SPLIT_ADAM=0 keeps the whole dense Adam on the caller's stream after the join (A/B)
bool split_adam_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_SPLIT_ADAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

int capture(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
            const dcue_plan_config* cfg, hipStream_t cs) {
  dcue::capturing_step() = true;
  const int st = issue_step(m, b, t, ws, ws_bytes, cfg, nullptr, nullptr, cs, nullptr, /*captured=*/true);
  dcue::capturing_step() = false;
  return st;
}

}  // namespace

extern "C" int dcue_plan_destroy(dcue_plan* p);

extern "C" int dcue_plan_create(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                                size_t ws_bytes, const dcue_plan_config* cfg, dcue_plan** plan_host) {
  if (!m || !b || !t || !ws || !cfg || !plan_host) return DCUE_ERR_INVALID;
  *plan_host = nullptr;
  if (cfg->flags & ~(DCUE_PLAN_SAMPLE_INBATCH | DCUE_PLAN_GRAPH)) return DCUE_ERR_INVALID;
  if ((cfg->flags & DCUE_PLAN_SAMPLE_INBATCH) &&
      (!cfg->mt || b->layout != DCUE_LAYOUT_GATHER || !b->neg_item || b->n_neg <= 0))
    return DCUE_ERR_INVALID;
  if (!dcue::side_pool()) return DCUE_ERR_HIP;  // side streams exist before capture starts
  if (!(cfg->flags & DCUE_PLAN_GRAPH)) {
    // the eager replay prepares step t+1's copy counts during launch t from the negatives it drew
    // itself; caller-written gather negatives would be read before the caller refreshed them
    if (b->layout == DCUE_LAYOUT_GATHER && !(cfg->flags & DCUE_PLAN_SAMPLE_INBATCH)) return DCUE_ERR_UNSUPPORTED;
    // eager plan: validate once by issuing nothing but the checks the calls make themselves
    const int B = b->n_rows, N = b->n_neg, M = b->n_items;
    const long nneg = (cfg->flags & DCUE_PLAN_SAMPLE_INBATCH) ? (long)B * N : 0;
    const long nacc = dcue::step_acc_words(&m->dims, B, N, M);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t bneg = al(sizeof(int32_t) * (nneg > 0 ? nneg : 1)), bcnt = al(sizeof(float) * M),
                 bacc = al(sizeof(unsigned long long) * nacc), bmt = al(sizeof(dcue_mt_state));
    // copy lists: in-batch plans (the prologue's histogram path holds M <= 2048 items)
    const bool lists = (cfg->flags & DCUE_PLAN_SAMPLE_INBATCH) && M <= dcue::kCopyListMaxItems;
    const size_t bptr = lists ? al(sizeof(int32_t) * (M + 1)) : 0,
                 bidx = lists ? al(sizeof(int32_t) * ((size_t)B * (N + 1))) : 0;
    // lookahead slots (plans of BatchNorm towers): xhat0 per slot
    const bool look = dcue::tower_has_bn(&m->dims);
    const size_t bxh = look ? al(sizeof(float) * (size_t)(M + 1) * dcue::kXp * dcue::kMels) : 0;
    // conv 1's output per slot (StepOpts::y1): [M][33][H_s] floats
    const size_t by1 = al(sizeof(float) * (size_t)M * dcue::layer_geom(1).lp * dcue::st_hidden(&m->dims));
    void* mem = nullptr;
    const size_t bsig = al(sizeof(unsigned) * dcue::kSigSlots);
    const size_t mem_bytes = 2 * (bneg + bcnt + bacc + bxh + bptr + bidx + by1) + bmt + bsig;
    DCUE_HIP_CHECK(hipMalloc(&mem, mem_bytes));
    if (dcue::poison_on()) {  // debug: a read of a word no kernel wrote shows as NaN
      DCUE_HIP_CHECK(hipMemset(mem, 0xFF, mem_bytes));
      DCUE_HIP_CHECK(hipDeviceSynchronize());
    }
    // the signal words start at 0, as the host's issue counters (after the poison fill)
    unsigned* sig = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(mem) + mem_bytes - bsig);
    DCUE_HIP_CHECK(hipMemset(sig, 0, bsig));
    DCUE_HIP_CHECK(hipDeviceSynchronize());
    dcue_plan* p = new dcue_plan;
    p->model = *m;
    p->batch = *b;
    p->tracks = *t;
    p->cfg = *cfg;
    p->ws = ws;
    p->ws_bytes = ws_bytes;
    p->ahead = mem;
    char* q = (char*)mem;
    for (int i = 0; i < 2; ++i) {
      p->neg[i] = (int32_t*)q; q += bneg;
      p->counts[i] = (float*)q; q += bcnt;
      p->acc[i] = (unsigned long long*)q; q += bacc;
      if (bxh) { p->xh[i] = (float*)q; q += bxh; }
      if (lists) {
        p->copy_ptr[i] = (int32_t*)q; q += bptr;
        p->copy_idx[i] = (int32_t*)q; q += bidx;
      }
      p->y1[i] = (float*)q; q += by1;
    }
    p->mt_ahead = (dcue_mt_state*)q;
    p->sig = sig;
    p->nacc = nacc;
    *plan_host = p;
    return DCUE_OK;
  }

  hipStream_t cs = nullptr;
  DCUE_HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  dcue::timer_take_captured();  // drop stale entries of an earlier failed capture
  int st = DCUE_OK;
  hipGraph_t graph = nullptr;
  if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) {
    st = DCUE_ERR_HIP;
  } else {
    st = capture(m, b, t, ws, ws_bytes, cfg, cs);
    // end the capture whatever happened, so the stream is usable and nothing leaks
    if (hipStreamEndCapture(cs, &graph) != hipSuccess && !st) st = DCUE_ERR_HIP;
  }
  std::vector<dcue::CapturedTimer> cap = dcue::timer_take_captured();
  (void)hipStreamDestroy(cs);
  if (st || !graph) {
    if (graph) (void)hipGraphDestroy(graph);
    return st ? st : DCUE_ERR_HIP;
  }

  dcue_plan* p = new dcue_plan;
  p->graph = graph;
  p->batch = *b;
  // timed kernels: a start record beside the kernel (same predecessors, ordered before it) and an
  // end record after it; the events are placeholders, re-pointed at every launch
  for (auto& c : cap) {
    hipGraphNode_t na = nullptr, nb = nullptr;
    hipEvent_t ea = dcue::timer_event(), eb = dcue::timer_event();
    if (!ea || !eb ||
        hipGraphAddEventRecordNode(&na, graph, c.preds.data(), c.preds.size(), ea) != hipSuccess ||
        hipGraphAddDependencies(graph, &na, &c.kernel, 1) != hipSuccess ||
        hipGraphAddEventRecordNode(&nb, graph, &c.kernel, 1, eb) != hipSuccess) {
      dcue::set_last_error("plan timer nodes", hipErrorInvalidValue, __FILE__, __LINE__);
      dcue::timer_release(ea);
      dcue::timer_release(eb);
      (void)hipGraphDestroy(graph);
      delete p;
      return DCUE_ERR_HIP;
    }
    p->timers.push_back(dcue_plan::TimerNodes{c.cls, na, nb});
    p->placeholders.push_back(ea);
    p->placeholders.push_back(eb);
  }
  const hipError_t ie = hipGraphInstantiate(&p->exec, graph, nullptr, nullptr, 0);
  if (ie != hipSuccess) {
    dcue::set_last_error("hipGraphInstantiate", ie, __FILE__, __LINE__);
    p->exec = nullptr;
    dcue_plan_destroy(p);
    return DCUE_ERR_HIP;
  }
  *plan_host = p;
  return DCUE_OK;
}

extern "C" int dcue_plan_launch(dcue_plan* p, const int64_t* users_src, const int32_t* item_track_src,
                                void* stream) {
  if (!p) return DCUE_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  const dcue_batch& b = p->batch;
  if (users_src == b.users) users_src = nullptr;
  if (item_track_src == b.item_track) item_track_src = nullptr;
  if (!p->exec) {
    TRY(issue_eager(p, users_src, item_track_src, s, nullptr));
    if (!p->comm) return DCUE_OK;
    // a bound communicator: the step's dense gradient leaves as the mean over the ranks, whatever
    // optimizer the caller runs next (SGD, Ranger, or Adam as a separate call)
    TRY(dcue::comm_exchange_step(p->comm, p->model.grads, p->late, p->n_dense, p->tails[1], s));
    return dcue::comm_divide(p->comm, p->model.grads, p->n_dense, s);
  }
  if (users_src)
    DCUE_HIP_CHECK(hipMemcpyAsync(const_cast<int64_t*>(b.users), users_src, sizeof(int64_t) * b.n_rows,
                                  hipMemcpyDeviceToDevice, s));
  if (item_track_src)
    DCUE_HIP_CHECK(hipMemcpyAsync(const_cast<int32_t*>(b.item_track), item_track_src,
                                  sizeof(int32_t) * b.n_items, hipMemcpyDeviceToDevice, s));
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> fresh;
  for (auto& tn : p->timers) {
    hipEvent_t a = dcue::timer_event(), e = dcue::timer_event();
    if (!a || !e) return DCUE_ERR_HIP;
    DCUE_HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(p->exec, tn.a, a));
    DCUE_HIP_CHECK(hipGraphExecEventRecordNodeSetEvent(p->exec, tn.b, e));
    fresh.push_back({tn.cls, {a, e}});
  }
  DCUE_HIP_CHECK(hipGraphLaunch(p->exec, s));
  for (auto& f : fresh) dcue::timer_add_recorded(f.first, f.second.first, f.second.second);
  return DCUE_OK;
}

extern "C" int dcue_plan_step(dcue_plan* p, const int64_t* users_src, const int32_t* item_track_src,
                              const dcue_adam_args* adam, void* stream) {
  HPROF("plan_step:enter (python)");
  if (!p) return DCUE_ERR_INVALID;
  if (!adam || p->exec) {  // graph replay (or no optimizer): the Adam step follows as one call
    const int st = dcue_plan_launch(p, users_src, item_track_src, stream);
    if (st || !adam) return st;
    return dcue_adam_step(&p->model, adam, stream);
  }
  if (adam->parts) return DCUE_ERR_INVALID;
  // eager: the user table's part of Adam rides on the user-tower stream inside the backward (it
  // needs only the embedding rows' gradient); the dense part follows once every gradient is in
  const dcue_batch& b = p->batch;
  if (users_src == b.users) users_src = nullptr;
  if (item_track_src == b.item_track) item_track_src = nullptr;
  dcue_adam_args emb = *adam, dense = *adam;
  emb.parts = DCUE_ADAM_EMBEDDING;
  dense.parts = DCUE_ADAM_DENSE;
  if (split_adam_on() && (!p->comm || split_comm_on())) {
    // the dense Adam split over two streams (StepOpts); with a communicator each part after its own
    // bucket's all-reduce (comm_exchange_split), the divide by the world size fused into the sweep
    if (p->comm) dense.grad_div = p->comm_world;
    TRY(issue_eager(p, users_src, item_track_src, (hipStream_t)stream, &emb, &dense));
    HPROF("plan_step:issue");
    return DCUE_OK;
  }
  const int st = issue_eager(p, users_src, item_track_src, (hipStream_t)stream, &emb);
  if (st) return st;
  HPROF("plan_step:issue");
  if (p->comm) {  // the DDP mean of the dense gradient: RCCL sum here, the divide inside Adam
    TRY(dcue::comm_exchange_step(p->comm, p->model.grads, p->late, p->n_dense, p->tails[1],
                                 (hipStream_t)stream));
    dense.grad_div = p->comm_world;
    HPROF("plan_step:exchange");
  }
  const int r = dcue_adam_step(&p->model, &dense, stream);
  HPROF("plan_step:adam");
  return r;
}

extern "C" int dcue_plan_set_comm(dcue_plan* p, dcue_comm* comm) {
  if (!p || p->exec) return DCUE_ERR_INVALID;  // eager plans only
  p->comm = comm;
  p->comm_world = 1;
  if (!comm) {
    p->sync_bn = false;
    return DCUE_OK;
  }
  int64_t off[DCUE_N_DENSE_SEGMENTS + 1];
  TRY(dcue_param_layout(&p->model.dims, off));
  p->late = off[DCUE_SEG_LATE];
  p->n_dense = off[DCUE_N_DENSE_SEGMENTS];
  p->comm_world = dcue::comm_world(comm);
  return DCUE_OK;
}

extern "C" int dcue_plan_set_sync_bn(dcue_plan* p, int32_t on) {
  if (!p || p->exec) return DCUE_ERR_INVALID;
  if (!on) {
    p->sync_bn = false;
    return DCUE_OK;
  }
  if (!p->comm) return DCUE_ERR_INVALID;  // bind the communicator first
  // the f32 conv-1 weight-gradient path materialises bn0(x) one step ahead on a side stream, before
  // this step's sums are exchanged; SyncBN runs on the split-f16 weight gradients (the default)
  if (!dcue::wgrad_f16_on()) return DCUE_ERR_UNSUPPORTED;
  p->sync_bn = true;
  return DCUE_OK;
}

extern "C" int dcue_plan_set_next(dcue_plan* p, const int32_t* next_item_track) {
  if (!p) return DCUE_ERR_INVALID;
  if (p->exec || !p->xh[0]) return DCUE_ERR_UNSUPPORTED;
  p->next_items = next_item_track;
  return DCUE_OK;
}

extern "C" int dcue_plan_sync(dcue_plan* p, void* stream) {
  if (!p) return DCUE_ERR_INVALID;
  if (p->exec) return DCUE_OK;  // graph replays run whole on the stream they were launched on
  // the user stream holds the step's last Adam work (split dense segments, user table); the weight
  // gradient streams are joined into it by then
  return dcue::join_user_stream((hipStream_t)stream);
}

extern "C" int dcue_plan_wait_side(dcue_plan* p, void* stream) {
  if (!p || p->exec || p->launches == 0 || !p->tails[1]) return DCUE_ERR_INVALID;
  // tails[1]: wgrad stream 0 after it joined the user stream's and wgrad stream 1's tails
  DCUE_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, p->tails[1], 0));
  return DCUE_OK;
}

extern "C" int dcue_plan_destroy(dcue_plan* p) {
  if (!p) return DCUE_OK;
  // a rolling-flush slice deferred to the next launch must still run: every row has to be replayed
  // within `cap` steps of the current one, or the history ring it needs is overwritten
  // It goes on the user stream, where the last step's user-table Adam (k_adam_touched) ran: a
  // normal launch issues it there too (after that step's user tower), and the caller's stream is
  // not ordered after k_adam_touched (nothing joins it back before the dense Adam).
  if (p->pending_flush >= 0 && p->model.emb_step) {
    dcue::SidePool* sp = dcue::side_pool();
    if (sp) {
      (void)dcue::launch_emb_flush_rows(&p->model, p->pending_flush, sp->st[0]);
      (void)hipStreamSynchronize(sp->st[0]);
    }
  }
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  for (hipEvent_t e : p->placeholders) dcue::timer_release(e);
  if (p->ahead) (void)hipFree(p->ahead);
  delete p;
  return DCUE_OK;
}
