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
};

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
  // the user rows' sync starts with the step (eager only: under capture a side stream joins the
  // graph only through an event of the capturing stream)
  if (!captured) o.sync_users = users_src ? users_src : b->users;
  int st = dcue::step_prologue(m, b, ws, ws_bytes,
                               (cfg->flags & DCUE_PLAN_SAMPLE_INBATCH) ? cfg->mt : nullptr, users_src,
                               items_src, s);
  if (!st) st = dcue::forward_impl(m, b, t, ws, ws_bytes, 1, cfg->margin, o, s);
  if (!st) st = dcue::backward_impl(m, b, t, ws, ws_bytes, nullptr, cfg->emb_grad_scale, o, s);
  return st;
}

int capture(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws, size_t ws_bytes,
            const dcue_plan_config* cfg, hipStream_t cs) {
  return issue_step(m, b, t, ws, ws_bytes, cfg, nullptr, nullptr, cs, nullptr, /*captured=*/true);
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
    // eager plan: validate once by issuing nothing but the checks the calls make themselves
    dcue_plan* p = new dcue_plan;
    p->model = *m;
    p->batch = *b;
    p->tracks = *t;
    p->cfg = *cfg;
    p->ws = ws;
    p->ws_bytes = ws_bytes;
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
  if (!p->exec)  // eager replay: the batch copies ride in the prologue block
    return issue_step(&p->model, &b, &p->tracks, p->ws, p->ws_bytes, &p->cfg, users_src, item_track_src, s);
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
  const int st = issue_step(&p->model, &b, &p->tracks, p->ws, p->ws_bytes, &p->cfg, users_src,
                            item_track_src, (hipStream_t)stream, &emb);
  if (st) return st;
  return dcue_adam_step(&p->model, &dense, stream);
}

extern "C" int dcue_plan_destroy(dcue_plan* p) {
  if (!p) return DCUE_OK;
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  for (hipEvent_t e : p->placeholders) dcue::timer_release(e);
  delete p;
  return DCUE_OK;
}
