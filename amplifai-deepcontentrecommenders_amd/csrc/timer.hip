// Live kernel timing with HIP events (dcue_timer_*): the launch sites of the timed kernel classes
// bind an event pair to the launch itself (hipExtLaunchKernel start/stop, LaunchTag), on every
// stride-th launch of the class. Under stream capture the
// launch's graph node and its predecessors are noted instead; the plan adds event-record nodes
// around the kernel node and re-points them at fresh events on every launch (plan.hip), so each
// replay is timed. One lock guards the state: the side-issue worker (side.hip) times its launches
// too.
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <map>
#include <mutex>
#include <string>

#include <utility>
#include <vector>

#include "dcue_internal.h"

namespace dcue {

namespace {
struct TimerState {
  int stride[DCUE_N_TIMED] = {};  // time every stride-th launch (0: off)
  long seen[DCUE_N_TIMED] = {};
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> recorded[DCUE_N_TIMED];
  std::vector<CapturedTimer> captured;
};
TimerState& ts() {
  static TimerState s;
  return s;
}
// the side-issue worker (side.hip) times its own launches: one lock around the shared state
std::recursive_mutex& tmu() {
  static std::recursive_mutex m;
  return m;
}
}  // namespace

hipEvent_t timer_event() {
  std::lock_guard<std::recursive_mutex> lk(tmu());
  TimerState& t = ts();
  if (!t.pool.empty()) {
    hipEvent_t e = t.pool.back();
    t.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing only (hipEventElapsedTime after a host wait): no system-scope fence at completion, which
  // would cost the timed stream a cache writeback (hip_runtime_api.h, hipEventDisableSystemFence)
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

void timer_add_recorded(int cls, hipEvent_t a, hipEvent_t b) { std::lock_guard<std::recursive_mutex> lk(tmu()); ts().recorded[cls].emplace_back(a, b); }

bool timer_take_turn(int cls) {
  std::lock_guard<std::recursive_mutex> lk(tmu());
  if (cls < 0 || cls >= DCUE_N_TIMED || !ts().stride[cls]) return false;
  return ts().seen[cls]++ % ts().stride[cls] == 0;
}

int timer_begin(TimerScope* sc, int cls, hipStream_t s) {
  sc->cls = cls;
  sc->s = s;
  sc->a = sc->b = nullptr;
  sc->capturing = false;
  sc->preds.clear();
  if (cls < 0 || cls >= DCUE_N_TIMED) return DCUE_OK;  // (no lock for untimed launches: most of them)
  std::lock_guard<std::recursive_mutex> lk(tmu());
  if (!ts().stride[cls]) return DCUE_OK;
  if (ts().seen[cls]++ % ts().stride[cls]) return DCUE_OK;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  DCUE_HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &st, nullptr, nullptr, &deps, &nd));
  if (st == hipStreamCaptureStatusActive) {  // the plan adds the record nodes after capture
    sc->capturing = true;
    sc->preds.assign(deps, deps + nd);
    return DCUE_OK;
  }
  sc->a = timer_event();
  sc->b = timer_event();
  if (!sc->a || !sc->b) return DCUE_ERR_HIP;
  // the pair is bound to the timed launch itself: its own dispatch timestamps, no record packets
  sc->saved = launch_tag();
  launch_tag() = LaunchTag{sc->a, sc->b, 0, false};
  return DCUE_OK;
}

int timer_end(TimerScope* sc) {
  if (!sc->capturing && !sc->a) return DCUE_OK;  // (an untimed launch: no lock)
  std::lock_guard<std::recursive_mutex> lk(tmu());
  if (sc->capturing) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    DCUE_HIP_CHECK(hipStreamGetCaptureInfo_v2(sc->s, &st, nullptr, nullptr, &deps, &nd));
    if (st == hipStreamCaptureStatusActive && nd == 1)
      ts().captured.push_back(CapturedTimer{sc->cls, sc->preds, deps[0]});
    return DCUE_OK;
  }
  if (!sc->a) return DCUE_OK;
  const int n = launch_tag().launches;
  launch_tag() = sc->saved;
  if (n && sc->saved.stop) launch_tag().missed = true;
  if (n != 1) {  // nothing (or more than the one kernel) launched: time the interval by records
    timer_release(sc->a);
    timer_release(sc->b);
    sc->a = nullptr;
    return n ? DCUE_ERR_INVALID : DCUE_OK;
  }
  timer_add_recorded(sc->cls, sc->a, sc->b);
  return DCUE_OK;
}

std::vector<CapturedTimer> timer_take_captured() {
  std::lock_guard<std::recursive_mutex> lk(tmu());
  std::vector<CapturedTimer> out;
  out.swap(ts().captured);
  return out;
}

void timer_release(hipEvent_t e) {
  std::lock_guard<std::recursive_mutex> lk(tmu());
  if (e) ts().pool.push_back(e);
}

namespace {
char g_last_error[512] = "";

struct HostProfile {
  bool on = false;
  std::chrono::steady_clock::time_point last;
  std::map<std::string, std::pair<double, long>> acc;
  std::vector<std::string> order;
  bool slow = false;  // DCUE_HOST_PROFILE=2: also every single interval above 100 us, as it happens
  HostProfile() {
    const char* e = getenv("DCUE_HOST_PROFILE");
    on = e && (e[0] == '1' || e[0] == '2');
    slow = e && e[0] == '2';
    last = std::chrono::steady_clock::now();
  }
  ~HostProfile() {
    if (!on) return;
    for (auto& k : order) {
      auto& v = acc[k];
      fprintf(stderr, "[dcue host] %-28s %8.2f us  x%ld\n", k.c_str(), v.first / (v.second ? v.second : 1),
              v.second);
    }
  }
};
HostProfile& hp() {
  static HostProfile p;
  return p;
}
}  // namespace

bool host_profile_on() { return hp().on; }

void host_profile_mark(const char* label) {
  HostProfile& p = hp();
  const auto now = std::chrono::steady_clock::now();
  const double us = std::chrono::duration<double, std::micro>(now - p.last).count();
  p.last = now;
  auto it = p.acc.find(label);
  if (it == p.acc.end()) {
    p.order.push_back(label);
    it = p.acc.emplace(label, std::make_pair(0.0, 0L)).first;
  }
  it->second.first += us;
  it->second.second += 1;
  if (p.slow && us > 100.0) fprintf(stderr, "[dcue host slow] %s %.1f us (call %ld)\n", label, us, it->second.second);
}

void set_last_error(const char* expr, hipError_t e, const char* file, int line) {
  const char* base = file;
  for (const char* q = file; *q; ++q)
    if (*q == '/') base = q + 1;
  snprintf(g_last_error, sizeof(g_last_error), "%s:%d: %s -> %s (%d)", base, line, expr,
           hipGetErrorString(e), (int)e);
}

}  // namespace dcue

extern "C" const char* dcue_last_error(void) { return dcue::g_last_error; }

extern "C" int dcue_timer_enable(int32_t kernel, int32_t enable) {
  if (kernel < 0 || kernel >= DCUE_N_TIMED) return DCUE_ERR_INVALID;
  if (enable < 0) return DCUE_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> lk(dcue::tmu());
  dcue::ts().stride[kernel] = enable;
  // the first timed launch is the enable-th (ABI 16; was the first): a timed launch costs the host
  // tens of microseconds, and the first launches after enabling are the ones a measurement starts with
  dcue::ts().seen[kernel] = 1;
  return DCUE_OK;
}

extern "C" int dcue_timer_read(int32_t kernel, double* total_ms_host, int64_t* launches_host) {
  if (kernel < 0 || kernel >= DCUE_N_TIMED || !total_ms_host || !launches_host) return DCUE_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> lk(dcue::tmu());
  auto& rec = dcue::ts().recorded[kernel];
  double total = 0.0;
  int64_t n = 0;
  for (auto& pr : rec) {
    DCUE_HIP_CHECK(hipEventSynchronize(pr.second));
    float ms = 0.f;
    DCUE_HIP_CHECK(hipEventElapsedTime(&ms, pr.first, pr.second));
    total += ms;
    ++n;
    dcue::timer_release(pr.first);
    dcue::timer_release(pr.second);
  }
  rec.clear();
  *total_ms_host = total;
  *launches_host = n;
  return DCUE_OK;
}

// each recorded launch's duration (the first `cap`; *launches_host counts all of them), then reset
extern "C" int dcue_timer_samples(int32_t kernel, float* ms_host, int64_t cap, int64_t* launches_host) {
  if (kernel < 0 || kernel >= DCUE_N_TIMED || !launches_host || cap < 0 || (cap > 0 && !ms_host))
    return DCUE_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> lk(dcue::tmu());
  auto& rec = dcue::ts().recorded[kernel];
  int64_t n = 0;
  for (auto& pr : rec) {
    DCUE_HIP_CHECK(hipEventSynchronize(pr.second));
    float ms = 0.f;
    DCUE_HIP_CHECK(hipEventElapsedTime(&ms, pr.first, pr.second));
    if (n < cap) ms_host[n] = ms;
    ++n;
    dcue::timer_release(pr.first);
    dcue::timer_release(pr.second);
  }
  rec.clear();
  *launches_host = n;
  return DCUE_OK;
}
