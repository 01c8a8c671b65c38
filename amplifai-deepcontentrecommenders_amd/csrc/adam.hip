// torch.optim.Adam over the flat dense buffer and the user table, plus the weight repack -- gfx950.
// Reference: optim.Adam as built at nn/dcue.py:143-147 and stepped at :209 (CPU single-tensor path).
#include <mutex>
#include <unordered_map>

#include "dcue_internal.h"
#include "tgemm.h"
#include "bn0adam.h"


DCUE_KTRACE_READER(adam)  // diagnostic builds only (dcue_common.h): kernel 0 = k_user_fwd

namespace dcue {

// (m, v) = (+0, +0) is a fixed point of the zero-gradient step without weight decay (adam_zero_elem:
// m - w*0 = +0, v*b2 = +0, sqrt(0)/bc2 = 0, denom = eps, p + (-lr_bc1)*(0/eps) = p + (-0) = p,
// signed zeros included): a user row never in a batch needs no replay, bit for bit what the dense
// sweep computes. The replay kernels skip such elements (no loads of p, no stores).
__device__ __forceinline__ bool idle_moments(float m, float v) {
  return (__float_as_uint(m) | __float_as_uint(v)) == 0u;
}
__device__ __forceinline__ bool idle_moments4(const float4& m, const float4& v) {
  return (__float_as_uint(m.x) | __float_as_uint(m.y) | __float_as_uint(m.z) | __float_as_uint(m.w) |
          __float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z) | __float_as_uint(v.w)) == 0u;
}
// The replay bound (adam_replay.h) of the staged window [j0, j1] (history slots j % cap in LDS),
// folded by wave 0 and published to *out; the caller syncs the block before reading it.
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}
__device__ __forceinline__ float wave_min(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o));
  return x;
}
__device__ __forceinline__ int wave_and(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x &= __shfl_xor(x, o);
  return x;
}
__device__ __forceinline__ void window_bound(const AdamScalars* hs, int j0, int j1, int cap, float gz,
                                             ReplayBound* out) {
  if (threadIdx.x >= 64) return;
  ReplayBound b = bound_init(gz);
  for (int j = j0 + (int)threadIdx.x; j <= j1; j += 64) bound_fold(b, hs[j % cap]);
  b.S = wave_max(b.S);
  b.b2min = wave_min(b.b2min);
  b.eps = wave_min(b.eps);
  b.ok = wave_and(b.ok);
  b.nd = wave_and(b.nd);
  if (threadIdx.x == 0) {
    bound_finalize(b, j1 - j0 + 1);
    *out = b;
  }
}

// frozen rows (adam_replay.h): a frozen row is brought current (m / v only) by the rolling slice once
// it is this many flush periods behind, so a later reader's recurrence stays short
constexpr int kFrzRefreshCaps = 8;

struct PackArgs;
PackArgs pack_args(const dcue_model* md, const int64_t* poff);
// conv layers 1..5, then the text conv (text tower; an empty segment otherwise)
constexpr int kPackSegs = 6;
struct PackArgs {
  PackSeg seg[kPackSegs];
};

// Packed position of element e of conv segment sg (W[o][c][k], k fastest): the forward B operand
// [k][cin/4][cout][4] and (layers >= 2) the dgrad one [ks-1-k][cout/4][cin][4].

// Adam over the flat dense buffer with the conv-weight repack fused in: a float4 that lies in a
// conv weight segment (segments are 4-float aligned) also writes its four packed copies.
// gdiv > 0: the gradient is an all-reduced sum over gdiv ranks; it becomes the mean first (stored
// back, as grad.div_(world) leaves it) -- DDP's averaging fused into the sweep.
// [lo, n) of the buffer (lo a multiple of 4): the plan's split step runs the head and the tail of
// the flat buffer as two launches on two streams.
__global__ __launch_bounds__(256) void k_adam_dense_pack(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         long lo, long n, AdamScalars s, PackArgs pa,
                                                         float* __restrict__ wpack, float gdiv, unsigned* sig) {
  const long n4 = n / 4;
  for (long i = lo / 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = ld4(p + 4 * i), gg = ld4(g + 4 * i), mm = ld4(m + 4 * i), vv = ld4(v + 4 * i);
    if (gdiv > 0.f) {
      gg.x = __fdiv_rn(gg.x, gdiv); gg.y = __fdiv_rn(gg.y, gdiv);
      gg.z = __fdiv_rn(gg.z, gdiv); gg.w = __fdiv_rn(gg.w, gdiv);
      st4(g + 4 * i, gg);
    }
    adam_elem(pp.x, gg.x, mm.x, vv.x, s);
    adam_elem(pp.y, gg.y, mm.y, vv.y, s);
    adam_elem(pp.z, gg.z, mm.z, vv.z, s);
    adam_elem(pp.w, gg.w, mm.w, vv.w, s);
    st4(p + 4 * i, pp); st4(m + 4 * i, mm); st4(v + 4 * i, vv);
    const long e0 = 4 * i;
#pragma unroll
    for (int q = 0; q < kPackSegs; ++q) {
      const PackSeg& sg = pa.seg[q];
      const long len = (long)sg.cout * sg.cin * sg.ks;
      if (e0 >= sg.src && e0 < sg.src + len) {
        const long e = e0 - sg.src;
        pack_store(sg, e + 0, pp.x, wpack);
        pack_store(sg, e + 1, pp.y, wpack);
        pack_store(sg, e + 2, pp.z, wpack);
        pack_store(sg, e + 3, pp.w, wpack);
      }
    }
  }
  for (long i = max(4 * n4, lo) + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    float gi = g[i];  // tail past the last float4: never a conv weight
    if (gdiv > 0.f) g[i] = gi = __fdiv_rn(gi, gdiv);
    adam_elem(p[i], gi, m[i], v[i], s);
  }
  dev_signal_wg(sig);  // (plans: the late segments' Adam, for the next step's conv 2)
}

// User table: one wave per row; rows without a gradient this step get g = 0 (the reference's dense
// embedding gradient), then the row's slot is cleared for the next step.
__global__ __launch_bounds__(256) void k_adam_embed(float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v,
                                                    const float* __restrict__ gcompact,
                                                    int32_t* slot, long n_rows, int E, AdamScalars s) {
  const int lane = threadIdx.x & 63;
  const long wave0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave0; r < n_rows; r += nwaves) {
    const int sl = slot[r];
    float* pr = p + r * E;
    float* mr = m + r * E;
    float* vr = v + r * E;
    const float* gr = sl >= 0 ? gcompact + (long)sl * E : nullptr;
    if ((E & 3) == 0) {
      for (int k4 = lane; k4 < E / 4; k4 += 64) {
        float4 pp = ld4(pr + 4 * k4), mm = ld4(mr + 4 * k4), vv = ld4(vr + 4 * k4);
        const float4 gg = gr ? ld4(gr + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        adam_elem(pp.x, gg.x, mm.x, vv.x, s);
        adam_elem(pp.y, gg.y, mm.y, vv.y, s);
        adam_elem(pp.z, gg.z, mm.z, vv.z, s);
        adam_elem(pp.w, gg.w, mm.w, vv.w, s);
        st4(pr + 4 * k4, pp); st4(mr + 4 * k4, mm); st4(vr + 4 * k4, vv);
      }
    } else {
      for (int k = lane; k < E; k += 64) adam_elem(pr[k], gr ? gr[k] : 0.f, mr[k], vr[k], s);
    }
    if (lane == 0 && sl >= 0) slot[r] = -1;
  }
}

// ------------------------------------------------------------- deferred user-table Adam
// The dense sweep's zero-gradient steps, replayed late with the recorded scalars of each step.
// adam_elem is the same function (and `gz` a runtime 0.0f), so every replayed element goes through
// the identical fp32 operation sequence as in k_adam_embed: results are bit-identical.
__device__ __forceinline__ AdamScalars* log_hist(dcue_emb_log* hdr) {
  return reinterpret_cast<AdamScalars*>(hdr + 1);
}

// Bring users' rows current to step_done (before a forward reads them). One workgroup per listed
// user; a row listed twice is claimed by one workgroup (CAS on its clock; INT_MIN = in progress).
__global__ __launch_bounds__(1024) void k_emb_sync(float* __restrict__ p, float* __restrict__ m,
                                                  float* __restrict__ v, dcue_emb_log* hdr,
                                                  int32_t* emb_step, const int64_t* users, int E,
                                                  float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ ReplayBound sb;
  __shared__ int s_from;
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  const int64_t u = users[blockIdx.x];
  __shared__ int s_frz;
  if (threadIdx.x == 0) {
    int from = T;  // nothing to do
    const int old = emb_step[u];
    if (old != INT_MIN && max(clock_of(old), F) < T && atomicCAS(&emb_step[u], old, INT_MIN) == old)
      from = max(clock_of(old), F);
    s_from = from;
    s_frz = is_frozen(old);
  }
  __syncthreads();
  const int from = s_from;
  if (from >= T) return;
  const AdamScalars* hist = log_hist(hdr);
  for (int j = from + 1 + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  __syncthreads();
  window_bound(hs, from + 1, T, cap, gz, &sb);
  __syncthreads();
  const ReplayBound b = sb;
  float* pr = p + u * E;
  float* mr = m + u * E;
  float* vr = v + u * E;
  // one element per thread: each element's replay is a dependent chain of VALU-bound steps, so the
  // row is spread over as many lanes as it has elements (launch: blockDim >= E)
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    float mm[1] = {mr[k]}, vv[1] = {vr[k]};
    if (idle_moments(mm[0], vv[0]) && (b.nd || s_frz)) continue;  // fixed point (idle_moments)
    if (s_frz) {  // frozen: the m / v recurrence, p unchanged (adam_replay.h)
      frz_replay(mm[0], vv[0], hs[T % cap].lerp_c, hs[T % cap].b2, T - from);
      mr[k] = mm[0]; vr[k] = vv[0];
      continue;
    }
    float pp[1] = {pr[k]};
    replay_run<1>(pp, mm, vv, hs, from + 1, T, cap, b, gz);
    pr[k] = pp[0]; mr[k] = mm[0]; vr[k] = vv[0];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    emb_step[u] = T;
  }
}

// Every row current to step_done. Lanes walk the outstanding steps in lockstep (LDS broadcast of
// each step's scalars) and skip the steps their row already has.
__global__ __launch_bounds__(256) void k_emb_flush(float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, const dcue_emb_log* hdr,
                                                   const int32_t* __restrict__ emb_step, long n_rows,
                                                   int E, float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ ReplayBound sb;
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  if (T <= F) return;
  const AdamScalars* hist = log_hist(const_cast<dcue_emb_log*>(hdr));
  // Only the ring's live window [lo, T] is staged (slot j % cap): the full flush may come thousands
  // of steps after the previous one, but the rolling slices keep every row within `cap` steps of T,
  // so no row needs an entry older than lo.
  const int lo = max(F + 1, T - cap + 1);
  for (int j = lo + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  __syncthreads();
  window_bound(hs, lo, T, cap, gz, &sb);
  __syncthreads();
  const ReplayBound b = sb;
  const long stride = (long)gridDim.x * blockDim.x;
  if ((E & 3) == 0) {
    const int E4 = E >> 2;
    const long n4 = n_rows * E4;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const int e = emb_step[i / E4];
      const int from = max(clock_of(e), F);
      const float4 m4 = ld4(m + 4 * i), v4 = ld4(v + 4 * i);
      if (idle_moments4(m4, v4) && (b.nd || is_frozen(e))) continue;  // fixed point (idle_moments)
      if (is_frozen(e)) {  // the recurrence from the row's own clock, however old (no history needed)
        float mm[4] = {m4.x, m4.y, m4.z, m4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
        frz_replay_n<4>(mm, vv, hs[T % cap].lerp_c, hs[T % cap].b2, T - from);
        st4(m + 4 * i, make_float4(mm[0], mm[1], mm[2], mm[3]));
        st4(v + 4 * i, make_float4(vv[0], vv[1], vv[2], vv[3]));
        continue;
      }
      const float4 p4 = ld4(p + 4 * i);
      float pp[4] = {p4.x, p4.y, p4.z, p4.w}, mm[4] = {m4.x, m4.y, m4.z, m4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
      replay_run<4>(pp, mm, vv, hs, max(from + 1, lo), T, cap, b, gz);
      // a long-idle element's replay leaves p bit-identical (adam_replay.h): no store then (the
      // flush's HBM traffic is p, m, v read and written; most rows skip a sixth of it)
      if ((__float_as_uint(pp[0]) ^ __float_as_uint(p4.x)) | (__float_as_uint(pp[1]) ^ __float_as_uint(p4.y)) |
          (__float_as_uint(pp[2]) ^ __float_as_uint(p4.z)) | (__float_as_uint(pp[3]) ^ __float_as_uint(p4.w)))
        st4(p + 4 * i, make_float4(pp[0], pp[1], pp[2], pp[3]));
      st4(m + 4 * i, make_float4(mm[0], mm[1], mm[2], mm[3]));
      st4(v + 4 * i, make_float4(vv[0], vv[1], vv[2], vv[3]));
    }
  } else {
    const long n = n_rows * E;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const int e = emb_step[i / E];
      const int from = max(clock_of(e), F);
      float mm[1] = {m[i]}, vv[1] = {v[i]};
      if (idle_moments(mm[0], vv[0]) && (b.nd || is_frozen(e))) continue;
      if (is_frozen(e)) {
        frz_replay(mm[0], vv[0], hs[T % cap].lerp_c, hs[T % cap].b2, T - from);
        m[i] = mm[0]; v[i] = vv[0];
        continue;
      }
      float pp[1] = {p[i]};
      replay_run<1>(pp, mm, vv, hs, max(from + 1, lo), T, cap, b, gz);
      p[i] = pp[0]; m[i] = mm[0]; v[i] = vv[0];
    }
  }
}

__global__ void k_emb_flush_done(dcue_emb_log* hdr) { hdr->flush_step = hdr->step_done; }

// ------------------------------------------------------------------- frozen-row epochs
// Thaw: every frozen row brought current to step_done by the recurrence (valid: every step up to it
// was inside the epoch) and its bit cleared -- before the first step outside the epoch is recorded.
__global__ __launch_bounds__(256) void k_emb_thaw(float* __restrict__ m, float* __restrict__ v,
                                                  const dcue_emb_log* hdr, int32_t* emb_step, long n_rows, int E,
                                                  int rows_per_block) {
  __shared__ int from_s[256], frz_s[256];
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  const AdamScalars last = log_hist(const_cast<dcue_emb_log*>(hdr))[T % cap];
  for (long rb = (long)blockIdx.x * rows_per_block; rb < n_rows; rb += (long)gridDim.x * rows_per_block) {
    const int nr = (int)min((long)rows_per_block, n_rows - rb);
    for (int i = threadIdx.x; i < nr; i += blockDim.x) {
      const int e = emb_step[rb + i];
      from_s[i] = max(clock_of(e), F);
      frz_s[i] = is_frozen(e);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nr * E; e += blockDim.x) {
      const int i = e / E;
      if (!frz_s[i] || from_s[i] >= T) continue;
      const long off = (rb + i) * E + (e - i * E);
      float mm = m[off], vv = v[off];
      if (idle_moments(mm, vv)) continue;
      frz_replay(mm, vv, last.lerp_c, last.b2, T - from_s[i]);
      m[off] = mm; v[off] = vv;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nr; i += blockDim.x)
      if (frz_s[i]) emb_step[rb + i] = max(from_s[i], T);
    __syncthreads();
  }
}

__global__ void k_frz_set(dcue_emb_log* hdr, int start, float S, float eps) {
  hdr->frz_start = start;
  hdr->frz_S = S;
  hdr->frz_eps = eps;
}

namespace {
struct FrzHost {
  bool on = false;
  float S = 0.f, eps = 0.f, lc = 0.f, b2 = 0.f;
};
std::mutex& frz_mu() {
  static std::mutex m;
  return m;
}
std::unordered_map<const void*, FrzHost>& frz_map() {
  static std::unordered_map<const void*, FrzHost> m;
  return m;
}
// DCUE_FROZEN_ROWS=0: no epochs, no frozen rows (A/B; the replay is then rounds 1-5's)
bool frozen_rows_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_FROZEN_ROWS");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

void frz_forget(const dcue_emb_log* hdr) {
  std::lock_guard<std::mutex> lk(frz_mu());
  frz_map().erase(hdr);
}

// Before step t's scalars are recorded into the log (on the recording kernel's stream): a step
// outside the current epoch thaws every frozen row first; a step that admits frozen rows opens an
// epoch bounded by its own |neg_step| and eps (the first Adam step's lr / (1 - beta1) bounds every
// later step of a schedule that never raises lr above its start).
int frz_before_record(const dcue_model* md, const AdamScalars& sc, int t, hipStream_t s) {
  if (!frozen_rows_on() || !md->emb_step || !md->emb_log) return DCUE_OK;
  std::lock_guard<std::mutex> lk(frz_mu());
  FrzHost& f = frz_map()[md->emb_log];
  const float a = fabsf(sc.neg_step);
  const bool q = sc.wd == 0.f && !std::signbit(sc.lerp_c) && sc.lerp_c >= 0.f && sc.lerp_c < 0.5f && sc.eps > 0.f &&
                 sc.b2 >= 0.f && sc.b2 < 1.f && sc.bc2_sqrt > 0.f && sc.bc2_sqrt <= 1.f && a <= 0x1p60f;
  if (f.on && (!q || sc.lerp_c != f.lc || sc.b2 != f.b2 || a > f.S || sc.eps < f.eps)) {
    const int E = md->dims.user_embdim;
    int rpb = 4096 / E;
    rpb = rpb < 1 ? 1 : (rpb > 256 ? 256 : rpb);
    long blocks = (md->dims.n_users + rpb - 1) / rpb;
    blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
    DCUE_LAUNCH(k_emb_thaw, dim3((unsigned)blocks), dim3(256), 0, s, md->emb_exp_avg, md->emb_exp_avg_sq,
                md->emb_log, md->emb_step, (long)md->dims.n_users, E, rpb);
    DCUE_LAUNCH_CHECK();
    DCUE_LAUNCH(k_frz_set, dim3(1), dim3(1), 0, s, md->emb_log, 0, 0.f, 0.f);
    DCUE_LAUNCH_CHECK();
    f.on = false;
  }
  if (!f.on && q) {
    f.on = true;
    f.S = a; f.eps = sc.eps; f.lc = sc.lerp_c; f.b2 = sc.b2;
    DCUE_LAUNCH(k_frz_set, dim3(1), dim3(1), 0, s, md->emb_log, t, a, sc.eps);
    DCUE_LAUNCH_CHECK();
  }
  return DCUE_OK;
}

// Rolling flush: at step t the rows of chunk t mod cap (a contiguous 1/cap of the table) are brought
// current, so every row is replayed at least once per `cap` steps -- the replay work spread evenly
// over the steps (it runs on the user-tower stream, beside the item tower) instead of a full-table
// sweep every cap steps. A workgroup owns whole rows: it reads their clocks, replays, then sets them.
// Round 6: the grid strides over groups of rows_per_block rows, so DCUE_SLICE_WGS can bound it (A/B
// diagnostic for the steady-state tax). Bounds of 64-512 workgroups made the slice
// slower without shortening the critical path, so the default stays one workgroup
// per group; a workgroup stages the window's history and replay bound once for all its groups.
__global__ __launch_bounds__(256) void k_emb_flush_rows(float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, const dcue_emb_log* hdr,
                                                        int32_t* emb_step, long r0, long r1, int E,
                                                        int rows_per_block, float gz) {
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ ReplayBound sb;
  __shared__ int from_s[256], mode_s[256], frz_s[256];
  const int T = hdr->step_done, F = hdr->flush_step, cap = hdr->cap;
  if (r0 + (long)blockIdx.x * rows_per_block >= r1) return;
  // frozen rows (adam_replay.h): under an epoch, a replayed row whose every element is long idle for
  // any future step gets the frozen bit; frozen rows are skipped, or -- once kFrzRefresh steps behind
  // -- only their m / v are brought current (the recurrence; no p traffic), so a later reader's replay
  // stays short
  const bool epoch = hdr->frz_start > 0 && T >= hdr->frz_start - 1;
  const float fS = hdr->frz_S, feps = hdr->frz_eps;
  const int refresh = kFrzRefreshCaps * cap;
  const AdamScalars* hist = reinterpret_cast<const AdamScalars*>(hdr + 1);
  const int lo = max(F + 1, T - cap + 1);
  for (int j = lo + (int)threadIdx.x; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
  __syncthreads();
  window_bound(hs, lo, T, cap, gz, &sb);
  __syncthreads();
  const ReplayBound b = sb;
  for (long rb = r0 + (long)blockIdx.x * rows_per_block; rb < r1; rb += (long)gridDim.x * rows_per_block) {
    const int nr = (int)min((long)rows_per_block, r1 - rb);
    for (int i = threadIdx.x; i < nr; i += blockDim.x) {
      const int e = emb_step[rb + i];
      const int from = max(clock_of(e), F);
      from_s[i] = from;
      // 0: replay (history), 1: frozen, refresh m / v, 2: frozen, skip
      mode_s[i] = !is_frozen(e) ? 0 : (T - from >= refresh ? 1 : 2);
      frz_s[i] = epoch ? 1 : 0;
    }
    __syncthreads();
    const float lc = hs[T % cap].lerp_c, b2 = hs[T % cap].b2;  // (the epoch's constants)
    if ((E & 3) == 0) {
      const int E4 = E >> 2;
      for (int e = threadIdx.x; e < nr * E4; e += blockDim.x) {
        const int i = e / E4;
        const int md = mode_s[i];
        if (md == 2) continue;
        const long off = (rb + i) * E + 4 * (e - i * E4);
        const float4 m4 = ld4(m + off), v4 = ld4(v + off);
        if (idle_moments4(m4, v4) && (b.nd || md == 1)) continue;  // fixed point (idle_moments)
        float mm[4] = {m4.x, m4.y, m4.z, m4.w}, vv[4] = {v4.x, v4.y, v4.z, v4.w};
        if (md == 1) {
          frz_replay_n<4>(mm, vv, lc, b2, T - from_s[i]);
        } else {
          const float4 p4 = ld4(p + off);
          float pp[4] = {p4.x, p4.y, p4.z, p4.w};
          replay_run<4>(pp, mm, vv, hs, from_s[i] + 1, T, cap, b, gz);
          if ((__float_as_uint(pp[0]) ^ __float_as_uint(p4.x)) | (__float_as_uint(pp[1]) ^ __float_as_uint(p4.y)) |
              (__float_as_uint(pp[2]) ^ __float_as_uint(p4.z)) | (__float_as_uint(pp[3]) ^ __float_as_uint(p4.w)))
            st4(p + off, make_float4(pp[0], pp[1], pp[2], pp[3]));  // long-idle: p unchanged, no store
          if (epoch) {
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 4; ++q) ok &= frz_elem_ok(pp[q], mm[q], vv[q], fS, feps);
            if (!ok) frz_s[i] = 0;
          }
        }
        st4(m + off, make_float4(mm[0], mm[1], mm[2], mm[3]));
        st4(v + off, make_float4(vv[0], vv[1], vv[2], vv[3]));
      }
    } else {
      for (int e = threadIdx.x; e < nr * E; e += blockDim.x) {
        const int i = e / E;
        const int md = mode_s[i];
        if (md == 2) continue;
        const long off = (rb + i) * E + (e - i * E);
        float mm[1] = {m[off]}, vv[1] = {v[off]};
        if (idle_moments(mm[0], vv[0]) && (b.nd || md == 1)) continue;
        if (md == 1) {
          frz_replay(mm[0], vv[0], lc, b2, T - from_s[i]);
        } else {
          float pp[1] = {p[off]};
          replay_run<1>(pp, mm, vv, hs, from_s[i] + 1, T, cap, b, gz);
          p[off] = pp[0];
          if (epoch && !frz_elem_ok(pp[0], mm[0], vv[0], fS, feps)) frz_s[i] = 0;
        }
        m[off] = mm[0]; v[off] = vv[0];
      }
    }
    __syncthreads();  // (every replay read from_s; the rows' values before their clocks)
    for (int i = threadIdx.x; i < nr; i += blockDim.x) {
      const int md = mode_s[i];
      if (md == 2) continue;  // (frozen, left behind)
      emb_step[rb + i] = T | (md == 1 || frz_s[i] ? kFrozenBit : 0);
    }
  }
}

int launch_emb_flush_rows(const dcue_model* md, int step, hipStream_t s) {
  const long n = md->dims.n_users;
  const int cap = md->emb_log_cap, E = md->dims.user_embdim;
  const int k = step % cap;
  const long r0 = n * k / cap, r1 = n * (k + 1) / cap;
  if (r1 <= r0) return DCUE_OK;
  int rpb = 4096 / E;  // rows per group: ~4 K elements (1 K float4) per pass of 256 threads
  if (rpb < 1) rpb = 1;
  if (rpb > 256) rpb = 256;
  static const long max_wgs = [] {
    const char* e = getenv("DCUE_SLICE_WGS");
    const long v = e ? atol(e) : 1L << 30;
    return v < 1 ? 1L : v;
  }();
  long blocks = (r1 - r0 + rpb - 1) / rpb;
  if (blocks > max_wgs) blocks = max_wgs;
  TimerScope tsc;
  int st = timer_begin(&tsc, DCUE_TIMED_EMB_SLICE, s);
  if (st) return st;
  DCUE_LAUNCH(k_emb_flush_rows, dim3((unsigned)blocks), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, r0, r1, E, rpb, 0.f);
  DCUE_LAUNCH_CHECK();
  return timer_end(&tsc);
}



static AdamScalars form_scalars(const dcue_adam_args* a);
// Step t for the rows that have a gradient (emb_rows from the backward); records step t's scalars.
__global__ __launch_bounds__(256) void k_adam_touched(float* __restrict__ p, float* __restrict__ m,
                                                      float* __restrict__ v,
                                                      const float* __restrict__ gcompact,
                                                      const int64_t* emb_rows, int32_t* emb_step,
                                                      dcue_emb_log* hdr, int E, int t, AdamScalars s,
                                                      float gz) {
  __shared__ int s_from;
  const int cap = hdr->cap, F = hdr->flush_step;
  const int n = hdr->grad_step == t ? hdr->n_touched : 0;
  const AdamScalars* hist = log_hist(hdr);
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    const int64_t u = emb_rows[b];
    if (u < 0) continue;
    if (threadIdx.x == 0) {
      const int e = emb_step[u];
      s_from = max(clock_of(e), F) | (is_frozen(e) ? kFrozenBit : 0);
    }
    __syncthreads();
    const int from = clock_of(s_from);
    const bool frz = is_frozen(s_from);
    float* pr = p + u * E;
    float* mr = m + u * E;
    float* vr = v + u * E;
    const float* gr = gcompact + (long)b * E;
    for (int k = threadIdx.x; k < E; k += blockDim.x) {
      float pp = pr[k], mm = mr[k], vv = vr[k];
      if (frz && from + 1 < t)  // (frozen: the recurrence with the epoch's constants, step t-1's)
        frz_replay(mm, vv, hist[(t - 1) % cap].lerp_c, hist[(t - 1) % cap].b2, t - 1 - from);
      else
        for (int j = from + 1; j < t; ++j) adam_replay(pp, mm, vv, hist[j % cap], gz);  // normally none
      adam_elem(pp, gr[k], mm, vv, s);
      pr[k] = pp; mr[k] = mm; vr[k] = vv;
    }
    __syncthreads();
    if (threadIdx.x == 0) emb_step[u] = t;
    __syncthreads();  // (s_from's next write)
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    log_hist(hdr)[t % cap] = s;
    hdr->step_done = t;
  }
}

// k_emb_grad (tail.hip) and k_adam_touched in one launch: workgroup b owns batch row b; a repeated
// user's first row sums the user's rows in batch order (the compact gradient, as k_emb_grad), and
// the same workgroup then steps the user's table row (as k_adam_touched: missed zero-gradient steps
// replayed first -- normally none -- then adam_elem). Workgroup 0 records the step's scalars.
__global__ __launch_bounds__(256) void k_emb_grad_adam(const float* __restrict__ de, const int64_t* users, int B,
                                                       int E, float scale, float* __restrict__ emb_grad,
                                                       int32_t* slot, int64_t* emb_rows, float* __restrict__ p,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       int32_t* emb_step, dcue_emb_log* hdr, int t, AdamScalars s,
                                                       float gz) {
  const int b = blockIdx.x;
  const int64_t u = users[b];
  const int cap = hdr->cap, F = hdr->flush_step;
  if (b == 0 && threadIdx.x == 0) {
    hdr->n_touched = B;
    hdr->grad_step = t;
  }
  bool first = true;
  for (int r = 0; r < b; ++r) first &= users[r] != u;
  if (!first) {
    if (threadIdx.x == 0) emb_rows[b] = -1;
  } else {
    const int e0 = emb_step[u];
    const int from = max(clock_of(e0), F);
    const bool frz = is_frozen(e0);
    const AdamScalars* hist = log_hist(hdr);
    float* pr = p + u * E;
    float* mr = m + u * E;
    float* vr = v + u * E;
    for (int k = threadIdx.x; k < E; k += blockDim.x) {
      float gsum = 0.f;
      for (int r = b; r < B; ++r)
        if (users[r] == u) gsum += de[(long)r * E + k];
      const float g = gsum * scale;
      emb_grad[(long)b * E + k] = g;
      float pp = pr[k], mm = mr[k], vv = vr[k];
      if (frz && from + 1 < t)  // (frozen: the recurrence with the epoch's constants, step t-1's)
        frz_replay(mm, vv, hist[(t - 1) % cap].lerp_c, hist[(t - 1) % cap].b2, t - 1 - from);
      else
        for (int j = from + 1; j < t; ++j) adam_replay(pp, mm, vv, hist[j % cap], gz);  // normally none
      adam_elem(pp, g, mm, vv, s);
      pr[k] = pp; mr[k] = mm; vr[k] = vv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      slot[u] = b;
      emb_rows[b] = u;
      emb_step[u] = t;
    }
  }
  if (b == 0 && threadIdx.x == 0) {
    log_hist(hdr)[t % cap] = s;
    hdr->step_done = t;
  }
}

int launch_emb_grad_adam(const dcue_model* md, const dcue_adam_args* a, const float* de, const int64_t* users, int B,
                         float scale, hipStream_t s) {
  if (!md->emb_step || !md->emb_rows || !md->emb_log) return DCUE_ERR_INVALID;
  const AdamScalars sc = form_scalars(a);
  TRY(frz_before_record(md, sc, a->step, s));
  DCUE_LAUNCH(k_emb_grad_adam, dim3((unsigned)B), dim3(256), 0, s, de, users, B, md->dims.user_embdim, scale,
              md->emb_grad, md->emb_slot, md->emb_rows, md->emb, md->emb_exp_avg, md->emb_exp_avg_sq, md->emb_step,
              md->emb_log, a->step, sc, 0.f);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// ------------------------------------------------------------------- fused user-tower forward
// userembedding.py:33-44 for 16 users per workgroup, in one launch: (deferred mode) the rows brought
// current, then h1 = relu(E[u]) W1^T + b1 and uf = relu(h1) W2^T + b2. Replaces k_emb_sync and two
// k_tgemm launches with the same arithmetic:
//  * sync: each row replays its missed zero-gradient steps with replay_run (bound over the live window
//    [lo, T], a superset of the row's own: still exact, adam_replay.h); a row listed twice in the batch
//    is claimed by one workgroup (CAS on its clock, INT_MIN = in progress, as k_emb_sync) and any other
//    workgroup that reads it waits, bounded, for the claimer's release of the clock;
//  * the GEMMs are tgemm_block's 16 x 64 blocks (tgemm.h), two at a time (threads 0-255 / 256-511),
//    so h1 and uf are bit-identical to the k_tgemm launches. h1 goes through global memory: written
//    and read back by this workgroup's own waves only (one CU's L1), ordered by the block barrier.
struct UserFwdArgs {
  TGemmArgs g1, g2;
  float *p, *m, *v;        // the table and its Adam moments (deferred mode)
  dcue_emb_log* hdr;
  int32_t* emb_step;       // null: dense mode, every row already current
  const int64_t* users;
  int B, E;
  unsigned* fail;          // set when a wait for another workgroup's claim gave up (never expected)
  unsigned* sig;           // plans: +1 per workgroup once its uf rows are stored (dev_signal_wg)
};

// 256-thread GEMM parts per workgroup. (3 -- 768 threads, 2 GEMM-1 rounds instead of 3 -- fits the
// LDS, 159 KB, but not the registers at 3 waves per SIMD: 93 VGPRs spilled; not kept, round 6)
constexpr int kUfParts = 2;
__global__ __launch_bounds__(256 * kUfParts) void k_user_fwd(UserFwdArgs a) {
  __shared__ TgLds L[kUfParts];
  __shared__ AdamScalars hs[DCUE_MAX_LOG_CAP];
  __shared__ ReplayBound sb;
  __shared__ int from_s[16], claim_s[16];
  __shared__ int64_t user_s[16];
  DCUE_KTW(0, 6);
  DCUE_KT(0, 0);
  const int t = threadIdx.x, half = t >> 8, th = t & 255;
  const int r0 = blockIdx.x * 16, nr = min(16, a.B - r0);
  if (a.emb_step) {
    const int T = a.hdr->step_done, F = a.hdr->flush_step, cap = a.hdr->cap;
    if (t < nr) {
      const int64_t u = a.users[r0 + t];
      user_s[t] = u;
      const int old = a.emb_step[u];
      int from = T, claimed = 0;
      if (old != INT_MIN && max(clock_of(old), F) < T && atomicCAS(&a.emb_step[u], old, INT_MIN) == old) {
        from = max(clock_of(old), F);
        claimed = is_frozen(old) ? 2 : 1;  // (2: frozen, the m / v recurrence)
      }
      from_s[t] = from;
      claim_s[t] = claimed;
    }
    const int lo = max(F + 1, T - cap + 1);
    const AdamScalars* hist = log_hist(a.hdr);
    for (int j = lo + t; j <= T; j += blockDim.x) hs[j % cap] = hist[j % cap];
    __syncthreads();
    DCUE_KT(0, 1);
    // (lo > T: nothing to replay -- no row is claimed -- but sb is still read below: give it a value)
    if (lo <= T) window_bound(hs, lo, T, cap, 0.f, &sb);
    else if (t == 0) sb = ReplayBound{};
    __syncthreads();
    const ReplayBound b = sb;
    // A thread's elements in groups of kUfG: the group's p / m / v loads go out together (clamped,
    // unconditional), then the replays run -- one load latency a group instead of one an element
    // (round 6: the replay phase was 30 us of the workgroup's 80, per-workgroup trace)
    constexpr int kUfG = 8;
    const int tot = nr * a.E;
    for (int e0 = t; e0 < tot; e0 += kUfG * (int)blockDim.x) {
      float pg[kUfG], mg[kUfG], vg[kUfG];
      long og[kUfG];
      int cg[kUfG], fg[kUfG];
#pragma unroll
      for (int j = 0; j < kUfG; ++j) {
        const int e = e0 + j * (int)blockDim.x;
        const int ec = e < tot ? e : e0;
        const int i = ec / a.E, k = ec - i * a.E;
        cg[j] = e < tot ? claim_s[i] : 0;
        fg[j] = from_s[i];
        og[j] = user_s[i] * a.E + k;
        mg[j] = a.m[og[j]];
        vg[j] = a.v[og[j]];
        pg[j] = a.p[og[j]];
      }
#pragma unroll
      for (int j = 0; j < kUfG; ++j) {
        if (!cg[j]) continue;
        const long off = og[j];
        float mm[1] = {mg[j]}, vv[1] = {vg[j]};
        if (idle_moments(mm[0], vv[0]) && (b.nd || cg[j] == 2)) continue;  // fixed point (idle_moments)
        if (cg[j] == 2) {  // frozen (adam_replay.h): p unchanged
          frz_replay(mm[0], vv[0], hs[T % cap].lerp_c, hs[T % cap].b2, T - fg[j]);
          a.m[off] = mm[0]; a.v[off] = vv[0];
          continue;
        }
        float pp[1] = {pg[j]};
        replay_run<1>(pp, mm, vv, hs, fg[j] + 1, T, cap, b, 0.f);
        a.p[off] = pp[0]; a.m[off] = mm[0]; a.v[off] = vv[0];
      }
    }
    __syncthreads();
    DCUE_KT(0, 2);
    // Every claimed clock is released before any lane waits: claimers and waiters are lanes of one
    // wave, and a wave spinning with its claimer lanes masked off would never release them (two
    // workgroups each waiting for a row the other holds would then both spin to the bound).
    if (t < nr && claim_s[t]) {
      __threadfence();  // the row's replayed values before its clock (other workgroups wait on it)
      __hip_atomic_store(a.emb_step + user_s[t], T, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (t < nr && !claim_s[t]) {
      int32_t* clk = a.emb_step + user_s[t];
      unsigned spins = 0;
      while (__hip_atomic_load(clk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == INT_MIN) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 22)) {  // never expected: reported (dcue_debug_fail_flags), not silent
          atomicOr(a.fail, 1u);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  DCUE_KT(0, 3);
  // GEMM 1: the N / 64 column blocks kUfParts at a time (every part runs the same number of rounds: an
  // out-of-range block stores nothing). Per-workgroup trace (round 6, profiles/r06_ktrace_user_fwd.txt):
  // claims 2.4 us, replay 30, GEMM 1 34 (three rounds of two 16 x 64 blocks at E = 300), GEMM 2 12
  const int gy1 = (a.g1.N + 63) / 64, gy2 = (a.g2.N + 63) / 64;
  const int ry1 = (gy1 + kUfParts - 1) / kUfParts * kUfParts, ry2 = (gy2 + kUfParts - 1) / kUfParts * kUfParts;
  for (int by = half; by < ry1; by += kUfParts) tgemm_block<1, 0, 1, 0>(a.g1, blockIdx.x, by, L[half], th);
  __syncthreads();
  DCUE_KT(0, 4);
  for (int by = half; by < ry2; by += kUfParts) tgemm_block<1, 0, 1, 0>(a.g2, blockIdx.x, by, L[half], th);
  dev_signal_wg(a.sig);
  DCUE_KT(0, 5);
  DCUE_KTW(0, 7);
}

int user_fwd_blocks(int B) { return (B + 15) / 16; }

int launch_user_fwd(const dcue_model* md, const TGemmArgs& g1, const TGemmArgs& g2, const int64_t* users, int B,
                    hipStream_t s, unsigned* sig) {
  if (g1.sak != 1 || g1.sbn == 1 || g2.sak != 1 || g2.sbn == 1 || !g1.arow || g2.arow) return DCUE_ERR_INVALID;
  UserFwdArgs a;
  a.g1 = g1; a.g2 = g2;
  a.p = md->emb; a.m = md->emb_exp_avg; a.v = md->emb_exp_avg_sq;
  a.hdr = md->emb_log; a.emb_step = md->emb_step;
  a.users = users; a.B = B; a.E = md->dims.user_embdim;
  unsigned* const fail = user_fwd_fail_flag();  // this device's word (cached per device)
  if (!fail) return DCUE_ERR_HIP;
  a.fail = fail;
  a.sig = sig;
  DCUE_LAUNCH(k_user_fwd, dim3((unsigned)user_fwd_blocks(B)), dim3(256 * kUfParts), 0, s, a);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

__global__ void k_emb_log_init(dcue_emb_log* hdr, int cap, int step) {
  hdr->step_done = step;
  hdr->flush_step = step;
  hdr->n_touched = 0;
  hdr->grad_step = -1;
  hdr->cap = cap;
  hdr->frz_start = 0;
  hdr->frz_S = 0.f;
  hdr->frz_eps = 0.f;
}

int launch_emb_log_init(const dcue_model* md, int cap, int step, hipStream_t s) {
  frz_forget(md->emb_log);
  DCUE_HIP_CHECK(hipMemsetAsync(md->emb_step, 0, sizeof(int32_t) * md->dims.n_users, s));
  DCUE_LAUNCH(k_emb_log_init, dim3(1), dim3(1), 0, s, md->emb_log, cap, step);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_emb_sync(const dcue_model* md, const int64_t* users, int n, hipStream_t s) {
  if (n <= 0) return DCUE_OK;
  const int E = md->dims.user_embdim;
  const int threads = E <= 64 ? 64 : (E >= 1024 ? 1024 : (E + 63) / 64 * 64);
  DCUE_LAUNCH(k_emb_sync, dim3((unsigned)n), dim3(threads), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, users, md->dims.user_embdim, 0.f);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int launch_emb_flush(const dcue_model* md, hipStream_t s) {
  const long n = md->dims.n_users * (long)md->dims.user_embdim;
  long blocks = (n / 4 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  TimerScope tsc;
  int st = timer_begin(&tsc, DCUE_TIMED_EMB_FLUSH, s);
  if (st) return st;
  DCUE_LAUNCH(k_emb_flush, dim3((unsigned)blocks), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                     md->emb_exp_avg_sq, md->emb_log, md->emb_step, (long)md->dims.n_users,
                     md->dims.user_embdim, 0.f);
  DCUE_LAUNCH_CHECK();
  if ((st = timer_end(&tsc))) return st;
  DCUE_LAUNCH(k_emb_flush_done, dim3(1), dim3(1), 0, s, md->emb_log);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

// host scalars as torch.optim.Adam forms them from Python floats (double), each rounded once to
// float where the CPU kernel takes it as a float scalar
static AdamScalars form_scalars(const dcue_adam_args* a) {
  const double bc1 = 1.0 - pow(a->beta1, (double)a->step);
  const double bc2 = 1.0 - pow(a->beta2, (double)a->step);
  const double w = 1.0 - a->beta1;
  AdamScalars sc;
  sc.neg_step = (float)(-(a->lr / bc1));
  // sign bit = the lerp's base (adam_replay.h lerp_base_g): -(1 - w) is -0 at beta1 = 0
  sc.lerp_c = w < 0.5 ? (float)w : -(1.0f - (float)w);
  sc.b2 = (float)a->beta2;
  sc.one_m_b2 = (float)(1.0 - a->beta2);
  sc.bc2_sqrt = (float)pow(bc2, 0.5);  // bias_correction2 ** 0.5
  sc.eps = (float)a->eps;
  sc.wd = (float)a->weight_decay;
  sc.inv_bc2_sqrt = 1.0f / sc.bc2_sqrt;  // IEEE single division on the host: RN(1/bc2_sqrt)
  return sc;
}

// bn0's gradients + Adam over segments [0, DCUE_SEG_LATE) in one launch (dcue_internal.h Bn0Adam):
// workgroup c owns input channel c -- W1[:, c, :] (gradient, Adam, repack), bn0's gamma/beta[c] --
// and workgroups 0 / 1 conv 1's bias and bn1's gamma/beta (whose gradients the conv-1 weight
// gradient already wrote). Gradient arithmetic: bn0_elem, as k_bn0_grads; Adam: adam_elem, as the
// dense sweep -- the plan's fused step and an eager backward + dcue_adam_step agree bit for bit.

__global__ __launch_bounds__(256) void k_bn0_grads_adam(const float* __restrict__ G, const float* __restrict__ E,
                                                        const float* gamma0, const float* beta0, const float* mean0,
                                                        const float* invstd0, int H, float* dgamma0, float* dbeta0,
                                                        Bn0AdamDev a) {
  critical_path_priority();
  __shared__ float rg[256], rb[256];
  bn0_channel<true>(G, E, gamma0, beta0, mean0, invstd0, H, dgamma0, dbeta0, a, nullptr, nullptr, nullptr,
                    blockIdx.x, threadIdx.x, rg, rb, true);
}

Bn0AdamDev bn0adam_dev(const Bn0Adam& a) {
  const dcue_model* md = a.md;
  Bn0AdamDev d;
  d.p = md->params; d.m = md->exp_avg; d.v = md->exp_avg_sq; d.g = md->grads;
  d.o_w1 = a.poff[2]; d.o_cb1 = a.poff[3];
  d.o_g0 = a.bn ? a.poff[0] : -1; d.o_b0 = a.bn ? a.poff[1] : -1;
  d.o_g1 = a.bn ? a.poff[4] : -1; d.o_b1 = a.bn ? a.poff[5] : -1;
  d.sc = form_scalars(&a.args);
  d.seg1 = pack_args(md, a.poff).seg[0];
  d.wpack = md->wpack;
  return d;
}

int launch_bn0_grads_adam(const float* G, const float* E, const float* gamma0, const float* beta0,
                          const float* mean0, const float* invstd0, int H, float* dgamma0, float* dbeta0,
                          const Bn0Adam& a, hipStream_t s) {
  const dcue_model* md = a.md;
  if (H > 256) return DCUE_ERR_UNSUPPORTED;  // k_bn0_grads_adam: 4H elements over 4 x 256 threads
  if (!md->params || !md->grads || !md->exp_avg || !md->exp_avg_sq || a.args.grad_div > 1.0) return DCUE_ERR_INVALID;
  const Bn0AdamDev d = bn0adam_dev(a);
  DCUE_LAUNCH(k_bn0_grads_adam, dim3(kMels), dim3(256), 0, s, G, E, gamma0, beta0, mean0, invstd0, H, dgamma0,
              dbeta0, d);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

long adam_dense_blocks(long len) { return len >= 512L * 1024 ? 512 : (len / 4 + 255) / 256 + 1; }

int launch_adam(const dcue_model* md, const dcue_adam_args* a, const int64_t* poff, hipStream_t s,
                bool flush_slice, long dense_lo, long dense_hi, bool defer_dgrad2, unsigned* sig) {
  const AdamScalars sc = form_scalars(a);
  const float gdiv = a->grad_div > 1.0 ? (float)a->grad_div : 0.f;
  const int parts = a->parts ? a->parts : (DCUE_ADAM_DENSE | DCUE_ADAM_EMBEDDING);
  const long n = dense_hi >= 0 ? dense_hi : poff[DCUE_N_DENSE_SEGMENTS];
  if (parts & DCUE_ADAM_DENSE) {  // Adam + the conv-weight repack in one sweep
    const long len = n - dense_lo;
    const long blocks = adam_dense_blocks(len);
    PackArgs pa = pack_args(md, poff);
    if (defer_dgrad2) pa.seg[1].bwd = pa.seg[1].f16b = -1;  // (the next forward of conv 2 writes them)
    DCUE_LAUNCH(k_adam_dense_pack, dim3((unsigned)blocks), dim3(256), 0, s, md->params, md->grads, md->exp_avg,
                       md->exp_avg_sq, dense_lo, n, sc, pa, md->wpack, gdiv, sig);
    DCUE_LAUNCH_CHECK();
  }
  if ((parts & DCUE_ADAM_EMBEDDING) && md->emb_step) {
    TRY(frz_before_record(md, sc, a->step, s));
    DCUE_LAUNCH(k_adam_touched, dim3(256), dim3(256), 0, s, md->emb, md->emb_exp_avg,
                       md->emb_exp_avg_sq, md->emb_grad, md->emb_rows, md->emb_step, md->emb_log,
                       md->dims.user_embdim, a->step, sc, 0.f);
    DCUE_LAUNCH_CHECK();
    // this step's slice of the rolling flush (or the caller issues it later: StepOpts)
    return flush_slice ? launch_emb_flush_rows(md, a->step, s) : DCUE_OK;
  } else if ((parts & DCUE_ADAM_EMBEDDING) && md->dims.n_users > 0) {
    long blocks = (md->dims.n_users + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    TimerScope tsc;
    int st = timer_begin(&tsc, DCUE_TIMED_ADAM_EMBED, s);
    if (st) return st;
    DCUE_LAUNCH(k_adam_embed, dim3((unsigned)blocks), dim3(256), 0, s, md->emb,
                       md->emb_exp_avg, md->emb_exp_avg_sq, md->emb_grad, md->emb_slot,
                       (long)md->dims.n_users, md->dims.user_embdim, sc);
    DCUE_LAUNCH_CHECK();
    if ((st = timer_end(&tsc))) return st;
  }
  return DCUE_OK;
}

// ------------------------------------------------------------------------- weight packing
// conv layer l forward B operand: [k][cin/4][cout][4]; dgrad (l >= 2): [k'][cout/4][cin][4] with
// k' = ks-1-k.
__global__ void k_pack(const float* __restrict__ params, float* wpack, PackArgs pa) {
  const PackSeg sg = pa.seg[blockIdx.y];
  const long n = (long)sg.cout * sg.cin * sg.ks;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
    pack_store(sg, e, params[sg.src + e], wpack);  // W[o][c][k]
}

PackArgs pack_args(const dcue_model* md, const int64_t* poff) {
  const int H = st_hidden(&md->dims), d = st_feature(&md->dims);
  const WpackLayout wl = wpack_layout(&md->dims);
  PackArgs pa;
  for (int l = 1; l <= 5; ++l) {
    PackSeg& sg = pa.seg[l - 1];
    sg.cin = l == 1 ? kMels : H;
    sg.cout = l == 5 ? d : H;
    sg.ks = layer_geom(l).ks;
    sg.src = poff[2 + 4 * (l - 1)];  // conv.layer{l}.weight
    sg.fwd = wl.conv_fwd[l];
    sg.bwd = l >= 2 ? wl.conv_bwd[l] : -1;
    sg.f16 = wl.conv_f16[l];
    sg.f16b = l >= 2 ? wl.conv_f16b[l] : -1;
    sg.cinp = sg.cin;
  }
  PackSeg& tx = pa.seg[5];  // text.conv.weight [C_s][E_w][3]: the split-f16 forward operand only
  tx.cin = md->dims.word_dim;
  tx.cinp = st_word(&md->dims);
  tx.cout = st_text(&md->dims);
  tx.ks = 3;
  tx.src = poff[28];
  tx.fwd = tx.bwd = tx.f16b = -1;
  tx.f16 = wl.text_f16;
  if (!tower_text(&md->dims)) tx.cout = tx.cin = 0;  // empty: no element lies in it
  return pa;
}

PackSeg pack_seg(const dcue_model* md, const int64_t* poff, int l) { return pack_args(md, poff).seg[l - 1]; }

int launch_pack(const dcue_model* md, const int64_t* poff, hipStream_t s) {
  const PackArgs pa = pack_args(md, poff);
  DCUE_LAUNCH(k_pack, dim3(64, kPackSegs), dim3(256), 0, s, md->params, md->wpack, pa);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // namespace dcue
