// Schedule-perturbation and probe diagnostics (include/dcue.h "debug"), for finding missing
// cross-stream orders and the first kernel that writes a bad value.
//
// * Delays: dcue_debug_delay(site, us) makes every later step issue a spin kernel of `us`
//   microseconds on the stream of the work at `site`, ahead of that work. A step's results must be
//   bit-identical under any such delay: every buffer is read and written in an order the streams'
//   events impose, not in an order the usual timing happens to give. A difference under a delay
//   names a missing wait (tests/test_gpu_races.py).
// * Probes: with a probe buffer bound (dcue_debug_probes), the step issues after each probed launch,
//   on that launch's stream, a check of its output: any non-finite element ORs a flag and takes the
//   atomic minimum of the 100 MHz wall clock, any non-zero element ORs another. The probes add no
//   order between streams, so a race still shows; the earliest time stamp names the first kernel
//   whose output went non-finite.
// * The fused user-tower forward (adam.hip k_user_fwd) reports a bounded wait that gave up into a
//   device word read by dcue_debug_fail_flags.
// * Poison: dcue_debug_poison(1) fills the scratch a plan allocates itself (dcue_plan_create) with
//   0xFF bytes -- float NaN -- so a read of a word no kernel wrote shows as a non-finite result.
#include <atomic>

#include "dcue_internal.h"

namespace dcue {

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_delay_us[DCUE_N_DEBUG_SITES];
std::atomic<ProbeRec*> g_probes{nullptr};
std::atomic<bool> g_poison{false};

const char* const kProbeNames[kNumProbes] = {
    "conv1 forward (y1)", "conv2 forward (y2)", "conv3 forward (y3)", "conv4 forward (y4)", "conv5 forward (y5)",
    "user tower h1", "user tower (uf)", "item features (fc)", "score kernel (scores)", "score kernel (du)",
    "score kernel (dfcopy)", "item gradient (df)", "fc input gradient (g5)", "dgrad 5 (g4)", "dgrad 4 (g3)",
    "dgrad 3 (g2)", "dgrad 2 (g1)", "user tower backward (de)", "user tower weight gradients",
    "weight gradients 3-5 + fc", "weight gradient 2", "fc / text weight gradients", "conv-1 weight gradient",
    "Adam bn0 / conv1 / bn1 (params)", "late Adam (params)",
};

// spin on the 100 MHz wall clock (s_memrealtime: a scalar read, no stores) for `ticks`
__global__ void k_spin(long long ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)wall_clock64();
  while ((long long)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

__global__ __launch_bounds__(256) void k_probe(const float* __restrict__ x, long n, ProbeRec* rec) {
  bool bad = false, nz = false;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t u = __float_as_uint(x[i]);
    bad |= (u & 0x7f800000u) == 0x7f800000u;
    nz |= (u & 0x7fffffffu) != 0u;
  }
  const bool any_bad = __any(bad), any_nz = __any(nz);
  if ((threadIdx.x & 63) == 0) {
    if (any_bad) {
      atomicOr(&rec->nonfinite, 1u);
      atomicMin(&rec->first_bad, (unsigned long long)wall_clock64());
    }
    if (any_nz) atomicOr(&rec->nonzero, 1u);
  }
}
}  // namespace

// the fused user-tower forward's "a bounded wait gave up" word (adam.hip)
__device__ unsigned g_user_fwd_fail;

// The symbol's address differs per device: looked up on the current device, cached per device id.
unsigned* user_fwd_fail_flag() {
  static std::atomic<unsigned*> cache[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  if (dev < kMaxDevices) {
    unsigned* c = cache[dev].load(std::memory_order_acquire);
    if (c) return c;
  }
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_user_fwd_fail)) != hipSuccess) return nullptr;
  if (dev < kMaxDevices) cache[dev].store(static_cast<unsigned*>(p), std::memory_order_release);
  return static_cast<unsigned*>(p);
}

int debug_delay(int site, hipStream_t s) {
  if (site < 0 || site >= DCUE_N_DEBUG_SITES) return DCUE_OK;
  const int us = g_delay_us[site].load(std::memory_order_relaxed);
  if (us <= 0) return DCUE_OK;
  DCUE_LAUNCH(k_spin, dim3(1), dim3(64), 0, s, (long long)us * 100);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

bool probes_on() { return g_probes.load(std::memory_order_relaxed) != nullptr; }

int probe(int id, const float* x, long n, hipStream_t s) {
  ProbeRec* base = g_probes.load(std::memory_order_relaxed);
  if (!base || !x || n <= 0 || id < 0 || id >= kNumProbes) return DCUE_OK;
  const long b = (n + 255) / 256;
  DCUE_LAUNCH(k_probe, dim3((unsigned)(b < 1 ? 1 : b > 512 ? 512 : b)), dim3(256), 0, s, x, n, base + id);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

bool poison_on() { return g_poison.load(std::memory_order_relaxed); }

bool legacy_orders() {
  static const bool on = [] {
    const char* e = getenv("DCUE_LEGACY_ORDERS");
    return e && e[0] == '1';
  }();
  return on;
}

}  // namespace dcue

extern "C" {

int dcue_debug_delay(int32_t site, int32_t microseconds) {
  if (site < 0 || site >= DCUE_N_DEBUG_SITES || microseconds < 0 || microseconds > 1000000) return DCUE_ERR_INVALID;
  dcue::g_delay_us[site].store(microseconds, std::memory_order_relaxed);
  return DCUE_OK;
}

int dcue_debug_probes(void* buf) {
  dcue::g_probes.store(static_cast<dcue::ProbeRec*>(buf), std::memory_order_relaxed);
  return DCUE_OK;
}

int dcue_debug_probe_count(void) { return dcue::kNumProbes; }

const char* dcue_debug_probe_name(int32_t i) {
  return i >= 0 && i < dcue::kNumProbes ? dcue::kProbeNames[i] : nullptr;
}

int dcue_debug_poison(int32_t on) {
  dcue::g_poison.store(on != 0, std::memory_order_relaxed);
  return DCUE_OK;
}

int dcue_debug_fail_flags(uint32_t* flags_host) {
  if (!flags_host) return DCUE_ERR_INVALID;
  unsigned v = 0;
  DCUE_HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(dcue::g_user_fwd_fail), sizeof v));
  const unsigned zero = 0;
  DCUE_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dcue::g_user_fwd_fail), &zero, sizeof zero));
  *flags_host = v;
  return DCUE_OK;
}

int dcue_debug_raise_fail_flags(uint32_t bits) {
  unsigned v = 0;
  DCUE_HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(dcue::g_user_fwd_fail), sizeof v));
  v |= bits;
  DCUE_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dcue::g_user_fwd_fail), &v, sizeof v));
  return DCUE_OK;
}

}  // extern "C"
