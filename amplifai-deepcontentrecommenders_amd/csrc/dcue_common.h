// Shared device/host helpers for libdcue_hip (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <climits>

#include "dcue.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace dcue {
// records the failing HIP call for dcue_last_error() (timer.hip)
void set_last_error(const char* expr, hipError_t e, const char* file, int line);
}  // namespace dcue

#define DCUE_HIP_CHECK(expr)                                      \
  do {                                                            \
    const hipError_t _dcue_e = (expr);                            \
    if (_dcue_e != hipSuccess) {                                  \
      dcue::set_last_error(#expr, _dcue_e, __FILE__, __LINE__);   \
      return DCUE_ERR_HIP;                                        \
    }                                                             \
  } while (0)
#define DCUE_LAUNCH_CHECK() DCUE_HIP_CHECK(hipGetLastError())

namespace dcue {
// Events bound to kernel launches (hipExtLaunchKernel) rather than recorded after them. An
// event-record packet between two dependent kernels idles the stream for ≈3 µs on MI355X / ROCm 7.2
// (≈5.5 µs when another stream waits on it); an event bound to the kernel's own dispatch costs
// ≈0.05 µs (measured, scratch-free: DESIGN.md §6). While `stop` is set every launch on this thread
// binds it (the last binding is the one a wait sees); `start` binds to the next launch only.
struct LaunchTag {
  hipEvent_t start = nullptr, stop = nullptr;
  int launches = 0;     // launches that bound `stop`
  bool missed = false;  // a nested scope's launches bound another event: `stop` must be recorded
};
LaunchTag& launch_tag();
// process-wide launch counter (dcue_launch_count)
void count_launch();
}  // namespace dcue

// Every kernel launch of the library goes through here (see LaunchTag).
#define DCUE_LAUNCH(kern, grid, block, shm, stream, ...)                                          \
  do {                                                                                            \
    ::dcue::LaunchTag& dcue_tag_ = ::dcue::launch_tag();                                          \
    ::dcue::count_launch();                                                                       \
    if (dcue_tag_.stop) {                                                                         \
      hipExtLaunchKernelGGL(kern, grid, block, shm, stream, dcue_tag_.start, dcue_tag_.stop, 0,   \
                            __VA_ARGS__);                                                         \
      dcue_tag_.start = nullptr;                                                                  \
      ++dcue_tag_.launches;                                                                       \
    } else {                                                                                      \
      hipLaunchKernelGGL(kern, grid, block, shm, stream, __VA_ARGS__);                            \
    }                                                                                             \
  } while (0)

// DCUE_KTRACE diagnostic builds (profiles/tools/build_ktrace.sh): thread 0 of each workgroup stores phase
// timestamps of selected kernels (slots 0-5 shader clock, 6-7 the 100 MHz wall clock) into
// dcue_ktrace_buf[kernel][block] (tail.hip), read back with dcue_ktrace_read. Compiled out otherwise.
constexpr int kKtraceKernels = 16, kKtraceBlocks = 512;
#ifdef DCUE_KTRACE
// one buffer per translation unit (no relocatable device code): each traced .hip file exports its
// own reader, dcue_ktrace_read_<file> (DCUE_KTRACE_READER)
static __device__ unsigned long long dcue_ktrace_buf[kKtraceKernels][kKtraceBlocks][8];
#define DCUE_KTRACE_READER(name)                                                           \
  extern "C" int dcue_ktrace_read_##name(void* host, size_t bytes) {                       \
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dcue_ktrace_buf), bytes) == hipSuccess ? 0 : 3; \
  }
#define DCUE_KT(kid, slot)                                                                          \
  do {                                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < kKtraceBlocks) dcue_ktrace_buf[kid][blockIdx.x][slot] = clock64(); \
  } while (0)
#define DCUE_KTW(kid, slot)                                                                              \
  do {                                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < kKtraceBlocks) dcue_ktrace_buf[kid][blockIdx.x][slot] = wall_clock64(); \
  } while (0)
#else
#define DCUE_KTRACE_READER(name)
#define DCUE_KT(kid, slot) \
  do {                     \
  } while (0)
#define DCUE_KTW(kid, slot) \
  do {                      \
  } while (0)
#endif

namespace dcue {

constexpr int kMels = DCUE_N_MELS;     // 128, truedcuemel1dbn.py:24
constexpr int kFrames = DCUE_N_FRAMES; // 131, datasets/dcuedataset.py:235
constexpr int kXp = kFrames + 5;        // zero-padded xhat0 rows per item: every conv-1 tap row exists
constexpr int kWave = 64;

// Tower variant (dcue_dims.tower): BatchNorm present, time-pooled skips into the fc
__host__ __device__ inline bool tower_has_bn(const dcue_dims* d) {
  return d->tower == DCUE_TOWER_BN || d->tower == DCUE_TOWER_RESBN || d->tower == DCUE_TOWER_TEXT;
}
// the mixed audio + text item tower (BASELINE config 4, text.hip)
__host__ __device__ inline bool tower_text(const dcue_dims* d) { return d->tower == DCUE_TOWER_TEXT; }
__host__ __device__ inline bool tower_res(const dcue_dims* d) {
  return d->tower == DCUE_TOWER_RES || d->tower == DCUE_TOWER_RESBN;
}
// Storage widths. The reference accepts any conv_hidden / feature_dim (dcue/dcue.py:39-47; its
// trainer's default is feature_dim = 100, nn/dcue.py:44). The kernels run at the width rounded up to
// 32, 64, 128 or 256 channels (their MFMA tiles and slab layouts), and the extra channels are
// zero-padded in every parameter that has them: zero weights, bias, BN gamma and beta give those
// channels exactly zero activations, features and gradients, so Adam keeps them zero for good and
// the real channels compute what the unpadded model does. The reference-shaped parameters are
// strided views of the padded segments (dcue_storage_dims).
__host__ __device__ inline int storage_width(int v) { return v <= 32 ? 32 : v <= 64 ? 64 : v <= 128 ? 128 : 256; }
__host__ __device__ inline int st_hidden(const dcue_dims* d) { return storage_width(d->conv_hidden); }
__host__ __device__ inline int st_feature(const dcue_dims* d) { return storage_width(d->feature_dim); }
// fc input width: d, or 4H + d with the four time-pooled block outputs (truedcuemel1dres.py:63-64).
// The time-pooled blocks keep the reference's H columns each (the fc weight is then a view of its
// padded [d_s][4H + d_s] segment); only the block-5 part is padded.
// The text tower's fc input is [s ; bn5(y5)]: the text features' text_dim columns (unpadded, as the
// res towers' pooled blocks) before the d_s audio columns.
__host__ __device__ inline int fc_in(const dcue_dims* d) {
  return tower_res(d) ? 4 * d->conv_hidden + st_feature(d)
       : tower_text(d) ? d->text_dim + st_feature(d) : st_feature(d);
}
// columns of the fc input before bn5(y5): the res towers' pooled blocks or the text features
__host__ __device__ inline int fc_off5(const dcue_dims* d) {
  return tower_res(d) ? 4 * d->conv_hidden : tower_text(d) ? d->text_dim : 0;
}
// text branch storage widths: channels C_s (64, 128 or 256: the forward's 64-channel column tiles)
// and the word width rounded up to the 32-channel MFMA k-step (the split-f16 weight pack's K)
__host__ __device__ inline int st_text(const dcue_dims* d) {
  return !tower_text(d) ? 0 : d->text_dim <= 64 ? 64 : storage_width(d->text_dim);
}
__host__ __device__ inline int st_word(const dcue_dims* d) {
  return !tower_text(d) ? 0 : (d->word_dim + 31) / 32 * 32;
}

// Per-layer geometry of the default item tower (truedcuemel1dbn.py:25-61).
//   conv positions Lconv = Lin + 2*pad - ks + 1, pooled Lp = floor(Lconv / pool); only the
//   R = Lp*pool conv rows that land in a pool window are computed (the reference drops the rest).
struct LayerGeom {
  int ks, pad, pool, lin, lp;
};
__host__ __device__ constexpr LayerGeom layer_geom(int l) {
  return l == 1 ? LayerGeom{4, 2, 4, 131, 33}
       : l == 2 ? LayerGeom{4, 2, 4, 33, 8}
       : l == 3 ? LayerGeom{4, 2, 4, 8, 2}
       : l == 4 ? LayerGeom{2, 1, 2, 2, 1}
                : LayerGeom{1, 0, 1, 1, 1};
}

// v_mfma_f32_16x16x4_f32: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15],
// D lane l, reg r = D[4*(l>>4)+r][l&15]. Exact f32 products, k-ordered f32 accumulation.
// Critical-path kernels raise their waves' issue priority: the off-path work that shares the CUs
// with them (the user table's rolling Adam flush, side-stream weight gradients, next-step draws)
// then takes the issue slots they leave, instead of stretching the step's chain.
__device__ __forceinline__ void critical_path_priority() { __builtin_amdgcn_s_setprio(2); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// XCD-aware block order (guide T1): blocks with equal id % 8 share an XCD (and its L2), so the
// logical index L gives each such group a contiguous range -- consecutive L then share an L2.
// Bijective for any nb. A placement guess only: a wrong one is slower, never wrong.
__device__ __forceinline__ int xcd_swizzle(int b, int nb) {
  const int x = b & 7, q = nb >> 3, r = nb & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Value ranges for the split-f16 forwards (conv.hip): per channel, the maximum of x and of -x as
// ORDERED keys (a float's bits with the sign folded so unsigned order is float order), so producers
// can merge them with integer atomicMax; a cleared word (0) is below every key and means "no value".
// One layer's range is [2][kRngC] words.
constexpr int kRngC = 256;
__device__ __forceinline__ unsigned ord_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_value(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// A cross-stream order kept on the device. A plan's producer on a side
// stream is followed there by k_signal, which stores a value into one of the plan's signal words
// (agent-scope atomic; the producer kernel's end released its data); the consumer kernel on the
// caller's stream, issued with no stream wait, polls the word at its start until it reaches the value
// (relaxed agent-scope loads, one lane), then takes an agent-scope acquire (this CU's L1 invalidated)
// before any load of the produced data. A HIP cross-queue event wait costs the waiting queue a
// barrier packet of 5-10 us even when its event completed long before; this costs one L2 round trip
// when the producer is done. Values grow by one per issue (wrap-safe compare). A wait that gives up
// (never expected: the producer is issued right after) sets bit 1 of the device fail word.
struct DevWait {
  const unsigned* flag;  // null: no wait
  unsigned val;
  unsigned* fail;
};
__device__ __forceinline__ void dev_wait(const DevWait& w) {
  if (!w.flag) return;
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while ((int)(__hip_atomic_load(w.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - w.val) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 21)) {
        if (w.fail) atomicOr(w.fail, 2u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// The producer side inside the producer kernel itself (no k_signal launch): every workgroup, once
// all its stores are done, releases them at agent scope and adds 1 to the signal word; the consumer
// waits for the word to reach the count of workgroups issued so far (the host adds each launch's grid
// size to its issue counter). All threads of the workgroup must call it (a barrier inside).
__device__ __forceinline__ void dev_signal_wg(unsigned* sig) {
  if (!sig) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// An order only: the kernel reads nothing the producer wrote, but later kernels on its stream must
// start after the producer (their own start-of-kernel acquire then sees its data). One lane polls at
// the end of the kernel's work; no barrier, no acquire.
__device__ __forceinline__ void dev_wait_order(const DevWait& w) {
  if (!w.flag || threadIdx.x != 0) return;
  unsigned spins = 0;
  while ((int)(__hip_atomic_load(w.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - w.val) < 0) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 21)) {
      if (w.fail) atomicOr(w.fail, 2u);
      break;
    }
  }
}

// bump allocator over a caller-owned workspace (host side)
struct Arena {
  char* base;
  size_t cap, used;
  template <typename T>
  T* take(size_t n) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + n * sizeof(T);
    // base == nullptr: the returned "pointer" is the byte offset (sizing / layout queries)
    return reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(base) + off);
  }
};

}  // namespace dcue
