// Check mode ("a HIP kernel bounds/NaN check mode"; the reference has none): probes a
// caller runs between training steps. Each one ORs its bit into a device flag word and never
// faults on the data it inspects, so a step's inputs can be validated before a kernel that would
// index with them runs, and its outputs (loss, parameters, gradients, the user table) after.
#include "dcue_internal.h"

namespace dcue {

// any element not finite (NaN or +-inf): exponent bits all ones
__global__ __launch_bounds__(256) void k_check_finite(const float* __restrict__ x, long n, int32_t* flags,
                                                      int32_t bit) {
  bool bad = false;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = ld4(x + 4 * i);
    const uint32_t e = 0x7f800000u;
    const uint32_t m = max(max(__float_as_uint(v.x) & e, __float_as_uint(v.y) & e),
                           max(__float_as_uint(v.z) & e, __float_as_uint(v.w) & e));
    bad |= m == e;
  }
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    bad |= (__float_as_uint(x[i]) & 0x7f800000u) == 0x7f800000u;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flags, bit);
}

// any id outside [0, limit)
template <typename T>
__global__ __launch_bounds__(256) void k_check_ids(const T* __restrict__ ids, long n, long limit, int32_t* flags,
                                                   int32_t bit) {
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long v = (long)ids[i];
    bad |= v < 0 || v >= limit;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flags, bit);
}

static unsigned check_blocks(long n) {
  const long b = (n / 4 + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

}  // namespace dcue

extern "C" {

int dcue_check_finite(const float* buf, int64_t n, int32_t* flags, int32_t bit, void* stream) {
  if (!flags || n < 0 || (n > 0 && !buf) || bit == 0) return DCUE_ERR_INVALID;
  if (n == 0) return DCUE_OK;
  DCUE_LAUNCH(dcue::k_check_finite, dim3(dcue::check_blocks(n)), dim3(256), 0, (hipStream_t)stream, buf,
              (long)n, flags, bit);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

int dcue_check_ids(const void* ids, int32_t id_bytes, int64_t n, int64_t limit, int32_t* flags, int32_t bit,
                   void* stream) {
  if (!flags || n < 0 || (n > 0 && !ids) || bit == 0 || (id_bytes != 4 && id_bytes != 8)) return DCUE_ERR_INVALID;
  if (n == 0) return DCUE_OK;
  const dim3 grid(dcue::check_blocks(4 * n));
  if (id_bytes == 4)
    DCUE_LAUNCH(dcue::k_check_ids<int32_t>, grid, dim3(256), 0, (hipStream_t)stream, (const int32_t*)ids, (long)n,
                (long)limit, flags, bit);
  else
    DCUE_LAUNCH(dcue::k_check_ids<int64_t>, grid, dim3(256), 0, (hipStream_t)stream, (const int64_t*)ids, (long)n,
                (long)limit, flags, bit);
  DCUE_LAUNCH_CHECK();
  return DCUE_OK;
}

}  // extern "C"
