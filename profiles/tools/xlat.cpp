// Micro-benchmark (diagnostic, not product): latency of the first loads of a kernel that follows a
// producer kernel on the same stream, as the in-batch conv chain has it -- a word the producer
// updated with device-scope atomics (BN accumulators), a line it wrote with plain stores (the
// layer output), a buffer nobody wrote this step (parameters), and a re-read of a line just loaded.
// Thread 0 of each workgroup times one dependent load at a time with the 100 MHz s_memrealtime.
//   hipcc --offload-arch=gfx950 -O3 -o xlat profiles/tools/xlat.cpp && ./xlat
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Args {  // a RowsArgs-sized argument block
  unsigned long long* acc;
  float* y;
  const float* param;
  float* far_buf;
  unsigned long long* out;
  const void* pad[36];
  int salt;
};

__global__ void k_prod(unsigned long long* acc, float* y, int n) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  if (threadIdx.x < 512) atomicAdd(acc + threadIdx.x, (unsigned long long)(blockIdx.x + 1));
  for (int i = t; i < n; i += gridDim.x * blockDim.x) y[i] = (float)i;
}

__device__ __forceinline__ unsigned long long stamp() {
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::: "memory");
  return __builtin_amdgcn_s_memrealtime();  // 100 MHz
}

__global__ void k_cons(Args a) {
  if (threadIdx.x != 0) return;
  unsigned long long t[8];
  float sink = 0.f;
  t[0] = stamp();
  sink += (float)__builtin_amdgcn_readfirstlane(a.salt);  // kernarg word (usually already loaded)
  t[1] = stamp();
  sink += (float)*(a.acc + (blockIdx.x * 2) % 512);  // atomically updated
  t[2] = stamp();
  sink += *(a.y + blockIdx.x * 1024);    // plain-stored by the producer
  t[3] = stamp();
  sink += *(a.param + blockIdx.x * 64);  // untouched this step (same pages each run)
  t[4] = stamp();
  sink += *(a.y + blockIdx.x * 1024);    // re-read (L2/L1 hit)
  t[5] = stamp();
  sink += *(a.far_buf + (size_t)blockIdx.x * (4u << 20) / 4);  // a new 4 MB-strided page per WG
  t[6] = stamp();
  unsigned long long* o = a.out + blockIdx.x * 8;
  for (int i = 0; i < 6; ++i) o[i] = t[i + 1] - t[i];
  o[6] = (unsigned long long)sink;
}

// Instruction fetch: a 16 KB run of straight-line code executed twice by each wave (a rolled loop
// of two passes). The first pass fetches it cold, the second from the instruction cache.
__global__ void k_icache(unsigned long long* out) {
  unsigned long long t[3];
  t[0] = stamp();
#pragma nounroll
  for (int pass = 0; pass < 2; ++pass) {
    asm volatile(".rept 4096\n s_nop 0\n .endr" ::: "memory");
    t[pass + 1] = stamp();
  }
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = t[1] - t[0];
    out[blockIdx.x * 2 + 1] = t[2] - t[1];
  }
}

int main() {
  const int nwg = 128, n = 1 << 20;
  unsigned long long *acc, *out;
  float *y, *param, *far_buf;
  CK(hipMalloc(&acc, 512 * 8));
  CK(hipMalloc(&out, nwg * 8 * 8));
  CK(hipMalloc(&y, (size_t)nwg * 1024 * 4 + n * 4));
  CK(hipMalloc(&param, nwg * 64 * 4));
  CK(hipMalloc(&far_buf, (size_t)nwg * (4u << 20)));
  CK(hipMemset(acc, 0, 512 * 8));
  CK(hipMemset(param, 0, nwg * 64 * 4));
  CK(hipMemset(far_buf, 0, (size_t)nwg * (4u << 20)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  Args a = {};
  a.acc = acc; a.y = y; a.param = param; a.far_buf = far_buf; a.out = out;
  const char* names[6] = {"kernarg", "atomic-updated", "plain-stored", "param (idle)", "re-read", "new page"};
  const double clk_mhz = 100.0;
  std::vector<unsigned long long> h(nwg * 8);
  for (int variant = 0; variant < 2; ++variant) {
    std::vector<std::vector<double>> lat(6);
    for (int it = 0; it < 50; ++it) {
      if (variant == 0) hipLaunchKernelGGL(k_prod, dim3(176), dim3(512), 0, s, acc, y, n);
      a.salt = it;
      hipLaunchKernelGGL(k_cons, dim3(nwg), dim3(64), 0, s, a);
      CK(hipStreamSynchronize(s));
      if (it < 5) continue;
      CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
      for (int b = 0; b < nwg; ++b)
        for (int i = 0; i < 6; ++i) lat[i].push_back(h[b * 8 + i] / clk_mhz);
    }
    printf("%s, us per dependent load, median / p90 over WGs x runs:\n",
           variant == 0 ? "after a producer kernel" : "no producer (kernel alone)");
    for (int i = 0; i < 6; ++i) {
      auto& v = lat[i];
      std::sort(v.begin(), v.end());
      printf("  %-16s %6.2f / %6.2f\n", names[i], v[v.size() / 2], v[v.size() * 9 / 10]);
    }
  }
  {
    std::vector<double> c0, c1;
    for (int it = 0; it < 20; ++it) {
      hipLaunchKernelGGL(k_prod, dim3(176), dim3(512), 0, s, acc, y, n);
      hipLaunchKernelGGL(k_icache, dim3(256), dim3(64), 0, s, out);
      CK(hipStreamSynchronize(s));
      std::vector<unsigned long long> hh(512);
      CK(hipMemcpy(hh.data(), out, 512 * 8, hipMemcpyDeviceToHost));
      for (int b = 0; b < 256; ++b) {
        c0.push_back(hh[b * 2] / clk_mhz);
        c1.push_back(hh[b * 2 + 1] / clk_mhz);
      }
    }
    std::sort(c0.begin(), c0.end());
    std::sort(c1.begin(), c1.end());
    printf("16 KB straight-line code (4096 single-issue instructions), us median / p90:\n");
    printf("  first pass (cold) %6.2f / %6.2f   second pass (cached) %6.2f / %6.2f\n", c0[c0.size() / 2],
           c0[c0.size() * 9 / 10], c1[c1.size() / 2], c1[c1.size() * 9 / 10]);
  }
  return 0;
}
