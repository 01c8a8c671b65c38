// Micro-benchmark: cost of cross-stream ordering on MI355X / ROCm 7.2 (scratch, not product).
// A chain of K small kernels on stream `m`; at fork points a side stream `s` runs a kernel that
// depends on the chain, and at join points the chain depends on the side stream.
//   mode 0: no cross-stream ordering (baseline)
//   mode 1: hipEvent: the fork kernel binds an event (hipExtLaunchKernel stop event), s waits it;
//           join: s records an event, m waits it
//   mode 2: device flags + hipStreamWaitValue32: the fork kernel's last workgroup writes an epoch
//           flag; s waits on it with hipStreamWaitValue32; join: the side kernel writes a flag, m
//           waits with hipStreamWaitValue32
//   mode 3: as mode 2, but the flags are written by hipStreamWriteValue32 after the kernel (no
//           kernel change)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t ck_e_ = (x); if (ck_e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(ck_e_)); return 1; } } while (0)

__global__ void k_work(float* buf, int iters, unsigned* ctr, unsigned* flag, unsigned epoch) {
  float x = buf[blockIdx.x * blockDim.x + threadIdx.x];
  for (int i = 0; i < iters; ++i) x = fmaf(x, 0.999f, 0.001f);
  buf[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned old = atomicAdd(ctr, 1u);
      if (old == gridDim.x - 1) {
        *ctr = 0;
        __threadfence_system();
        __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

int main() {
  const int K = 20, NB = 64, ITER = 2000, REP = 200;
  const int forks[] = {4, 9, 14}, joins[] = {7, 12, 17};
  float* buf;
  unsigned *ctr, *flag;
  CK(hipMalloc(&buf, sizeof(float) * 1024 * 256 * 4));
  CK(hipMalloc(&ctr, 4096));
  {
    hipError_t e = hipExtMallocWithFlags((void**)&flag, 4096, hipMallocSignalMemory);
    printf("signal memory 4096 B: %s\n", hipGetErrorString(e));
    if (e != hipSuccess) CK(hipMalloc(&flag, 4096));
  }
  int wv = 0;
  CK(hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("CanUseStreamWaitValue %d\n", wv);
  CK(hipMemset(buf, 0, sizeof(float) * 1024 * 256 * 4));
  CK(hipMemset(ctr, 0, 4096));
  CK(hipMemset(flag, 0, 4096));
  hipStream_t m, s;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(64);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int mode = 0; mode < 4; ++mode) {
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipDeviceSynchronize());
      unsigned epoch = 1000 * (mode * 2 + pass + 1);
      auto h0 = std::chrono::steady_clock::now();
      CK(hipEventRecord(t0, m));
      for (int r = 0; r < REP; ++r) {
        int evi = 0;
        for (int k = 0; k < K; ++k) {
          bool fork = false, join = false;
          for (int f : forks) fork |= f == k;
          for (int j : joins) join |= j == k;
          if (join && mode == 1) CK(hipStreamWaitEvent(m, ev[32 + (k % 8)], 0));
          if (join && (mode == 2 || mode == 3))
            CK(hipStreamWaitValue32(m, flag + 64 + 16 * (k % 8), epoch + r, hipStreamWaitValueGte, 0xffffffffu));
          if (fork && mode == 1) {
            hipExtLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, m, nullptr, ev[k % 8], 0, buf, ITER,
                                  (unsigned*)nullptr, (unsigned*)nullptr, 0u);
          } else if (fork && mode == 2) {
            hipLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, m, buf, ITER, ctr + 16 * (k % 8),
                               flag + 16 * (k % 8), epoch + r);
          } else {
            hipLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, m, buf, ITER, (unsigned*)nullptr,
                               (unsigned*)nullptr, 0u);
            if (fork && mode == 3) CK(hipStreamWriteValue32(m, flag + 16 * (k % 8), epoch + r, 0));
          }
          if (fork) {  // side work depending on kernel k; the chain joins it 3 kernels later
            if (mode == 1) CK(hipStreamWaitEvent(s, ev[k % 8], 0));
            if (mode == 2 || mode == 3)
              CK(hipStreamWaitValue32(s, flag + 16 * (k % 8), epoch + r, hipStreamWaitValueGte, 0xffffffffu));
            const int jk = k + 3;
            if (mode == 2)
              hipLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, s, buf + 256 * NB, ITER, ctr + 64 + 16 * (jk % 8),
                                 flag + 64 + 16 * (jk % 8), epoch + r);
            else
              hipLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, s, buf + 256 * NB, ITER, (unsigned*)nullptr,
                                 (unsigned*)nullptr, 0u);
            if (mode == 1) CK(hipEventRecord(ev[32 + (jk % 8)], s));
            if (mode == 3) CK(hipStreamWriteValue32(s, flag + 64 + 16 * (jk % 8), epoch + r, 0));
          }
          evi++;
        }
      }
      CK(hipEventRecord(t1, m));
      auto h1 = std::chrono::steady_clock::now();
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      const double host_us = std::chrono::duration<double, std::micro>(h1 - h0).count() / REP;
      printf("mode %d pass %d: %.2f us/iteration GPU (wall of m), host issue %.2f us/iteration\n", mode, pass,
             ms * 1000.0 / REP, host_us);
    }
  }
  // one kernel alone: its duration (the chain's per-kernel floor)
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(t0, m));
  for (int r = 0; r < REP * K; ++r)
    hipLaunchKernelGGL(k_work, dim3(NB), dim3(256), 0, m, buf, ITER, (unsigned*)nullptr, (unsigned*)nullptr, 0u);
  CK(hipEventRecord(t1, m));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, t0, t1));
  printf("plain chain: %.2f us per kernel\n", ms * 1000.0 / (REP * K));
  return 0;
}
