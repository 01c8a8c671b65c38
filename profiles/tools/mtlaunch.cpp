// Micro-benchmark: host cost of kernel launches issued by one thread vs two threads (two streams).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x) do { hipError_t ck_e_ = (x); if (ck_e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(ck_e_)); return 1; } } while (0)

struct Big { float* p; long a[60]; };  // ~500 B of kernel arguments, like the library's RowsArgs

__global__ void k_small(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.a[3] == 12345) b.p[0] += 1.f;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 4096));
  hipStream_t m, s;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Big b = {};
  b.p = buf;
  const int N = 20000;
  auto issue = [&](hipStream_t st, int n) {
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, b);
  };
  for (int pass = 0; pass < 3; ++pass) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    issue(m, N);
    issue(s, N);
    auto t1 = std::chrono::steady_clock::now();
    CK(hipDeviceSynchronize());
    auto t2 = std::chrono::steady_clock::now();
    std::thread th([&] { issue(s, N); });
    issue(m, N);
    th.join();
    auto t3 = std::chrono::steady_clock::now();
    CK(hipDeviceSynchronize());
    // small-argument launches for comparison
    auto t4 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2 * N; ++i) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, m, Big{});
    auto t5 = std::chrono::steady_clock::now();
    CK(hipDeviceSynchronize());
    // event record + wait pairs
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
    auto t6 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) {
      hipEventRecord(ev, m);
      hipStreamWaitEvent(s, ev, 0);
    }
    auto t7 = std::chrono::steady_clock::now();
    CK(hipDeviceSynchronize());
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    printf("pass %d: one thread %.2f us/launch, two threads %.2f us/launch (wall / launches), "
           "same stream %.2f us/launch, record+wait pair %.2f us\n", pass, us(t0, t1) / (2 * N),
           us(t2, t3) / (2 * N), us(t4, t5) / (2 * N), us(t6, t7) / N);
  }
  return 0;
}
