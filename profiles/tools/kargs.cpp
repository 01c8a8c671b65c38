// Micro-benchmark: host issue cost vs kernel-argument size and event binding (scratch, not product).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t ck_e_ = (x); if (ck_e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(ck_e_)); return 1; } } while (0)

template <int NB> struct Args { float* p; long a[NB]; };

template <int NB>
__global__ void k_small(Args<NB> b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.a[NB - 1] == 12345) b.p[0] += 1.f;
}
__global__ void k_ptr(const Args<250>* b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b->a[249] == 12345) b->p[0] += 1.f;
}

template <int NB>
double run(hipStream_t m, hipEvent_t ev, float* buf, int n) {
  Args<NB> b = {};
  b.p = buf;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    if (ev)
      hipExtLaunchKernelGGL(k_small<NB>, dim3(64), dim3(256), 0, m, nullptr, ev, 0, b);
    else
      hipLaunchKernelGGL(k_small<NB>, dim3(64), dim3(256), 0, m, b);
  }
  auto t1 = std::chrono::steady_clock::now();
  hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 1 << 16));
  CK(hipMemset(buf, 0, 1 << 16));
  hipStream_t m;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
  const int N = 20000;
  for (int pass = 0; pass < 3; ++pass) {
    double a = run<1>(m, nullptr, buf, N), b = run<62>(m, nullptr, buf, N), c = run<250>(m, nullptr, buf, N);
    double d = run<62>(m, ev, buf, N), e = run<250>(m, ev, buf, N), f = run<1>(m, ev, buf, N);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_ptr, dim3(64), dim3(256), 0, m, (const Args<250>*)buf);
    auto t1 = std::chrono::steady_clock::now();
    hipDeviceSynchronize();
    double g = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    printf("pass %d us/launch: 16B %.2f, 512B %.2f, 2KB %.2f | bound event: 16B %.2f 512B %.2f 2KB %.2f | "
           "pointer arg %.2f\n", pass, a, b, c, f, d, e, g);
  }
  return 0;
}
