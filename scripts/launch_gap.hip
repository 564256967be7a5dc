// launch_gap.hip -- diagnostic: time between back-to-back dependent kernels on one
// stream on this part (the floor under a per-step launch), for grids shaped like the
// step kernel's.  hipcc --offload-arch=gfx950 -O3 scripts/launch_gap.hip -o scripts/bin/launch_gap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                          \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;  // never true: keeps the argument live
}

// One dword per workgroup, plain or write-through: a few bytes left dirty in L2.
__global__ void k_touch(int* p, int wt) {
  if (threadIdx.x == 0) {
    if (wt) __hip_atomic_store(p + blockIdx.x, (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else p[blockIdx.x] = (int)blockIdx.x;
  }
}

int main() {
  int* d = nullptr;
  CK(hipMalloc(&d, 1 << 24));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int N = 2000;
  const int grids[] = {1, 256, 4096, 8192, 65536};
  for (int g : grids) {
    for (int kind = 0; kind < 3; ++kind) {
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(g), dim3(64), 0, s, (int*)nullptr);
        else hipLaunchKernelGGL(k_touch, dim3(g), dim3(64), 0, s, d, kind == 2 ? 1 : 0);
      };
      for (int i = 0; i < 50; ++i) launch();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < N; ++i) launch();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      // one launch timed by events bound to its dispatch
      std::vector<float> one;
      for (int i = 0; i < 200; ++i) {
        if (kind == 0) hipExtLaunchKernelGGL(k_empty, dim3(g), dim3(64), 0, s, e0, e1, 0, (int*)nullptr);
        else hipExtLaunchKernelGGL(k_touch, dim3(g), dim3(64), 0, s, e0, e1, 0, d, kind == 2 ? 1 : 0);
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        one.push_back(t);
      }
      double avg = 0;
      for (float t : one) avg += t;
      avg /= one.size();
      std::printf("grid %6d %-9s  back-to-back %.2f us per launch   single kernel (dispatch events) %.2f us\n", g,
                  kind == 0 ? "empty" : kind == 1 ? "touch" : "touch_wt", ms * 1e3 / N, avg * 1e3);
    }
  }
  // graph of 100 dependent launches of the 8192-workgroup touch kernel
  {
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_touch, dim3(8192), dim3(64), 0, s, d, 0);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("graph of 100 x touch(8192): %.2f us per kernel\n", ms * 1e3 / 2000);
  }
  return 0;
}
