// launch_ramp.hip -- diagnostic: how fast one-round grids of 64-thread workgroups get
// their waves started on this part, and what slows the ramp: static LDS per workgroup,
// the VGPR allocation, and work the already-started waves do (VALU, memory, sleep).
// Each wave stores s_memrealtime (100 MHz, chip-wide) at its start and end.  `wg <n>`
// lines: the same waves packed n per workgroup (k_ramp_wg).
//   hipcc --offload-arch=gfx950 -O3 scripts/launch_ramp.hip -o scripts/bin/launch_ramp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                           \
    }                                                                     \
  } while (0)

// WORK: 0 none, 1 VALU loop (~10 us), 2 memory (16 loads + 18 1-KB stores), 3 s_sleep (~10 us)
// PRIO: the wave raises its issue priority (s_setprio 3) until its start is stamped
template <int LDS, int WORK, int PRIO = 0>
__global__ __launch_bounds__(64) void k_ramp(uint64_t* t, float* buf, int iters) {
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  __shared__ float s[LDS > 0 ? LDS / 4 : 1];
  float acc = (float)threadIdx.x;
  if constexpr (LDS > 0) {
    s[threadIdx.x] = acc;
    __builtin_amdgcn_s_barrier();
    acc += s[(threadIdx.x + 1) & 63];
  }
  if constexpr (WORK == 1) {
    for (int i = 0; i < iters; ++i) acc = acc * 1.0001f + 0.5f;
  } else if constexpr (WORK == 2) {
    const float* in = buf + (size_t)blockIdx.x * 4096;
    float4 v[4];
    for (int k = 0; k < 4; ++k) v[k] = reinterpret_cast<const float4*>(in)[threadIdx.x + 64 * k];
    for (int k = 0; k < 4; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    float* out = buf + (size_t)8192 * 4096 + (size_t)blockIdx.x * 4608;
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int k = 0; k < 18; ++k)
      __builtin_nontemporal_store(f4{acc, acc, acc, acc}, reinterpret_cast<f4*>(out) + threadIdx.x + 64 * k);
  } else if constexpr (WORK == 3) {
    for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
  } else if constexpr (WORK == 4) {  // SALU chain
    uint32_t v = __builtin_amdgcn_readfirstlane((uint32_t)iters);
    for (int i = 0; i < iters; ++i) asm volatile("s_mul_i32 %0, %0, 3\n s_add_u32 %0, %0, 1" : "+s"(v));
    acc += (float)v;
  } else if constexpr (WORK == 5) {  // dependent LDS round trips
    __shared__ float q[64];
    q[threadIdx.x] = acc;
    for (int i = 0; i < iters; ++i) {
      acc = q[(threadIdx.x + (int)acc) & 63] + 1.0f;
      q[threadIdx.x] = acc;
    }
  } else if constexpr (WORK == 6) {  // VALU with a short sleep every 32 iterations
    for (int i = 0; i < iters; ++i) {
      acc = acc * 1.0001f + 0.5f;
      if ((i & 31) == 31) __builtin_amdgcn_s_sleep(1);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x] = t0;
    t[2 * blockIdx.x + 1] = t1;
  }
  if (acc == -1.0f) buf[0] = acc;  // keeps the work
}

// NW independent waves per workgroup (wave w of block i is wave i * NW + w of the grid)
template <int NW, int WORK>
__global__ __launch_bounds__(64 * NW) void k_ramp_wg(uint64_t* t, float* buf, int iters) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, w = blockIdx.x * NW + (threadIdx.x >> 6);
  float acc = (float)lane;
  if constexpr (WORK == 1) {
    for (int i = 0; i < iters; ++i) acc = acc * 1.0001f + 0.5f;
  } else if constexpr (WORK == 5) {
    __shared__ float q[64 * NW];
    float* qw = q + 64 * (threadIdx.x >> 6);
    qw[lane] = acc;
    for (int i = 0; i < iters; ++i) {
      acc = qw[(lane + (int)acc) & 63] + 1.0f;
      qw[lane] = acc;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    t[2 * w] = t0;
    t[2 * w + 1] = t1;
  }
  if (acc == -1.0f) buf[0] = acc;
}

static int report(const char* name, int waves, uint64_t* dt) {
  std::vector<uint64_t> h(2 * (size_t)waves);
  CK(hipMemcpy(h.data(), dt, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t s0 = ~0ull, s1 = 0, e1 = 0;
  std::vector<double> life;
  for (int i = 0; i < waves; ++i) {
    s0 = std::min(s0, h[2 * i]);
    s1 = std::max(s1, h[2 * i]);
    e1 = std::max(e1, h[2 * i + 1]);
    life.push_back((h[2 * i + 1] - h[2 * i]) / 100.0);
  }
  std::sort(life.begin(), life.end());
  std::printf("%-22s waves %5d  start ramp %6.2f us  first start -> last end %6.2f us  wave life p50 %6.2f us\n", name, waves,
              (s1 - s0) / 100.0, (e1 - s0) / 100.0, life[life.size() / 2]);
  return 0;
}

template <int NW, int WORK>
int run_wg(const char* what, int waves, int iters, uint64_t* dt, float* buf) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((k_ramp_wg<NW, WORK>), dim3(waves / NW), dim3(64 * NW), 0, 0, dt, buf, iters);
    CK(hipDeviceSynchronize());
  }
  char name[64];
  std::snprintf(name, sizeof name, "wg %d %s", NW, what);
  return report(name, waves, dt);
}

template <int LDS, int WORK, int PRIO = 0>
int run(const char* name, int grid, int iters, uint64_t* dt, float* buf) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((k_ramp<LDS, WORK, PRIO>), dim3(grid), dim3(64), 0, 0, dt, buf, iters);
    CK(hipDeviceSynchronize());
  }
  std::vector<uint64_t> h(2 * (size_t)grid);
  CK(hipMemcpy(h.data(), dt, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t s0 = ~0ull, s1 = 0, e1 = 0;
  std::vector<double> life;
  for (int i = 0; i < grid; ++i) {
    s0 = std::min(s0, h[2 * i]);
    s1 = std::max(s1, h[2 * i]);
    e1 = std::max(e1, h[2 * i + 1]);
    life.push_back((h[2 * i + 1] - h[2 * i]) / 100.0);
  }
  std::sort(life.begin(), life.end());
  std::printf("%-22s grid %5d  start ramp %6.2f us  first start -> last end %6.2f us  wave life p50 %6.2f us\n", name, grid,
              (s1 - s0) / 100.0, (e1 - s0) / 100.0, life[life.size() / 2]);
  return 0;
}

int main(int argc, char**) {
  uint64_t* dt = nullptr;
  float* buf = nullptr;
  CK(hipMalloc(&dt, 2 * 65536 * 8));
  CK(hipMalloc(&buf, (size_t)8192 * (4096 + 4608) * 4));
  CK(hipMemset(buf, 0, (size_t)8192 * (4096 + 4608) * 4));
  if (argc > 1) {  // launch_ramp wg: one-round grids of 1-, 2-, 4- and 8-wave workgroups
    for (int waves : {8192, 4096}) {
      if (run_wg<1, 0>("empty", waves, 0, dt, buf) || run_wg<2, 0>("empty", waves, 0, dt, buf) ||
          run_wg<4, 0>("empty", waves, 0, dt, buf) || run_wg<8, 0>("empty", waves, 0, dt, buf))
        return 1;
      for (int iters : {500, 5000, 20000}) {
        char what[32];
        std::snprintf(what, sizeof what, "valu %d", iters);
        if (run_wg<1, 1>(what, waves, iters, dt, buf) || run_wg<2, 1>(what, waves, iters, dt, buf) ||
            run_wg<4, 1>(what, waves, iters, dt, buf) || run_wg<8, 1>(what, waves, iters, dt, buf))
          return 1;
      }
      if (run_wg<1, 5>("lds-chain 200", waves, 200, dt, buf) || run_wg<4, 5>("lds-chain 200", waves, 200, dt, buf))
        return 1;
    }
    return 0;
  }
  for (int grid : {8192}) {
    if (run<0, 1>("valu-short", grid, 500, dt, buf)) return 1;
    if (run<0, 6>("valu-short+sleep/32", grid, 500, dt, buf)) return 1;
    if (run<0, 4>("salu", grid, 2000, dt, buf)) return 1;
    if (run<0, 5>("lds-chain", grid, 200, dt, buf)) return 1;
  }
  for (int grid : {4096, 8192}) {
    if (run<0, 0>("empty", grid, 0, dt, buf)) return 1;
    if (run<4968, 0>("lds4968", grid, 0, dt, buf)) return 1;
    if (run<0, 1>("valu", grid, 20000, dt, buf)) return 1;
    if (run<0, 1, 1>("valu+startprio", grid, 20000, dt, buf)) return 1;
    if (run<0, 1>("valu-short", grid, 500, dt, buf)) return 1;
    if (run<0, 1, 1>("valu-short+startprio", grid, 500, dt, buf)) return 1;
    if (run<4968, 1>("lds4968+valu", grid, 20000, dt, buf)) return 1;
    if (run<0, 2>("memory", grid, 0, dt, buf)) return 1;
    if (run<4968, 2>("lds4968+memory", grid, 0, dt, buf)) return 1;
    if (run<0, 3>("sleep", grid, 200, dt, buf)) return 1;
  }
  return 0;
}
