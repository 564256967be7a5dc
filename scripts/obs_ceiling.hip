// obs_ceiling.hip -- diagnostic: the observation stream of the step kernel with nothing
// else in the kernel.  One 64-lane workgroup per board, 18,000 B per board (a 10x10
// observation) back to back, 128-B-aligned 1-KB windows, the store policy of
// write_obs_lines (td_step.hip): whole lines non-temporal and the two lines a board shares
// with its neighbours plain (edge_wt = 2), or every line write-through (the small batches'
// obs_wt); block i steps board xcd_board(i) (td_kernels.h) or board i.  The buffer comes
// from hipMalloc or hipExtMallocWithFlags(hipDeviceMallocContiguous) (td_alloc_device).
// Rates are bytes / the mean of 20 launches (hipEvents) after 3 warm-up launches.
//   hipcc --offload-arch=gfx950 -O3 scripts/obs_ceiling.hip -o scripts/bin/obs_ceiling
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_board(int i, int B) {
  const int x = i & 7, q = B / 8, r = B % 8;
  return x * q + (x < r ? x : r) + i / 8;
}

// WHOLE / SHARED: buffer-store aux bits (0 plain, 2 non-temporal, 16 sc1)
template <int WHOLE, int SHARED, bool XCD>
__global__ __launch_bounds__(64) void obs(char* out, int nb, int rowb) {
  const int b = XCD ? xcd_board((int)blockIdx.x, nb) : (int)blockIdx.x, lane = threadIdx.x;
  const size_t start = (size_t)b * rowb;
  const int n4 = rowb / 16, mis = (int)((start >> 4) & 7);
  const int head = mis ? 8 - mis : 0, tail = ((n4 + mis) & ~7) - mis;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, rowb, 0x00020000);
  const int K = (n4 + mis + 63) / 64;
  for (int k = 0; k < K; ++k) {
    const int i = lane - mis + 64 * k;
    const unsigned off = (unsigned)i * 16u;  // i < 0: out of range, dropped
    const bool shared = i < head || i >= tail;
    const u32x4 v = u32x4{(unsigned)b, (unsigned)i, 0u, 0u};
    if (WHOLE == SHARED) {
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, WHOLE);
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? 0x80000000u : off, 0, WHOLE);
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? off : 0x80000000u, 0, SHARED);
    }
  }
}

template <class F>
static double timed(F launch, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  const int n = 20;
  for (int i = 0; i < n; ++i) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return bytes / (ms / n * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  // argv[1] = 20 or 30: 16,384 boards of a 20x20 (72,000 B) or 30x30 (162,000 B) observation
  if (argc > 1) {
    const int L = std::atoi(argv[1]), nb = 16384, rowb = 45 * L * L * 4;
    const size_t bytesz = (size_t)nb * rowb + 4096;
    for (int contig = 0; contig < 2; ++contig) {
      char* buf = nullptr;
      if (contig) CK(hipExtMallocWithFlags((void**)&buf, bytesz, hipDeviceMallocContiguous));
      else CK(hipMalloc(&buf, bytesz));
      CK(hipMemset(buf, 0, bytesz));
      const double bytes = (double)nb * rowb;
      const double px = timed([&] { hipLaunchKernelGGL((obs<2, 0, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      const double ax = timed([&] { hipLaunchKernelGGL((obs<0, 0, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      std::printf("%s %dx%d %5d boards (%7.1f MB) | nt + plain shared (xcd map) %.2f | all plain %.2f TB/s | %.1f us at nt+plain\n",
                  contig ? "contiguous" : "hipMalloc ", L, L, nb, bytes / 1e6, px, ax, bytes / (px * 1e12) * 1e6);
      CK(hipFree(buf));
    }
    return 0;
  }
  const int rowb = 18000;
  const size_t maxb = (size_t)65536 * rowb + 4096;
  for (int contig = 0; contig < 2; ++contig) {
    char* buf = nullptr;
    if (contig) CK(hipExtMallocWithFlags((void**)&buf, maxb, hipDeviceMallocContiguous));
    else CK(hipMalloc(&buf, maxb));
    CK(hipMemset(buf, 0, maxb));
    for (int nb : {65536, 32768, 8192, 4096}) {
      const double bytes = (double)nb * rowb;
      const double px = timed([&] { hipLaunchKernelGGL((obs<2, 0, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      const double p0 = timed([&] { hipLaunchKernelGGL((obs<2, 0, false>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      const double wx = timed([&] { hipLaunchKernelGGL((obs<16, 16, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      const double ax = timed([&] { hipLaunchKernelGGL((obs<0, 0, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes);
      std::printf("%s %5d boards (%7.1f MB) | nt + plain shared: xcd map %.2f, board i %.2f | all sc1 (xcd) %.2f | all plain (xcd) %.2f TB/s"
                  " | %.1f us at nt+plain/xcd\n",
                  contig ? "contiguous" : "hipMalloc ", nb, bytes / 1e6, px, p0, wx, ax, bytes / (px * 1e12) * 1e6);
    }
    CK(hipFree(buf));
  }
  return 0;
}
