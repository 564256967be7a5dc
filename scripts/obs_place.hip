// obs_place.hip -- diagnostic: does the observation stream go faster when the boards one
// CU writes at a time are NEIGHBOURS in memory?  The step's store shape (one 64-lane wave
// per board, 18,000 B per board in 128-B-aligned 1-KB windows, whole lines non-temporal and
// the two lines a board shares with its neighbours plain) with three placements:
//   xcd   block i -> xcd_board(i): the product's map; the ~32 boards a CU holds at once lie
//         ~B/256 boards apart
//   cu    each wave takes the next board of ITS CU's contiguous chunk of B/256 boards (a
//         per-CU ticket; a CU whose chunk is used up takes tickets from the other chunks)
//   cuil  the same tickets, interleaved: ticket n of CU c -> board n * NCU + c (the atomic's
//         cost without the contiguity)
// The CU of a wave is read from HW_REG_HW_ID / HW_REG_XCC_ID and numbered by a one-time
// registration pass.  Ticket counters are zeroed by hipMemsetAsync before each launch; the
// memset alone is timed and subtracted.
//   hipcc --offload-arch=gfx950 -O3 scripts/obs_place.hip -o scripts/bin/obs_place
#include <hip/hip_runtime.h>

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
constexpr int NKEY = 4096, MAXCU = 512;

__device__ __forceinline__ int xcd_board(int i, int B) {
  const int x = i & 7, q = B / 8, r = B % 8;
  return x * q + (x < r ? x : r) + i / 8;
}

__device__ __forceinline__ int cu_key() {
  const unsigned hw = __builtin_amdgcn_s_getreg(0xf804);   // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg(0xf814);  // HW_REG_XCC_ID
  return (int)(((xcc & 15u) << 8) | ((hw >> 8) & 0xffu));  // xcc, se, sh, cu
}

// One pass: every CU that runs a wave gets a compact number (registration order).
__global__ __launch_bounds__(64) void k_register(int* key2cu, int* ncu) {
  if (threadIdx.x) return;
  const int k = cu_key();
  if (atomicCAS(&key2cu[k], -1, -2) == -1) key2cu[k] = atomicAdd(ncu, 1);
}

__device__ __forceinline__ void write_board(char* out, int b, int rowb, int lane, int WHOLE, int SHARED) {
  const size_t start = (size_t)b * rowb;
  const int n4 = rowb / 16, mis = (int)((start >> 4) & 7);
  const int head = mis ? 8 - mis : 0, tail = ((n4 + mis) & ~7) - mis;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, rowb, 0x00020000);
  const int K = (n4 + mis + 63) / 64;
  for (int k = 0; k < K; ++k) {
    const int i = lane - mis + 64 * k;
    const unsigned off = (unsigned)i * 16u;
    const bool shared = i < head || i >= tail;
    const u32x4 v = u32x4{(unsigned)b, (unsigned)i, 0u, 0u};
    if (WHOLE == 2) {
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? 0x80000000u : off, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? off : 0x80000000u, 0, 0);
    } else {  // every line write-through (the small batches' policy)
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
    }
  }
}

// MODE 0 xcd map, 1 per-CU contiguous chunks, 2 per-CU tickets interleaved
template <int MODE, int WHOLE>
__global__ __launch_bounds__(64) void k_obs(char* out, int nb, int rowb, const int* key2cu, int ncu, int* ctr) {
  const int lane = threadIdx.x;
  int b;
  if (MODE == 0) {
    b = xcd_board((int)blockIdx.x, nb);
  } else {
    int c = key2cu[cu_key()];
    if (c < 0 || c >= ncu) c = 0;  // (a CU the registration pass missed)
    const int per = (nb + ncu - 1) / ncu;
    int got = -1;
    if (lane == 0) {
      for (int j = 0; j < ncu && got < 0; ++j) {  // own chunk first, then the others
        const int cc = (c + j) % ncu;
        const int n = atomicAdd(&ctr[cc], 1);
        const int bb = MODE == 1 ? cc * per + n : n * ncu + cc;
        if (n < per && bb < nb) got = bb;
      }
    }
    b = __builtin_amdgcn_readfirstlane(__shfl(got, 0));
    if (b < 0) return;
  }
  write_board(out, b, rowb, lane, WHOLE, 0);
}

int main() {
  const int rowb = 18000;
  const size_t maxb = (size_t)65536 * rowb + 4096;
  char* buf = nullptr;
  CK(hipExtMallocWithFlags((void**)&buf, maxb, hipDeviceMallocContiguous));
  CK(hipMemset(buf, 0, maxb));
  int *key2cu, *ncu_d, *ctr;
  CK(hipMalloc(&key2cu, NKEY * 4));
  CK(hipMalloc(&ncu_d, 4));
  CK(hipMalloc(&ctr, MAXCU * 4));
  CK(hipMemset(key2cu, 0xff, NKEY * 4));
  CK(hipMemset(ncu_d, 0, 4));
  for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_register, dim3(65536), dim3(64), 0, 0, key2cu, ncu_d);
  CK(hipDeviceSynchronize());
  int ncu = 0;
  CK(hipMemcpy(&ncu, ncu_d, 4, hipMemcpyDeviceToHost));
  std::printf("CUs registered: %d\n", ncu);
  if (ncu < 1 || ncu > MAXCU) return 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch, bool memset) {
    for (int i = 0; i < 3; ++i) {
      if (memset) CK(hipMemsetAsync(ctr, 0, MAXCU * 4, 0));
      launch();
    }
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) {
      if (memset) CK(hipMemsetAsync(ctr, 0, MAXCU * 4, 0));
      launch();
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 20 * 1e3;  // us per launch
  };
  const double ms_us = timed([] {}, true);
  std::printf("memset alone %.2f us per launch\n", ms_us);
  for (int nb : {65536, 32768, 8192}) {
    const double bytes = (double)nb * rowb;
    const double t0 = timed([&] { hipLaunchKernelGGL((k_obs<0, 2>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr); }, false);
    const double t1 = timed([&] { hipLaunchKernelGGL((k_obs<1, 2>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr); }, true) - ms_us;
    const double t2 = timed([&] { hipLaunchKernelGGL((k_obs<2, 2>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr); }, true) - ms_us;
    std::printf("%5d boards nt+plain: xcd %.1f us %.2f TB/s | cu-contiguous %.1f us %.2f TB/s | cu-interleaved %.1f us %.2f TB/s\n", nb,
                t0, bytes / t0 / 1e6, t1, bytes / t1 / 1e6, t2, bytes / t2 / 1e6);
    if (nb == 8192) {
      const double w0 = timed([&] { hipLaunchKernelGGL((k_obs<0, 16>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr); }, false);
      const double w1 = timed([&] { hipLaunchKernelGGL((k_obs<1, 16>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr); }, true) - ms_us;
      std::printf("%5d boards all sc1: xcd %.1f us %.2f TB/s | cu-contiguous %.1f us %.2f TB/s\n", nb, w0, bytes / w0 / 1e6, w1,
                  bytes / w1 / 1e6);
    }
  }
  // coverage check of the ticket placement: every board written exactly once
  {
    const int nb = 65536;
    CK(hipMemset(buf, 0, (size_t)nb * rowb));
    CK(hipMemset(ctr, 0, MAXCU * 4));
    hipLaunchKernelGGL((k_obs<1, 2>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb, key2cu, ncu, ctr);
    CK(hipDeviceSynchronize());
    int bad = 0;
    for (int b = 0; b < nb && bad < 5; b += 97) {
      unsigned w[4];
      const size_t off = (size_t)b * rowb + 128;
      CK(hipMemcpy(w, buf + (off & ~(size_t)15), 16, hipMemcpyDeviceToHost));
      if (w[0] != (unsigned)b) { std::printf("board %d: word %u\n", b, w[0]); ++bad; }
    }
    std::printf("coverage check: %s\n", bad ? "FAILED" : "ok");
  }
  return 0;
}
