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

// Store shapes (argv[1] == "shapes"): W bytes per lane per instruction (4 / 8 / 16), AUX
// the buffer-store aux bits of the whole lines (the two shared lines plain), BPW boards per workgroup stepped one after the
// other (a block of BPW consecutive boards, blocks spread over the XCDs as xcd_board
// spreads boards), NW waves per workgroup splitting each board's row by instruction.
// SPLIT 0: the NW waves take a board's instructions in turn; 1: each a contiguous share of
// them; 2: each wave its own board (NW boards per workgroup, BPW must be 1).
// THR >= 0: s_waitcnt vmcnt(THR) after every store instruction (stores in flight per wave)
template <int W, int AUX, int BPW, int NW, int SPLIT = 0, int THR = -1>
__global__ __launch_bounds__(64 * NW) void obs_shape(char* out, int nb, int rowb) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int per = SPLIT == 2 ? NW : BPW;
  const int blk = xcd_board((int)blockIdx.x, nb / per);
  for (int j = 0; j < BPW; ++j) {
    const int b = SPLIT == 2 ? blk * NW + wv : blk * BPW + j;
    const size_t start = (size_t)b * rowb;
    const int mis = (int)(start & 127);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, rowb, 0x00020000);
    const int K = (rowb + mis + 64 * W - 1) / (64 * W);
    const int q = (K + NW - 1) / NW;
    const int k0 = SPLIT == 0 ? wv : SPLIT == 1 ? wv * q : 0;
    const int k1 = SPLIT == 1 ? (k0 + q < K ? k0 + q : K) : K;
    const int dk = SPLIT == 0 ? NW : 1;
    for (int k = k0; k < k1; k += dk) {
      const int o = k * 64 * W + lane * W - mis;
      const unsigned off = o < 0 ? 0x80000000u : (unsigned)o;
      // the two lines the board shares with its neighbours: plain stores (as the product)
      const int line = (o + mis) >> 7;
      const bool shared = (mis && line == 0) || (((rowb + mis) & 127) && line == ((rowb + mis) >> 7));
      const unsigned ow = shared ? 0x80000000u : off, os = shared ? off : 0x80000000u;
      if constexpr (W == 16) {
        const u32x4 v{(unsigned)b, (unsigned)o, 0u, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, ow, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, os, 0, 0);
      } else if constexpr (W == 8) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 v{(unsigned)b, (unsigned)o};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, ow, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, os, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)o, rs, ow, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)o, rs, os, 0, 0);
      }
      if constexpr (THR == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (THR == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      if constexpr (THR == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if constexpr (THR == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      if constexpr (THR == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
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
  if (argc > 1 && argv[1][0] == 's') {
    const int nb = 65536, rowb = 18000;
    const size_t bytesz = (size_t)nb * rowb + 4096;
    char* buf = nullptr;
    CK(hipExtMallocWithFlags((void**)&buf, bytesz, hipDeviceMallocContiguous));
    CK(hipMemset(buf, 0, bytesz));
    const double bytes = (double)nb * rowb;
#define SHAPE(W, AUX, BPW, NW, SPLIT, LDSB, THR)                                                              \
  std::printf("shape W=%2d aux=%2d boards/wg=%2d waves/wg=%2d split=%d lds=%5d vmcnt=%2d  %.2f TB/s\n", W, AUX, BPW, NW, SPLIT, \
              LDSB, THR,                                                                                        \
              timed([&] { hipLaunchKernelGGL((obs_shape<W, AUX, BPW, NW, SPLIT, THR>), dim3(nb / (SPLIT == 2 ? NW : BPW)),   \
                                             dim3(64 * NW), LDSB, 0, buf, nb, rowb); }, bytes))
    std::printf("reference: nt + plain shared (xcd map) %.2f TB/s\n",
                timed([&] { hipLaunchKernelGGL((obs<2, 0, true>), dim3(nb), dim3(64), 0, 0, buf, nb, rowb); }, bytes));
    // waves per board (split 0 / 1), waves per workgroup each with its own board (split 2),
    // fewer resident workgroups (dynamic LDS), 8-byte lanes
    SHAPE(16, 2, 1, 1, 0, 0, -1); SHAPE(16, 2, 1, 2, 0, 0, -1); SHAPE(16, 2, 1, 4, 0, 0, -1); SHAPE(16, 2, 1, 8, 0, 0, -1);
    SHAPE(16, 2, 1, 16, 0, 0, -1); SHAPE(16, 2, 1, 4, 1, 0, -1); SHAPE(16, 2, 1, 8, 1, 0, -1); SHAPE(16, 2, 1, 16, 1, 0, -1);
    SHAPE(16, 2, 1, 4, 2, 0, -1); SHAPE(16, 2, 1, 16, 2, 0, -1);
    SHAPE(16, 2, 1, 1, 0, 20480, -1); SHAPE(16, 2, 1, 1, 0, 40960, -1); SHAPE(16, 2, 1, 4, 0, 40960, -1);
    SHAPE(8, 2, 1, 8, 0, 0, -1);
    // one wave per board, stores in flight per wave capped
    SHAPE(16, 2, 1, 1, 0, 0, 0); SHAPE(16, 2, 1, 1, 0, 0, 1); SHAPE(16, 2, 1, 1, 0, 0, 2); SHAPE(16, 2, 1, 1, 0, 0, 4);
    SHAPE(16, 2, 1, 1, 0, 0, 8); SHAPE(16, 2, 1, 2, 0, 0, 1); SHAPE(16, 2, 1, 4, 0, 0, 0);
    CK(hipFree(buf));
    return 0;
  }
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
