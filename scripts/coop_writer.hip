// coop_writer.hip -- diagnostic for VERDICT r05 item 4 (the 7-TB/s store shape): can the
// waves of a workgroup write their boards' observations TOGETHER, window by window, as each
// board's step finishes -- no barrier between the board work and the stores -- and does
// that stream faster than every wave writing its own board?
//
// Each wave "steps" one board: a VALU loop whose length varies by board (hash of b: 0.5x to
// 1.5x `iters`), standing in for the board work.  Then:
//   own    the wave writes its own board's 18 windows (the step kernels' shape today)
//   coop   the wave appends its board to the workgroup's LDS queue and joins the writers:
//          every wave of the workgroup takes the next (queued board, window) item from an
//          LDS counter and writes it, waiting (s_sleep) only when the next item's board is
//          not queued yet.  Few boards are in flight per CU, each written by many waves.
// 18,000 B per board (10x10), 128-B-aligned 1-KB windows, whole lines non-temporal, the two
// lines a board shares with its neighbours plain; boards of a workgroup are consecutive and
// workgroups spread over the XCDs as xcd_board spreads boards.  Contiguous allocation.
//   hipcc --offload-arch=gfx950 -O3 scripts/coop_writer.hip -o scripts/bin/coop_writer
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
constexpr int ROWB = 18000;
constexpr int KWIN = (ROWB / 16 + 7 + 63) / 64;  // windows per board (line-aligned start)

__device__ __forceinline__ int xcd_block(int i, int n) {
  const int x = i & 7, q = n / 8, r = n % 8;
  return x * q + (x < r ? x : r) + i / 8;
}

__device__ __forceinline__ void write_window(char* out, int b, int k, int lane) {
  const size_t start = (size_t)b * ROWB;
  const int n4 = ROWB / 16, mis = (int)((start >> 4) & 7);
  const int head = mis ? 8 - mis : 0, tail = ((n4 + mis) & ~7) - mis;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, ROWB, 0x00020000);
  const int i = lane - mis + 64 * k;
  const unsigned off = (unsigned)i * 16u;
  const bool shared = i < head || i >= tail;
  const u32x4 v = u32x4{(unsigned)b, (unsigned)i, 0u, 0u};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? 0x80000000u : off, 0, 2);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? off : 0x80000000u, 0, 0);
}

__device__ __forceinline__ float board_work(int b, int iters, int lane) {
  const unsigned h = (unsigned)b * 2654435761u;
  const int n = iters / 2 + (int)((unsigned long long)iters * (h >> 16) / 65536u);  // 0.5x .. 1.5x
  float acc = (float)lane;
  for (int i = 0; i < n; ++i) acc = acc * 1.0001f + 0.5f;
  return acc;
}

// COOP 0: each wave writes its own board; 1: the workgroup's waves write the queued boards
// together; 2: no stores (the board work alone)
template <int W, int COOP>
__global__ __launch_bounds__(64 * W) void k_step(char* out, int nb, int iters, float* sink) {
  __shared__ int q[W];
  __shared__ unsigned q_tail, next_item;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = xcd_block((int)blockIdx.x, nb / W);
  const int b = g * W + wv;
  if (COOP == 1) {
    if (threadIdx.x == 0) { q_tail = 0u; next_item = 0u; }
    if (lane == 0) q[wv] = -1;  // (an entry is written after the tail moves: -1 until then)
    __syncthreads();  // (zeroed once, before any board work)
  }
  const float acc = board_work(b, iters, lane);
  if (acc == -1.0f) sink[b] = acc;  // (never: keeps the loop)
  if (COOP == 2) return;  // the board work alone
  if (COOP == 0) {
    for (int k = 0; k < KWIN; ++k) write_window(out, b, k, lane);
    return;
  }
  if (lane == 0) {
    const unsigned p = __hip_atomic_fetch_add(&q_tail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&q[p], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  for (;;) {
    unsigned it = 0;
    if (lane == 0) it = __hip_atomic_fetch_add(&next_item, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    it = __builtin_amdgcn_readfirstlane(__shfl((int)it, 0));
    if (it >= (unsigned)(W * KWIN)) break;
    const unsigned qi = it / KWIN, k = it % KWIN;
    int bb = -1;
    for (;;) {  // the queued board at position qi (every board of the workgroup is queued eventually)
      bb = __hip_atomic_load(&q[qi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (__hip_atomic_load(&q_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > qi && bb >= 0) break;
      __builtin_amdgcn_s_sleep(2);
    }
    write_window(out, __builtin_amdgcn_readfirstlane(bb), (int)k, lane);
  }
}

int main(int argc, char** argv) {
  const int nb = 65536;
  const size_t bytesz = (size_t)nb * ROWB + 4096;
  char* buf = nullptr;
  float* sink = nullptr;
  CK(hipExtMallocWithFlags((void**)&buf, bytesz, hipDeviceMallocContiguous));
  CK(hipMemset(buf, 0, bytesz));
  CK(hipMalloc(&sink, nb * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 20 * 1e3;
  };
  const double bytes = (double)nb * ROWB;
  for (int iters : {0, 1000, 3000, 6000}) {
#define RUN(W)                                                                                                        \
  {                                                                                                                   \
    const double to = timed([&] { hipLaunchKernelGGL((k_step<W, 0>), dim3(nb / W), dim3(64 * W), 0, 0, buf, nb, iters, sink); }); \
    const double tc = timed([&] { hipLaunchKernelGGL((k_step<W, 1>), dim3(nb / W), dim3(64 * W), 0, 0, buf, nb, iters, sink); }); \
    std::printf("iters %5d  waves/wg %2d  own %.1f us (%.2f TB/s)  coop %.1f us (%.2f TB/s)\n", iters, W, to, bytes / to / 1e6, tc, \
                bytes / tc / 1e6);                                                                                    \
  }
    RUN(1) RUN(4) RUN(8) RUN(16)
  }
  // the board work alone (no stores): what the overlap could reach
  for (int iters : {1000, 3000, 6000}) {
    const double t = timed([&] { hipLaunchKernelGGL((k_step<8, 2>), dim3(nb / 8), dim3(512), 0, 0, buf, nb, iters, sink); });
    std::printf("iters %5d  board work alone (no stores, 8 waves/wg) %.1f us\n", iters, t);
  }
  // coverage: every window of every board written once by the coop writer
  CK(hipMemset(buf, 0, bytesz));
  hipLaunchKernelGGL((k_step<8, 1>), dim3(nb / 8), dim3(512), 0, 0, buf, nb, 1000, sink);
  CK(hipDeviceSynchronize());
  unsigned* h = (unsigned*)std::malloc(bytesz);
  CK(hipMemcpy(h, buf, (size_t)nb * ROWB, hipMemcpyDeviceToHost));
  long bad = 0;
  for (int b = 0; b < nb; ++b)
    for (int u = 0; u < ROWB / 16; u += 7) {
      const size_t w = ((size_t)b * ROWB + (size_t)u * 16) / 4;
      if (h[w] != (unsigned)b) ++bad;
    }
  std::printf("coverage: %ld bad units\n", bad);
  return bad != 0;
}
