// Store cache-policy probe for the observation stream (diagnostic, not shipped).
// Every variant writes B boards x 18,000 B in the step kernel's shape: one wave per
// board, 128-B-aligned 1-KB windows of the batch stream (scripts/membench.hip
// flat_nt_shift), with a different cache-policy field on global_store_dwordx4.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BOARD_F4 = 1125;  // 18,000 B

template <int P>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
  if constexpr (P == 0) *p = v;
  else if constexpr (P == 1) __builtin_nontemporal_store(v, p);
  else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0" :: "v"(p), "v"(v) : "memory");
  else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" :: "v"(p), "v"(v) : "memory");
  else if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(p), "v"(v) : "memory");
  else if constexpr (P == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(p), "v"(v) : "memory");
  else if constexpr (P == 6) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}

template <int P>
__global__ __launch_bounds__(64) void shift(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  for (long g = a0 + lane; g < hi; g += 64)
    if (g >= lo) st<P>(out + g, f32x4{(float)g, 1.f, 2.f, 3.f});
}

// 2 KB per wave-iteration: each lane writes two consecutive 16-B units
template <int P>
__global__ __launch_bounds__(64) void shift2(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  for (long g = a0 + 2 * lane; g < hi; g += 128) {
    if (g >= lo) st<P>(out + g, f32x4{(float)g, 1.f, 2.f, 3.f});
    if (g + 1 >= lo && g + 1 < hi) st<P>(out + g + 1, f32x4{(float)g, 1.f, 2.f, 3.f});
  }
}

// whole-line-only stream (no partial lines: boards padded to 18,048 B), nt
template <int P>
__global__ __launch_bounds__(64) void padded(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * 1128;
  for (int i = lane; i < 1128; i += 64) st<P>(o + i, f32x4{(float)i, 1.f, 2.f, 3.f});
}

// whole lines only: the lines a board shares with its neighbours are skipped
// (diagnostic lower bound), optionally written to a side buffer of one 128-B line per
// boundary for a fix-up launch
template <bool SCRATCH>
__global__ __launch_bounds__(64) void whole(f32x4* out, f32x4* scr, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  const long f0 = (lo + 7) & ~7l, f1 = hi & ~7l;  // whole lines [f0, f1)
  for (long g = a0 + lane; g < hi; g += 64) {
    const f32x4 v = f32x4{(float)g, 1.f, 2.f, 3.f};
    if (g >= f0 && g < f1) __builtin_nontemporal_store(v, out + g);
    else if (SCRATCH && g >= lo) scr[g < f0 ? (size_t)b * 8 + (g & 7) : (size_t)(b + 1) * 8 + (g & 7)] = v;
  }
}
// whole lines with policy P, the two shared lines with policy Q
template <int P, int Q>
__global__ __launch_bounds__(64) void split(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  const long f0 = (lo + 7) & ~7l, f1 = hi & ~7l;
  for (long g = a0 + lane; g < hi; g += 64) {
    const f32x4 v = f32x4{(float)g, 1.f, 2.f, 3.f};
    if (g >= f0 && g < f1) st<P>(out + g, v);
    else if (g >= lo) st<Q>(out + g, v);
  }
}
// boundary line of board b (between b - 1 and b), composed from the side buffer
__global__ __launch_bounds__(256) void fixup(f32x4* out, const f32x4* scr, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x, b = i >> 3, k = i & 7;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4;
  if ((lo & 7) == 0) return;
  __builtin_nontemporal_store(scr[i], out + (lo & ~7l) + k);
}

// The 2p-middle-multi memory skeleton: per board read 19,200 B of int64 flags
// (non-temporal 16-B loads, K per lane in flight), then write the 72,000-B (45, 20, 20)
// observation in 128-B-aligned 1-KB windows (shared lines sc1).  LDS bytes per
// workgroup as the step kernel (occupancy), or none.
constexpr int OBS2 = 4500, ACT2 = 1200;  // 16-B units per board
template <int K, int LDS>
__global__ __launch_bounds__(64) void skel2p(f32x4* out, const f32x4* act, int B, int rd) {
  __shared__ float pad[LDS / 4 + 1];
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;
  if (rd) {
    const f32x4* a = act + (size_t)b * ACT2;
    for (int base = 0; base < ACT2; base += 64 * K) {
      f32x4 v[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = base + 64 * k + lane;
        v[k] = e < ACT2 ? __builtin_nontemporal_load(a + e) : f32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int k = 0; k < K; ++k) acc += v[k].x + v[k].w;
    }
  }
  if (LDS) { pad[lane] = acc; __syncthreads(); acc = pad[(lane + 1) & 63]; }
  const long lo = (long)b * OBS2, hi = lo + OBS2, a0 = lo & ~7l;
  const long f0 = (lo + 7) & ~7l, f1 = hi & ~7l;
  for (long g = a0 + lane; g < hi; g += 64) {
    const f32x4 v = f32x4{acc, 1.f, 2.f, (float)g};
    if (g >= f0 && g < f1) st<1>(out + g, v);
    else if (g >= lo) st<6>(out + g, v);
  }
}

// 30x30 observation stream (162,000 B per board, one wave per board, 1-KB windows,
// shared lines sc1) at the step kernel's LDS footprint (13 workgroups per CU) or none
constexpr int OBS3 = 10125;  // 16-B units per board
template <int LDS>
__global__ __launch_bounds__(64) void large(f32x4* out, int B) {
  __shared__ float pad[LDS / 4 + 1];
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;
  if (LDS) { pad[lane] = (float)b; __syncthreads(); acc = pad[(lane + 1) & 63]; }
  const long lo = (long)b * OBS3, hi = lo + OBS3, a0 = lo & ~7l;
  const long f0 = (lo + 7) & ~7l, f1 = hi & ~7l;
  for (long g = a0 + lane; g < hi; g += 64) {
    const f32x4 v = f32x4{acc, 1.f, 2.f, (float)g};
    if (g >= f0 && g < f1) st<1>(out + g, v);
    else if (g >= lo) st<6>(out + g, v);
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 65536;
  const size_t bytes = (size_t)B * BOARD_F4 * 16;
  f32x4* out;
  CK(hipMalloc(&out, (size_t)B * 1128 * 16 + 4096));
  f32x4* scr;
  CK(hipMalloc(&scr, ((size_t)B + 1) * 8 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / reps;
    printf("%-14s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  const dim3 g(B), t(64);
  for (int rep = 0; rep < 2; ++rep) {
    run("plain", [&] { hipLaunchKernelGGL(shift<0>, g, t, 0, 0, out, B); });
    if (rep == 0) {
      // correctness of the fix-up composition: whole+fix must equal the shift stream
      hipLaunchKernelGGL(shift<0>, g, t, 0, 0, out, B);
      float* ref = (float*)malloc(bytes);
      float* got = (float*)malloc(bytes);
      CK(hipMemcpy(ref, out, bytes, hipMemcpyDeviceToHost));
      CK(hipMemset(out, 0, bytes));
      hipLaunchKernelGGL(whole<true>, g, t, 0, 0, out, scr, B);
      hipLaunchKernelGGL(fixup, dim3((B * 8 + 255) / 256), dim3(256), 0, 0, out, scr, B);
      CK(hipMemcpy(got, out, bytes, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < bytes / 4; ++i) bad += ref[i] != got[i];
      printf("fix-up composition mismatches: %zu\n", bad);
      free(ref); free(got);
    }
    run("nt", [&] { hipLaunchKernelGGL(shift<1>, g, t, 0, 0, out, B); });
    run("sc0", [&] { hipLaunchKernelGGL(shift<2>, g, t, 0, 0, out, B); });
    run("sc0_nt", [&] { hipLaunchKernelGGL(shift<3>, g, t, 0, 0, out, B); });
    run("sc1_nt", [&] { hipLaunchKernelGGL(shift<4>, g, t, 0, 0, out, B); });
    run("sc0_sc1_nt", [&] { hipLaunchKernelGGL(shift<5>, g, t, 0, 0, out, B); });
    run("sc1", [&] { hipLaunchKernelGGL(shift<6>, g, t, 0, 0, out, B); });
    run("nt_2k", [&] { hipLaunchKernelGGL(shift2<1>, g, t, 0, 0, out, B); });
    run("sc0_nt_2k", [&] { hipLaunchKernelGGL(shift2<3>, g, t, 0, 0, out, B); });
    run("pad_nt", [&] { hipLaunchKernelGGL(padded<1>, g, t, 0, 0, out, B); });
    run("whole_only", [&] { hipLaunchKernelGGL(whole<false>, g, t, 0, 0, out, scr, B); });
    run("whole+scr", [&] { hipLaunchKernelGGL(whole<true>, g, t, 0, 0, out, scr, B); });
    run("whole+fix", [&] { hipLaunchKernelGGL(whole<true>, g, t, 0, 0, out, scr, B);
                            hipLaunchKernelGGL(fixup, dim3((B * 8 + 255) / 256), dim3(256), 0, 0, out, scr, B); });
    run("split_nt_plain", [&] { hipLaunchKernelGGL((split<1, 0>), g, t, 0, 0, out, B); });
    run("split_nt_sc1", [&] { hipLaunchKernelGGL((split<1, 6>), g, t, 0, 0, out, B); });
    run("split_nt_sc0", [&] { hipLaunchKernelGGL((split<1, 2>), g, t, 0, 0, out, B); });
    run("split_nt_s01nt", [&] { hipLaunchKernelGGL((split<1, 5>), g, t, 0, 0, out, B); });
    run("pad_sc0_nt", [&] { hipLaunchKernelGGL(padded<3>, g, t, 0, 0, out, B); });
  }
  CK(hipFree(out));
  {
    const int B2 = 16384;
    f32x4 *o2, *a2;
    CK(hipMalloc(&o2, (size_t)B2 * OBS2 * 16));
    CK(hipMalloc(&a2, (size_t)B2 * ACT2 * 16 * 4));  // 4 action batches, cycled (> MALL)
    CK(hipMemset(a2, 0, (size_t)B2 * ACT2 * 16 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run2 = [&](const char* name, auto launch) {
      for (int i = 0; i < 4; ++i) launch(i);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      const int reps = 20;
      for (int i = 0; i < reps; ++i) launch(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / reps;
      printf("%-14s %8.1f us  %6.2f TB/s (read+write)\n", name, us,
             (double)B2 * (OBS2 + ACT2) * 16 / (us * 1e-6) / 1e12);
    };
    const dim3 g2(B2), t2(64);
    for (int rep = 0; rep < 2; ++rep) {
      run2("2p_write_only", [&](int i) { hipLaunchKernelGGL((skel2p<8, 7760>), g2, t2, 0, 0, o2, a2 + (size_t)(i & 3) * B2 * ACT2, B2, 0); });
      run2("2p_k8_lds", [&](int i) { hipLaunchKernelGGL((skel2p<8, 7760>), g2, t2, 0, 0, o2, a2 + (size_t)(i & 3) * B2 * ACT2, B2, 1); });
      run2("2p_k19_lds", [&](int i) { hipLaunchKernelGGL((skel2p<19, 7760>), g2, t2, 0, 0, o2, a2 + (size_t)(i & 3) * B2 * ACT2, B2, 1); });
      run2("2p_k8_nolds", [&](int i) { hipLaunchKernelGGL((skel2p<8, 0>), g2, t2, 0, 0, o2, a2 + (size_t)(i & 3) * B2 * ACT2, B2, 1); });
      run2("2p_k19_nolds", [&](int i) { hipLaunchKernelGGL((skel2p<19, 0>), g2, t2, 0, 0, o2, a2 + (size_t)(i & 3) * B2 * ACT2, B2, 1); });
    }
  }
  {
    const int B3 = 16384;
    f32x4* o3;
    CK(hipMalloc(&o3, (size_t)B3 * OBS3 * 16 + 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run3 = [&](const char* name, auto launch) {
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      const int reps = 10;
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / reps;
      printf("%-14s %8.1f us  %6.2f TB/s\n", name, us, (double)B3 * OBS3 * 16 / (us * 1e-6) / 1e12);
    };
    for (int rep = 0; rep < 2; ++rep) {
      run3("30x30_lds12k", [&] { hipLaunchKernelGGL((large<12272>), dim3(B3), dim3(64), 0, 0, o3, B3); });
      run3("30x30_lds6k", [&] { hipLaunchKernelGGL((large<6000>), dim3(B3), dim3(64), 0, 0, o3, B3); });
      run3("30x30_nolds", [&] { hipLaunchKernelGGL((large<0>), dim3(B3), dim3(64), 0, 0, o3, B3); });
    }
    CK(hipFree(o3));
  }
  return 0;
}
