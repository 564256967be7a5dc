// Write-bandwidth probe for the observation store pattern (diagnostic, not shipped).
// Each variant writes B boards x 18,000 B (the 10x10 obs) and reports TB/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int Q = 25, NCH = 45, BOARD_F4 = NCH * Q;  // 1125 float4 per board

// (a) the step kernel's pattern: lanes 0-49 write channel pairs, 23 stores per board
__global__ __launch_bounds__(64) void pairs(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B || g >= 2) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = 0; i < 23; ++i) {
    const int ch = 2 * i + g;
    if (ch < NCH) o[ch * Q + q] = f32x4{(float)ch, 1.f, 2.f, 3.f};
  }
}

// (b) flattened: all 64 lanes, consecutive float4 (18 stores per board)
__global__ __launch_bounds__(64) void flat(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < BOARD_F4; i += 64) o[i] = f32x4{(float)i, 1.f, 2.f, 3.f};
}

// (c) flattened with non-temporal stores
__global__ __launch_bounds__(64) void flat_nt(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < BOARD_F4; i += 64) __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, o + i);
}

// (d) pairs pattern with non-temporal stores
__global__ __launch_bounds__(64) void pairs_nt(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B || g >= 2) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = 0; i < 23; ++i) {
    const int ch = 2 * i + g;
    if (ch < NCH) __builtin_nontemporal_store(f32x4{(float)ch, 1.f, 2.f, 3.f}, o + ch * Q + q);
  }
}

// (e) grid-stride streaming write of the same bytes, 256-thread blocks
__global__ __launch_bounds__(256) void stream(f32x4* out, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    out[i] = f32x4{(float)i, 1.f, 2.f, 3.f};
}

// (f) pairs pattern + per-board dependent latency (a global load round trip first)
__global__ __launch_bounds__(64) void pairs_lat(f32x4* out, const int* in, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B) return;
  const int v = in[(size_t)b * 64 + lane];
  if (g >= 2) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = 0; i < 23; ++i) {
    const int ch = 2 * i + g;
    if (ch < NCH) o[ch * Q + q] = f32x4{(float)v, 1.f, 2.f, 3.f};
  }
}

// (g) the step's whole memory pattern without its compute: read a 3 KB state
// record, write the 18 KB observation, write 384 B of state back
__global__ __launch_bounds__(64) void mixed(f32x4* out, f32x4* st, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B) return;
  f32x4* sb = st + (size_t)b * 192;
  const f32x4 r0 = sb[lane], r1 = sb[64 + lane], r2 = sb[128 + lane];
  const float v = r0.x + r1.y + r2.z;
  f32x4* o = out + (size_t)b * BOARD_F4;
  if (g < 2)
    for (int i = 0; i < 23; ++i) {
      const int ch = 2 * i + g;
      if (ch < NCH) o[ch * Q + q] = f32x4{v, 1.f, 2.f, (float)ch};
    }
  if (lane < 24) sb[lane] = r0 + r1;
}

// (h) same, with the state write-back before the observation
__global__ __launch_bounds__(64) void mixed_ro(f32x4* out, f32x4* st, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* sb = st + (size_t)b * 192;
  const f32x4 r0 = sb[lane], r1 = sb[64 + lane], r2 = sb[128 + lane];
  const float v = r0.x + r1.y + r2.z;
  if (lane < 24) sb[lane] = r0 + r1;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < BOARD_F4; i += 64) o[i] = f32x4{v, 1.f, 2.f, (float)i};
}

// (i) mixed with R x 1 KB of state reads, optional LDS footprint (occupancy) and
// SPIN dependent VALU ops between the read and the observation writes
template <int R, int LDS, int SPIN>
__global__ __launch_bounds__(64) void mixed_t(f32x4* out, f32x4* st, int B) {
  __shared__ float pad[LDS / 4 + 1];
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B) return;
  f32x4* sb = st + (size_t)b * 192;
  float v = 0.f;
  f32x4 r0 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < R; ++k) { const f32x4 t = sb[64 * k + lane]; v += t.x; r0 += t; }
  if (LDS) { pad[lane] = v; v += pad[(lane + 1) & 63]; }
#pragma unroll 1
  for (int k = 0; k < SPIN; ++k) v = v * 1.0001f + 0.5f;
  f32x4* o = out + (size_t)b * BOARD_F4;
  if (g < 2)
    for (int i = 0; i < 23; ++i) {
      const int ch = 2 * i + g;
      if (ch < NCH) o[ch * Q + q] = f32x4{v, 1.f, 2.f, (float)ch};
    }
  if (lane < 24) sb[lane] = r0;
}


// (j) 256-thread workgroups, one wave per board (4 boards per workgroup), nt stores
__global__ __launch_bounds__(256) void flat4_nt(f32x4* out, int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < BOARD_F4; i += 64) __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, o + i);
}

// (k) persistent waves: grid-stride over boards, nt stores
__global__ __launch_bounds__(64) void persist_nt(f32x4* out, int B) {
  const int lane = threadIdx.x;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    f32x4* o = out + (size_t)b * BOARD_F4;
    for (int i = lane; i < BOARD_F4; i += 64) __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, o + i);
  }
}

// (l) stream with nt stores
__global__ __launch_bounds__(256) void stream_nt(f32x4* out, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, out + i);
}

// (m) one wave per board, boards padded to 128-B aligned starts (18,048 B stride)
constexpr int BOARD_F4_PAD = 1128;
__global__ __launch_bounds__(64) void flat_nt_al(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4_PAD;
  for (int i = lane; i < BOARD_F4; i += 64) __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, o + i);
}

// (n) one wave per TWO boards (36,000 contiguous bytes), nt
__global__ __launch_bounds__(64) void flat2_nt(f32x4* out, int B) {
  const int b = blockIdx.x * 2, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < 2 * BOARD_F4; i += 64) __builtin_nontemporal_store(f32x4{(float)i, 1.f, 2.f, 3.f}, o + i);
}

// (o) flat, plain stores, 256-thread blocks 4 boards
__global__ __launch_bounds__(256) void flat4(f32x4* out, int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  f32x4* o = out + (size_t)b * BOARD_F4;
  for (int i = lane; i < BOARD_F4; i += 64) o[i] = f32x4{(float)i, 1.f, 2.f, 3.f};
}

// (p) one wave per board, nt stores in 128-B-aligned 1-KB windows of the batch's
// stream: only the two lines a board shares with its neighbours are partial
__global__ __launch_bounds__(64) void flat_nt_shift(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  for (long g = a0 + lane; g < hi; g += 64)
    if (g >= lo) __builtin_nontemporal_store(f32x4{(float)g, 1.f, 2.f, 3.f}, out + g);
}

// (q) pairs pattern, nt, boards at 128-B-aligned starts
__global__ __launch_bounds__(64) void pairs_nt_al(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B || g >= 2) return;
  f32x4* o = out + (size_t)b * BOARD_F4_PAD;
  for (int i = 0; i < 23; ++i) {
    const int ch = 2 * i + g;
    if (ch < NCH) __builtin_nontemporal_store(f32x4{(float)ch, 1.f, 2.f, 3.f}, o + ch * Q + q);
  }
}

// (r) pairs pattern, plain, boards at 128-B-aligned starts
__global__ __launch_bounds__(64) void pairs_al(f32x4* out, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B || g >= 2) return;
  f32x4* o = out + (size_t)b * BOARD_F4_PAD;
  for (int i = 0; i < 23; ++i) {
    const int ch = 2 * i + g;
    if (ch < NCH) o[ch * Q + q] = f32x4{(float)ch, 1.f, 2.f, 3.f};
  }
}

// (s) = (p) with the step's state traffic: 3 KB read first, 384 B written back
__global__ __launch_bounds__(64) void mixed_shift(f32x4* out, f32x4* st, int B) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  f32x4* sb = st + (size_t)b * 192;
  const f32x4 r0 = sb[lane], r1 = sb[64 + lane], r2 = sb[128 + lane];
  const float v = r0.x + r1.y + r2.z;
  const long lo = (long)b * BOARD_F4, hi = lo + BOARD_F4, a0 = lo & ~7l;
  for (long g = a0 + lane; g < hi; g += 64)
    if (g >= lo) __builtin_nontemporal_store(f32x4{v, 1.f, 2.f, (float)g}, out + g);
  if (lane < 24) sb[lane] = r0 + r1;
}

// (t) = mixed (pairs, plain) but nt
__global__ __launch_bounds__(64) void mixed_nt(f32x4* out, f32x4* st, int B) {
  const int b = blockIdx.x, lane = threadIdx.x, q = lane % Q, g = lane / Q;
  if (b >= B) return;
  f32x4* sb = st + (size_t)b * 192;
  const f32x4 r0 = sb[lane], r1 = sb[64 + lane], r2 = sb[128 + lane];
  const float v = r0.x + r1.y + r2.z;
  f32x4* o = out + (size_t)b * BOARD_F4;
  if (g < 2)
    for (int i = 0; i < 23; ++i) {
      const int ch = 2 * i + g;
      if (ch < NCH) __builtin_nontemporal_store(f32x4{v, 1.f, 2.f, (float)ch}, o + ch * Q + q);
    }
  if (lane < 24) sb[lane] = r0 + r1;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 65536;
  const size_t n4 = (size_t)B * BOARD_F4, bytes = n4 * 16;
  f32x4* out;
  int* in;
  CK(hipMalloc(&out, bytes + (size_t)B * 48 + 4096));
  CK(hipMalloc(&in, (size_t)B * 64 * 4));
  CK(hipMemset(in, 0, (size_t)B * 64 * 4));
  f32x4* st;
  CK(hipMalloc(&st, (size_t)B * 192 * 16));
  CK(hipMemset(st, 0, (size_t)B * 192 * 16));
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
    printf("%-10s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  run("pairs", [&] { hipLaunchKernelGGL(pairs, dim3(B), dim3(64), 0, 0, out, B); });
  run("pairs_nt", [&] { hipLaunchKernelGGL(pairs_nt, dim3(B), dim3(64), 0, 0, out, B); });
  run("flat", [&] { hipLaunchKernelGGL(flat, dim3(B), dim3(64), 0, 0, out, B); });
  run("flat_nt", [&] { hipLaunchKernelGGL(flat_nt, dim3(B), dim3(64), 0, 0, out, B); });
  run("pairs_lat", [&] { hipLaunchKernelGGL(pairs_lat, dim3(B), dim3(64), 0, 0, out, in, B); });
  run("mixed", [&] { hipLaunchKernelGGL(mixed, dim3(B), dim3(64), 0, 0, out, st, B); });
  run("mixed_ro", [&] { hipLaunchKernelGGL(mixed_ro, dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r1", [&] { hipLaunchKernelGGL((mixed_t<1, 0, 0>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r2", [&] { hipLaunchKernelGGL((mixed_t<2, 0, 0>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r3", [&] { hipLaunchKernelGGL((mixed_t<3, 0, 0>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r1_lds", [&] { hipLaunchKernelGGL((mixed_t<1, 6304, 0>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r3_lds", [&] { hipLaunchKernelGGL((mixed_t<3, 6304, 0>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r3_s1k", [&] { hipLaunchKernelGGL((mixed_t<3, 6304, 1000>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r3_s2k", [&] { hipLaunchKernelGGL((mixed_t<3, 6304, 2000>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r1_s2k", [&] { hipLaunchKernelGGL((mixed_t<1, 6304, 2000>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("m_r1_s4k", [&] { hipLaunchKernelGGL((mixed_t<1, 6304, 4000>), dim3(B), dim3(64), 0, 0, out, st, B); });
  run("stream", [&] { hipLaunchKernelGGL(stream, dim3(4096), dim3(256), 0, 0, out, n4); });
  run("stream_nt", [&] { hipLaunchKernelGGL(stream_nt, dim3(4096), dim3(256), 0, 0, out, n4); });
  run("stream_nt16k", [&] { hipLaunchKernelGGL(stream_nt, dim3(16384), dim3(256), 0, 0, out, n4); });
  run("flat4_nt", [&] { hipLaunchKernelGGL(flat4_nt, dim3((B + 3) / 4), dim3(256), 0, 0, out, B); });
  run("flat4", [&] { hipLaunchKernelGGL(flat4, dim3((B + 3) / 4), dim3(256), 0, 0, out, B); });
  run("persist2k", [&] { hipLaunchKernelGGL(persist_nt, dim3(2048), dim3(64), 0, 0, out, B); });
  run("persist8k", [&] { hipLaunchKernelGGL(persist_nt, dim3(8192), dim3(64), 0, 0, out, B); });
  run("flat_nt_al", [&] { hipLaunchKernelGGL(flat_nt_al, dim3(B), dim3(64), 0, 0, out, B); });
  run("flat_nt_shift", [&] { hipLaunchKernelGGL(flat_nt_shift, dim3(B), dim3(64), 0, 0, out, B); });
  run("pairs_nt_al", [&] { hipLaunchKernelGGL(pairs_nt_al, dim3(B), dim3(64), 0, 0, out, B); });
  run("pairs_al", [&] { hipLaunchKernelGGL(pairs_al, dim3(B), dim3(64), 0, 0, out, B); });
  run("mixed_shift", [&] { hipLaunchKernelGGL(mixed_shift, dim3(B), dim3(64), 0, 0, out, st, B); });
  run("mixed_nt", [&] { hipLaunchKernelGGL(mixed_nt, dim3(B), dim3(64), 0, 0, out, st, B); });
  run("flat_nt2", [&] { hipLaunchKernelGGL(flat_nt, dim3(B), dim3(64), 0, 0, out, B); });
  run("flat_nt_al2", [&] { hipLaunchKernelGGL(flat_nt_al, dim3(B), dim3(64), 0, 0, out, B); });
  run("flat2_nt", [&] { hipLaunchKernelGGL(flat2_nt, dim3(B / 2), dim3(64), 0, 0, out, B); });
  CK(hipFree(out));
  CK(hipFree(in));
  return 0;
}
