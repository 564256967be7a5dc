// hbm_ceiling.hip -- diagnostic: the write / read / mixed streaming rates of this part
// against the footprint, to place the step kernel's observation stream (1.18 GB of
// 16-B stores per launch at 65,536 boards) against what HBM3E takes: grid-stride kernels
// (256-thread blocks, 16 B per lane per instruction) over footprints of 32 MB - 2 GB,
// then 1,180 MB written in contiguous per-wave chunks of 1-256 KB.  Every footprint is
// swept repeatedly (steady state: the Infinity Cache holds the last 256 MiB of it) and
// timed over 20 launches.
//   hipcc --offload-arch=gfx950 -O3 scripts/hbm_ceiling.hip -o scripts/bin/hbm_ceiling
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

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// kind 0 plain, 1 non-temporal, 2 write-through (sc1)
template <int KIND>
__global__ __launch_bounds__(256) void wr(f32x4* out, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  const f32x4 v = f32x4{1.f, 2.f, 3.f, (float)threadIdx.x};
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) {
    if constexpr (KIND == 0) out[i] = v;
    else if constexpr (KIND == 1) __builtin_nontemporal_store(v, out + i);
    else {
      // sc1 buffer stores need a 32-bit offset: rebase per 1-GiB window
      const size_t base = i & ~(size_t)((1u << 26) - 1);
      const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(out + base, 0, 0x7fffffff, 0x00020000);
      (void)rs;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r2, (int)((i - base) * 16), 0, 16);
    }
  }
}

__global__ __launch_bounds__(256) void rd(const f32x4* in, size_t n, float* sink) {
  const size_t stride = (size_t)gridDim.x * 256;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) acc += in[i];
  if (acc.x == 12345.f) sink[0] = acc.y + acc.z + acc.w;  // never true: keeps the loads
}

// one read for every `ratio` writes (the step kernel reads ~1/10 of what it writes)
__global__ __launch_bounds__(256) void mix(const f32x4* in, f32x4* out, size_t n, int ratio, float* sink) {
  const size_t stride = (size_t)gridDim.x * 256;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) {
    if (i % ratio == 0) acc += in[i / ratio];
    __builtin_nontemporal_store(f32x4{1.f, 2.f, 3.f, acc.x}, out + i);
  }
  if (acc.x == 12345.f) sink[0] = acc.y;
}

// one wave per workgroup; a wave writes whole contiguous chunks of `chunk` float4 (the
// step kernel's shape: a board's 18 KB observation from one wave), chunks in order
template <int KIND>
__global__ __launch_bounds__(64) void wr_chunk(f32x4* out, size_t n_chunks, int chunk) {
  const f32x4 v = f32x4{1.f, 2.f, 3.f, (float)threadIdx.x};
  for (size_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    f32x4* o = out + c * (size_t)chunk;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(o, 0, chunk * 16, 0x00020000);
    for (int j = threadIdx.x; j < chunk; j += 64) {
      if constexpr (KIND == 0) o[j] = v;
      else if constexpr (KIND == 1) __builtin_nontemporal_store(v, o + j);
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, j * 16, 0, 16);
    }
  }
}

static void chunked(f32x4* b, int cus, hipEvent_t e0, hipEvent_t e1) {
  const size_t bytes = (size_t)1180 << 20;
  std::printf("\n1,180 MB written in contiguous per-wave chunks (one 64-thread wave per workgroup, %d workgroups)\n",
              cus * 32);
  std::printf("%10s %12s %12s %12s\n", "chunk", "plain", "nt", "sc1");
  const int chunks_kb[] = {1, 4, 16, 18, 64, 256};
  for (int kb : chunks_kb) {
    const int chunk = kb == 18 ? 1125 : kb * 64;  // float4 per chunk (18 KB: the 10x10 observation, 1,125 units)
    const size_t n_chunks = bytes / 16 / chunk;
    double r[3];
    for (int k = 0; k < 3; ++k) {
      auto launch = [&]() {
        if (k == 0) hipLaunchKernelGGL(wr_chunk<0>, dim3(cus * 32), dim3(64), 0, 0, b, n_chunks, chunk);
        else if (k == 1) hipLaunchKernelGGL(wr_chunk<1>, dim3(cus * 32), dim3(64), 0, 0, b, n_chunks, chunk);
        else hipLaunchKernelGGL(wr_chunk<2>, dim3(cus * 32), dim3(64), 0, 0, b, n_chunks, chunk);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      r[k] = (double)n_chunks * chunk * 16 * 20 / (ms * 1e-3) / 1e12;
    }
    std::printf("%7d KB %9.2f TB/s %9.2f TB/s %9.2f TB/s\n", kb, r[0], r[1], r[2]);
  }
}

int main(int argc, char** argv) {
  const size_t max_bytes = (size_t)2 << 30;
  f32x4 *a = nullptr, *b = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&b, max_bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, max_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;  // 8 blocks of 256 threads per CU: 32 waves per CU
  const size_t sizes_mb[] = {32, 64, 128, 192, 256, 384, 512, 1024, 1180, 2048};
  std::printf("%8s %12s %12s %12s %12s %14s\n", "MB", "write plain", "write nt", "write sc1", "read", "mix 1:10 (r+w)");
  for (size_t mb : sizes_mb) {
    const size_t bytes = mb << 20, n = bytes / 16;
    double r[5];
    for (int k = 0; k < 5; ++k) {
      auto launch = [&]() {
        if (k == 0) hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(256), 0, 0, b, n);
        else if (k == 1) hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(256), 0, 0, b, n);
        else if (k == 2) hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(256), 0, 0, b, n);
        else if (k == 3) hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, a, n, sink);
        else hipLaunchKernelGGL(mix, dim3(grid), dim3(256), 0, 0, a, b, n, 10, sink);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      const int reps = 20;
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = k == 4 ? (double)bytes * 1.1 : (double)bytes;
      r[k] = moved * reps / (ms * 1e-3) / 1e12;
    }
    std::printf("%8zu %9.2f TB/s %9.2f TB/s %9.2f TB/s %9.2f TB/s %11.2f TB/s\n", mb, r[0], r[1], r[2], r[3], r[4]);
  }
  chunked(b, cus, e0, e1);
  return 0;
}
