// write_ceiling.hip -- diagnostic: HBM write rates of the store shapes that matter for the
// step kernel's observation stream, next to the guide's plain-store row
// (MI355X_MICROARCH.md, "plain stores of the same shape": one dword per lane, 256 B per
// wave-instruction, random 2,304-B rows of a 75 MB or 302 MB table, 8 waves per CU,
// 6.0-6.2 TB/s).  Every kernel writes a whole table per launch; rates are bytes written
// / the mean of 20 launches (hipEvents), after 3 warm-up launches.
//   row   : rows of R bytes in random order, each swept by one wave with consecutive
//           instructions (dword = 256 B per instruction, b128 = 1 KB), persistent waves
//           (8 per CU unless stated)
//   board : the step kernel's shape -- one 64-lane workgroup per 18,000-B row (a 10x10
//           observation), rows back to back in board order, 1-KB windows aligned to
//           128-B lines (lanes outside the row dropped by the buffer range), whole lines
//           non-temporal and the two lines shared with the neighbours sc1
//   hipcc --offload-arch=gfx950 -O3 scripts/write_ceiling.hip -o scripts/bin/write_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// aux bits of a buffer store: 0 plain, 2 non-temporal, 16 sc1 (write-through)
template <int W, int AUX>  // W: bytes per lane per instruction (4 or 16)
__global__ __launch_bounds__(256) void rows(char* base, const unsigned* order, int nrows, int rowb) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4) + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const int per = 64 * W;
  for (int r = wave; r < nrows; r += nw) {
    char* row = base + (size_t)order[r] * rowb;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, rowb, 0x00020000);
    for (int o = 0; o < rowb; o += per) {
      const int off = o + lane * W;
      if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32((unsigned)r, rs, off, 0, AUX);
      else __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)r, 1u, 2u, 3u}, rs, off, 0, AUX);
    }
  }
}

// One workgroup per board, the board's 18,000 B written in 128-B-aligned 1-KB windows.
template <int WHOLE_AUX, int SHARED_AUX>
__global__ __launch_bounds__(64) void boards(char* out, int rowb) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const size_t start = (size_t)b * rowb;
  const int n4 = rowb / 16, mis = (int)((start >> 4) & 7);
  const int head = mis ? 8 - mis : 0, tail = ((n4 + mis) & ~7) - mis;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, rowb, 0x00020000);
  const int K = (n4 + mis + 63) / 64;
  for (int k = 0; k < K; ++k) {
    const int i = lane - mis + 64 * k;
    const unsigned off = (unsigned)i * 16u;  // i < 0: huge, dropped
    const bool shared = i < head || i >= tail;
    const u32x4 v = u32x4{(unsigned)b, (unsigned)i, 0u, 0u};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? 0x80000000u : off, 0, WHOLE_AUX);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? off : 0x80000000u, 0, SHARED_AUX);
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
  return bytes / (ms / n * 1e-3) / 1e12;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t maxb = (size_t)1200 << 20;
  char* buf = nullptr;
  CK(hipMalloc(&buf, maxb + 4096));
  CK(hipMemset(buf, 0, maxb + 4096));
  std::printf("CUs %d\n", cus);
  const size_t tables[] = {(size_t)75 << 20, (size_t)302 << 20, (size_t)1180 << 20};
  for (int rowb : {2304, 18432}) {
    for (size_t tb : tables) {
      const int nrows = (int)(tb / rowb);
      std::vector<unsigned> ord(nrows);
      for (int i = 0; i < nrows; ++i) ord[i] = i;
      srand(7);
      for (int i = nrows - 1; i > 0; --i) std::swap(ord[i], ord[rand() % (i + 1)]);
      unsigned* dord = nullptr;
      CK(hipMalloc(&dord, nrows * 4));
      CK(hipMemcpy(dord, ord.data(), nrows * 4, hipMemcpyHostToDevice));
      const double bytes = (double)nrows * rowb;
      for (int wpc : {8, 16}) {
        const int grid = cus * wpc / 4;
        const double d0 = timed([&] { hipLaunchKernelGGL((rows<4, 0>), dim3(grid), dim3(256), 0, 0, buf, dord, nrows, rowb); }, bytes);
        const double d2 = timed([&] { hipLaunchKernelGGL((rows<4, 2>), dim3(grid), dim3(256), 0, 0, buf, dord, nrows, rowb); }, bytes);
        const double q0 = timed([&] { hipLaunchKernelGGL((rows<16, 0>), dim3(grid), dim3(256), 0, 0, buf, dord, nrows, rowb); }, bytes);
        const double q2 = timed([&] { hipLaunchKernelGGL((rows<16, 2>), dim3(grid), dim3(256), 0, 0, buf, dord, nrows, rowb); }, bytes);
        const double q16 = timed([&] { hipLaunchKernelGGL((rows<16, 16>), dim3(grid), dim3(256), 0, 0, buf, dord, nrows, rowb); }, bytes);
        std::printf("rows %5d B  table %5zu MB  %2d waves/CU | dword plain %.2f nt %.2f | b128 plain %.2f nt %.2f sc1 %.2f TB/s\n",
                    rowb, tb >> 20, wpc, d0, d2, q0, q2, q16);
      }
      CK(hipFree(dord));
    }
  }
  for (int nb : {8192, 16384, 65536}) {
    for (int rowb : {18000, 18432}) {
      const double bytes = (double)nb * rowb;
      const double a = timed([&] { hipLaunchKernelGGL((boards<2, 16>), dim3(nb), dim3(64), 0, 0, buf, rowb); }, bytes);
      const double p = timed([&] { hipLaunchKernelGGL((boards<0, 0>), dim3(nb), dim3(64), 0, 0, buf, rowb); }, bytes);
      const double w = timed([&] { hipLaunchKernelGGL((boards<16, 16>), dim3(nb), dim3(64), 0, 0, buf, rowb); }, bytes);
      std::printf("boards %5d x %5d B (%6.1f MB) | nt + sc1-shared %.2f | plain %.2f | sc1 %.2f TB/s\n", nb, rowb,
                  bytes / 1e6, a, p, w);
    }
  }
  return 0;
}
