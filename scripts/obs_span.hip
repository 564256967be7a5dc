// obs_span.hip -- diagnostic: is the 7-TB/s store shape (16 waves writing one board's
// 18,000-B row at once, a workgroup per board: obs_ceiling.hip shapes) fast because few
// boards are being written per CU, or because the boards being written at any moment lie in
// a narrow address band?  The same stores with three board orders:
//   lin   block i -> xcd_board(i): each XCD walks its contiguous range in block order (the
//         resident workgroups write neighbouring boards)
//   scat  block i -> the same XCD range, but the (i / 8)-th board of it bit-reversed: the
//         resident workgroups write boards spread over the XCD's whole range
// for 16 waves per board (2 boards per CU written at a time) and 1 wave per board (32).
// 65,536 boards x 18,000 B, whole lines non-temporal, the two shared lines plain; contiguous.
//   hipcc --offload-arch=gfx950 -O3 scripts/obs_span.hip -o scripts/bin/obs_span
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
constexpr int ROWB = 18000, NB = 65536, PER = NB / 8, PBITS = 13;  // 8,192 boards per XCD range
static_assert((1 << PBITS) == PER, "bit reversal over the XCD range");

template <bool SCAT>
__device__ __forceinline__ int board_of(int i) {
  const int x = i & 7;
  int j = i >> 3;
  if (SCAT) j = (int)(__builtin_bitreverse32((unsigned)j) >> (32 - PBITS));
  return x * PER + j;
}

// NW waves per workgroup, one board per workgroup; wave w writes windows w, w + NW, ...
template <int NW, bool SCAT>
__global__ __launch_bounds__(64 * NW) void k_span(char* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = board_of<SCAT>((int)blockIdx.x);
  const size_t start = (size_t)b * ROWB;
  const int mis = (int)(start & 127);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + start, 0, ROWB, 0x00020000);
  const int K = (ROWB + mis + 1023) / 1024;
  for (int k = wv; k < K; k += NW) {
    const int o = k * 1024 + lane * 16 - mis;
    const unsigned off = o < 0 ? 0x80000000u : (unsigned)o;
    const int line = (o + mis) >> 7;
    const bool shared = (mis && line == 0) || (((ROWB + mis) & 127) && line == ((ROWB + mis) >> 7));
    const u32x4 v{(unsigned)b, (unsigned)o, 0u, 0u};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? 0x80000000u : off, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, shared ? off : 0x80000000u, 0, 0);
  }
}

int main() {
  const size_t bytesz = (size_t)NB * ROWB + 4096;
  char* buf = nullptr;
  CK(hipExtMallocWithFlags((void**)&buf, bytesz, hipDeviceMallocContiguous));
  CK(hipMemset(buf, 0, bytesz));
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
  const double bytes = (double)NB * ROWB;
#define SPAN(NW, S)                                                                                              \
  {                                                                                                              \
    const double t = timed([&] { hipLaunchKernelGGL((k_span<NW, S>), dim3(NB), dim3(64 * NW), 0, 0, buf); });     \
    std::printf("waves/board %2d  order %s  %.1f us  %.2f TB/s\n", NW, S ? "scat" : "lin ", t, bytes / t / 1e6); \
  }
  for (int r = 0; r < 2; ++r) {
    SPAN(16, false) SPAN(16, true) SPAN(4, false) SPAN(4, true) SPAN(1, false) SPAN(1, true)
  }
  // coverage of the scattered order: every board written once
  CK(hipMemset(buf, 0, bytesz));
  hipLaunchKernelGGL((k_span<16, true>), dim3(NB), dim3(1024), 0, 0, buf);
  CK(hipDeviceSynchronize());
  long bad = 0;
  for (int b = 0; b < NB; b += 13) {
    unsigned w = 0;
    CK(hipMemcpy(&w, buf + (size_t)b * ROWB + 256, 4, hipMemcpyDeviceToHost));
    bad += w != (unsigned)b;
  }
  std::printf("coverage: %ld bad\n", bad);
  return bad != 0;
}
