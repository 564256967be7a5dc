// td_wave.h -- wave-level helpers shared by the step and layout kernels (td_step.hip,
// td_wavegen.h): exact-rounding f64 / f32 intrinsics, ballots and lane broadcasts,
// agent-scope relaxed accesses, the board claim, state stores and the wave sync.
#pragma once
#include <hip/hip_runtime.h>

#include "td_kernels.h"

namespace td {

// ---------------------------------------------------------------------------
// exact-rounding helpers (Python float / numpy float32 semantics)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double dsub(double a, double b) { return __dsub_rn(a, b); }
__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double ddiv(double a, double b) { return __ddiv_rn(a, b); }
__device__ __forceinline__ double pymin(double a, double b) { return b < a ? b : a; }  // min(a, b)
__device__ __forceinline__ float f32(double x) { return __double2float_rn(x); }

__device__ __forceinline__ int ctz64(uint64_t m) { return __builtin_ctzll(m); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
// Lane l's value (l wave-uniform): a scalar broadcast, no LDS traffic.
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rdl(float v, int l) { return __int_as_float((int)rdl((uint32_t)__float_as_int(v), l)); }
__device__ __forceinline__ double rdl(double v, int l) {
  return __hiloint2double((int)rdl((uint32_t)__double2hiint(v), l), (int)rdl((uint32_t)__double2loint(v), l));
}

// Agent-scope relaxed accesses through the global address space (global_load /
// global_store ... sc1, never flat): the words two concurrently running grids
// hand over (layout tags, ring counters).
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A board's layout stream (np_mt) and its ring tail are written only by the refill
// wave holding the board's claim word (several refills may be in flight on side
// streams).  Take it with an agent-scope CAS + acquire; give it back after the
// wave's stores have drained.  Everything the claim protects is stored write-through
// (sc1, st_relaxed), so no release fence is needed (MI355X_MICROARCH.md, publish
// recipe R1): a release fence writes back the XCD's whole L2, full of the step
// kernel's dirty observation lines, and ~490 of them per refill launch cost the
// 20x20 multi-action step 3.6 % (335.5 -> 323.7 us per step without them).
__device__ __forceinline__ bool claim_board(uint32_t* claim, int lane) {
  uint32_t got = 0;
  if (lane == 0) got = atomicCAS(claim, 0u, 1u) == 0u ? 1u : 0u;
  got = __builtin_amdgcn_readfirstlane(got);
  if (got) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return got != 0;
}
__device__ __forceinline__ void release_board(uint32_t* claim, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lane == 0) st_relaxed(claim, 0u);
}

// Per-board state and output stores: plain stores.  These arrays hold a few bytes per
// board, so a line is shared by neighbouring boards and the XCD L2 merges the plain
// stores; 65,536 boards at L = 10 measured 224 us plain, 227 us write-through and 287 us
// non-temporal (partial-line writes to HBM, round 1).
template <class T>
__device__ __forceinline__ void sst(T* p, T v) { *p = v; }

// The step of one board runs in one wave: its LDS hand-offs between lanes need the
// wave's LDS operations drained and the compiler kept from moving memory accesses
// across, not a workgroup barrier -- so the small-batch kernel can give a board a
// second wave that waits at one real barrier for the observation (td_step_kernel_small2).
__device__ __forceinline__ void wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace td
