// td_board.h -- board rules and observation encoding of the step kernels (td_step.hip):
// fail codes, the tower nibble of an LDS cell word, Chebyshev distance, Enemy.damage, the
// binary / broadcast / distance / enemy channel classes of the (45, L, L) observation, the
// dry-ring wait and the kernarg-segment read of the step arguments.
#pragma once
#include <hip/hip_runtime.h>

#include "td_common.h"
#include "td_kernels.h"
#include "td_wave.h"

namespace td {

constexpr int MAX_KERNEL_L = 32;  // generic-L kernels: L <= 32

enum : int { FC_OK = 0, FC_COST = 1, FC_POS = 2, FC_LVMAX = 3, FC_TARGET = 4, FC_CAP = 6 };  // utils/fail_code.py

// The tower on a cell lives in the LDS copy of its cell word, bits 10-13 (unused by the
// layout format, td_layout.h): bit 3 of the nibble = a tower, bit 2 its level, bits 0-1
// its type.  (A byte map of its own cost NC bytes of LDS per board: 900 at 30x30, where the
// board image bounds residency.)  HBM cell words never carry it (store_cells masks it).
constexpr uint32_t kTwBits = 0xFu << 10;
__device__ __forceinline__ uint32_t tw_nib(int lv, int type) { return (0x8u | ((uint32_t)lv << 2) | (uint32_t)type) << 10; }
// the tower byte of a cell word: 0 none, else 0x80 | lv << 2 | type
__device__ __forceinline__ uint32_t twr_of(uint32_t w) {
  const uint32_t n = (w >> 10) & 0xFu;
  return (n & 8u) ? (0x80u | (n & 7u)) : 0u;
}
// packed cell words (pack_obs_cells): the march direction and the distance to the end
__device__ __forceinline__ int pk_dir(uint32_t w) { return (int)((w >> 21) & 3u); }
__device__ __forceinline__ int pk_dist(uint32_t w) { return (int)(w >> 24); }

// Division by the board side L of a cell index (0 <= v < 1024, L <= 32) with one 24-bit
// multiply, v_mul_u32_u24 (full rate): v / L = (v * Lm) >> 16, Lm = ceil(2^16 / L), exact
// since (1024 - 1) * (Lm * L - 2^16) < 32 * 1024 < 2^16.  (Division by a constant takes
// v_mul_hi_u32, and the remainder a v_mul_lo_u32: quarter-rate instructions.)
__host__ __device__ constexpr uint32_t side_magic(int L) { return (65536u + (uint32_t)L - 1u) / (uint32_t)L; }
__device__ __forceinline__ int div_side(int v, uint32_t Lm) { return (int)(__umul24((uint32_t)v, Lm) >> 16); }

// x / D for 0 <= x < LIM, the same way at a compile-time divisor (the observation's unit
// -> channel): the smallest shift S with (LIM - 1) * e < 2^S, e = M * D - 2^S
// (Granlund-Montgomery), and a product below 2^32.
template <int D, int LIM>
struct Div24 {
  static constexpr int pick() {
    for (int s = 8; s <= 24; ++s) {
      const long long m = ((1ll << s) + D - 1) / D, e = m * D - (1ll << s);
      if ((long long)(LIM - 1) * e < (1ll << s) && (long long)(LIM - 1) * m < (1ll << 32) && m < (1ll << 24)) return s;
    }
    return -1;
  }
  static constexpr int S = pick();
  static_assert(S > 0, "no exact 24-bit reciprocal");
  static constexpr uint32_t M = (uint32_t)(((1ll << S) + D - 1) / D);
  __device__ static int div(int x) { return (int)(__umul24((uint32_t)x, M) >> S); }
};

__device__ __forceinline__ int cheb(int a, int b, int L, uint32_t Lm) {
  const int ra = div_side(a, Lm), rb = div_side(b, Lm);
  int dr = ra - rb, dc = (a - ra * L) - (b - rb * L);
  dr = dr < 0 ? -dr : dr;
  dc = dc < 0 ? -dc : dc;
  return dr > dc ? dr : dc;
}

// Enemy.damage, TDElements.py:19-28
__device__ __forceinline__ double damage(double LP, double atk, double def, bool magic) {
  double dmg = magic ? atk : (dsub(atk, def) < 0.0 ? 0.0 : dsub(atk, def));
  double lo = dmul(atk, 0.05);
  if (dmg < lo) dmg = lo;
  LP = dsub(LP, dmg);
  if (LP <= 0.0) LP = 0.0;
  return LP;
}

// Binary observation channels as bits of one word per cell (bit c = channel c):
// 0-3 roads, 4 end, 6-8 starts, 14 buildable (map[6] == 0), 15-16 tower level,
// 17-20 tower type (TDBoard.py:113-133).
constexpr uint32_t kBinaryChannels = 0x1FC1DFu;

__device__ __forceinline__ uint32_t cell_bits(uint32_t w, uint32_t tw) {
  uint32_t m = (w & 0x1Fu) | (((w >> 5) & 7u) << 6) | ((w >> 24) == 0u ? (1u << 14) : 0u);
  if (tw & 0x80u) m |= (1u << (15u + ((tw >> 2) & 1u))) | (1u << (17u + (tw & 3u)));
  return m;
}

__device__ __forceinline__ float bitf(uint32_t m, int ch) { return (float)((m >> ch) & 1u); }

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Channel kinds of the observation (TDBoard.get_states, :112-143).
enum ObsKind : int { OK_BIN, OK_CONST, OK_D9, OK_ENEMY };
__host__ __device__ constexpr int obs_kind(int ch) {
  return ch == 9 ? OK_D9
       : (ch < 32 && ((kBinaryChannels >> ch) & 1u)) ? OK_BIN
       : (ch >= 25 && ch < 41) ? OK_ENEMY
       : OK_CONST;
}

// Channel classes of the observation as 64-bit channel masks (TDBoard.get_states,
// :112-143): bits of the packed cell word, the enemy_LP planes, channel 9 (distance
// by table), and the broadcast channels.
constexpr uint64_t kChBin = kBinaryChannels;
constexpr uint64_t kChD9 = 1ull << 9;
constexpr uint64_t kChEnemy = 0xFFFFull << 25;
constexpr uint64_t kChAll = (1ull << NCH) - 1;
constexpr uint64_t kChConst = kChAll & ~(kChBin | kChD9 | kChEnemy);

// The step wave of board b found layout `head` unpublished at the episode end.  If a
// refill wave holds the board's claim it is drawing exactly this layout (an empty ring
// is urgent: its draw runs to the end): wait for the tag, bounded (1 s; a wait that gives
// up sets FLAG_CLAIM_TIMEOUT in *flags).  Otherwise the ring ran dry with no refill beside
// the step: the board is flagged no_layout by the caller.  (The step wave drawing the
// layout itself measured 4.5x slower steps: the called draw spills 0.5-1 KB of scratch
// per lane in every step kernel, profiles/r03/s4.)  True when layout `head` is ready.
__device__ __forceinline__ bool take_dry_ring(const StepArgs& a, int b, uint32_t head, int* flags) {
  uint32_t* const slot = a.nxt + ((size_t)b * NSLOT + head % NSLOT) * a.slot_words;
  const uint32_t want = slot_tag(head);
  // a board whose earlier wait already gave up does not wait again (every later step of a
  // claim never given back would otherwise stall 1 s): it takes the layout if it is there
  if (*flags & FLAG_CLAIM_TIMEOUT) return ld_relaxed(slot) == want;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (ld_relaxed(a.lay_claim + b) == 0u) return ld_relaxed(slot) == want;
    if (ld_relaxed(slot) == want) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 >= kTakeSpinTicks) {
      *flags |= FLAG_CLAIM_TIMEOUT;
      return false;
    }
    __builtin_amdgcn_s_sleep(64);
  }
}

// The kernel's StepArgs, read through the kernarg segment where each field is used
// (scalar loads that hit the constant cache) instead of being held in SGPRs for the
// whole kernel: with 80 SGPRs (8 waves per SIMD) the small kernels otherwise spilled ~50
// SGPRs into VGPR lanes and read them back with ~150 v_readlane (static counts, L = 10):
// +1.4 % at 4,096 / 8,192 boards (profiles/r03/s10).  The large kernel keeps its
// by-value arguments (106 SGPRs at 7 waves per SIMD; read through the segment it fell
// to 83 SGPRs, ran 8 waves per SIMD and lost 4.6 % at 65,536 boards).  The StepArgs must
// be the kernel's first argument (kernarg offset 0).
__device__ __forceinline__ const StepArgs& kargs(const StepArgs& a) {
  (void)a;
  return *(const StepArgs*)__builtin_amdgcn_kernarg_segment_ptr();  // (C cast: leaves the constant address space)
}

}  // namespace td
