// td_step.hip -- the batched gym-TD step on CDNA4 (gfx950).
//
// One 64-lane wavefront (= one workgroup) owns one board for the whole step:
// the board's slice of the SoA record is staged in LDS, every serial phase of the
// reference runs wave-uniform with wave ballots standing in for the reference's
// "first enemy in list order" scans, and the (45, L, L) float32 observation is
// written with 16-byte coalesced stores straight from LDS tables.
//
// Reference order of one env step:
//   cool-downs                     TDDefense.py:38-39 / TDAttack.py:31-32 / TDMulti.py:50-51
//   defender action                TDDefense.py:40-77, TDMulti.py:208-258
//   attacker action / opponent     TDGymBasic.py:81-108, TDAttack.py:36-48, TDMulti.py:199-241
//   TDBoard.step                   TDBoard.py:295-368
//   done / get_states / info       TDBoard.py:370-385, 85-144, TDDefense.py:81-87
//
// Floating point: the file is compiled with -ffp-contract=off and every f64/f32
// operation is an explicit correctly-rounded intrinsic where the reference's
// Python/numpy rounding order matters.
#include <hip/hip_runtime.h>

#include <hip/hip_ext.h>

#include "td_board.h"
#include "td_kernels.h"
#include "td_layout.h"
#include "td_rng.h"
#include "td_wave.h"
#include "td_wavegen.h"

#include <type_traits>
#include <utility>

namespace td {


// ---------------------------------------------------------------------------
// per-board LDS image
// ---------------------------------------------------------------------------
template <int NC>
struct alignas(16) Smem {
  static_assert(NC % 4 == 0, "cell and tower maps are moved in 16-B / 4-B units");
  uint32_t cell[NC];      // cell words (td_layout.h), + the tower on the cell in bits 10-13 (tw_nib)
  uint8_t grp[4][NC];     // enemy group (head enemy index) per (type, cell), 0xFF none
  union {
    struct {              // load .. march: the enemy list (written back right after the march)
      double eLP[ECAP];
      double eMg[ECAP];
    };
    float gst[ECAP][4];   // stats .. obs: group stats min, max, avg, count/8 by head enemy
  };
  uint32_t eInf[ECAP];
  double tCd[TCAP];
  uint32_t tInf[TCAP];
  union {
    struct {              // actions: the attacker's clusters (TD-atk / TD-2p), written out right after
      int32_t atk[24];
      int32_t real_atk[24];  // info['RealAction'] of the attacker
      int32_t fail_atk[4];   // info['FailCode'] of the attacker (-1 = no entry)
    };
    struct {              // observation
      float chv[48];      // broadcast channel values
      float d9[64];       // channel 9 by distance (road length < 2L <= 64)
    };
  };
  uint32_t early_go;         // td_step_kernel_small2: the binary-plane windows may be written early
  int32_t flags0;            // the board's flags as loaded (store_board: is the header's second half dirty?)
  TdDevCfg cfg;           // constant block, staged once per board: per-lane table lookups hit LDS
};

template <int NC>
__device__ __forceinline__ void set_tower(Smem<NC>& S, int cell, uint32_t nib) {
  S.cell[cell] = (S.cell[cell] & ~kTwBits) | nib;
}

// Stage the constant block into LDS (16 bytes per lane).
template <int NC>
__device__ __forceinline__ void stage_cfg(Smem<NC>& S, const TdDevCfg* g, int l = (int)(threadIdx.x & 63)) {
  static_assert(sizeof(TdDevCfg) % 16 == 0 && sizeof(TdDevCfg) <= 64 * 16, "cfg staging");
  if (l < (int)(sizeof(TdDevCfg) / 16))
    reinterpret_cast<uint4*>(&S.cfg)[l] = reinterpret_cast<const uint4*>(g)[l];
}
// The same in two halves, so that a step kernel issues the board's loads between them:
// staged in one piece, the block's load was waited for (vmcnt(0)) before any of the
// board's loads went out -- one L2 round trip in front of every board's step.
__device__ __forceinline__ uint4 load_cfg(const TdDevCfg* g, int l) {
  return l < (int)(sizeof(TdDevCfg) / 16) ? reinterpret_cast<const uint4*>(g)[l] : uint4{0u, 0u, 0u, 0u};
}
template <int NC>
__device__ __forceinline__ void store_cfg(Smem<NC>& S, uint4 v, int l) {
  if (l < (int)(sizeof(TdDevCfg) / 16)) reinterpret_cast<uint4*>(&S.cfg)[l] = v;
}

// Wave-uniform scalar board state (identical in every lane).
struct U {
  double cost_def, cost_atk, ep_ret, progress;
  double max_cost;  // captured at reset (TDBoard.py:70)
  int steps, base_LP, atk_cd, def_cd, n, nt, num_roads, end_cell, maxdist, flags, episodes;
  int max_base_LP;  // captured at reset (TDBoard.py:72)
  bool cells_dirty;  // map[6] changed (tower built / destroyed) or a new layout: write the cells back
  bool tw_dirty;     // the tower list changed (build / upgrade / destruct, reset): write tw_inf back
  uint64_t starts;  // start cells of roads 0-2, 16 bits each (a shift, not an indexed field: keeps U in registers)
  __device__ __forceinline__ int start(int road) const { return (int)((starts >> (16 * road)) & 0xffffu); }
  __device__ __forceinline__ void set_starts(uint32_t s0, uint32_t s1, uint32_t s2) {
    starts = (uint64_t)s0 | ((uint64_t)s1 << 16) | ((uint64_t)s2 << 32);
  }
};

struct Ctx {
  const TdDevCfg& C;  // the current constant block (epoch ep), staged in LDS
  int L, NCr, lane;
  const TdDevCfg* tab;  // every epoch's block (HBM)
  int ep;
  uint32_t Lm = side_magic(L);  // div_side's multiplier
};

// A value an enemy or tower captured when it was created or upgraded (TDElements.py:
// 4-43, 45-63, 134-170): from the block of its epoch -- the staged current one, or
// (after a paramConfig) an older block in HBM.
// The two loads are kept apart by an empty asm on the HBM value, waited for inside its
// branch: otherwise the compiler merges them into one FLAT load of a selected pointer,
// which waits with vmcnt(0) and lgkmcnt(0) at every call (16 FLAT loads in the small
// kernel).  Apart: -0.4 to -0.5 % at 32,768-65,536 boards, +-0.5 % below (r05/s26, s27;
// +-0.6 % in round 3, r03/s17).  The older block's address takes a 24-bit multiply
// (ep * sizeof(TdDevCfg) < 2^24); as x.tab[ep] it took a quarter-rate v_mad_u64_u32.
template <class F>
__device__ __forceinline__ double captured(const Ctx& x, int ep, F f) {
  double v = f(x.C);
  if (ep != x.ep) {
    double w = f(*reinterpret_cast<const TdDevCfg*>(reinterpret_cast<const char*>(x.tab) +
                                                    __umul24((uint32_t)ep, (uint32_t)sizeof(TdDevCfg))));
    __asm__ volatile("" : "+v"(w));
    v = w;
  }
  return v;
}

// ---------------------------------------------------------------------------
// CPython MT19937 for the built-in opponent, state in HBM, wave-parallel twist
// ---------------------------------------------------------------------------
// CPython MT19937 with a lazy twist: word p of a new block is twisted when it is
// drawn.  In sequential order word p of the new block depends on old[p], old[p+1]
// (new[0] for p = 623) and old[p+397] (p < 227) or new[p-227] (p >= 227), all of
// which are available when p is drawn in order, so draws are bit-identical to
// CPython's block twist without ever running the 624-word loop in the step.
// State: w[0..623], pos = w[624], tw = w[625] (words [tw, 624) not yet twisted).
struct WaveMt {
  uint32_t* w;
  uint32_t pos, tw;
  uint32_t cache = 0, cbase = 0, cn = 0;  // lane j: tempered output for position cbase + j (j < cn)
  __device__ __forceinline__ void wrap() {
    tw = 0;
    pos = 0;
  }

  // Pre-draws still unused at the current position (0 after a block wrap).
  __device__ __forceinline__ uint32_t cached_left() const {
    const uint32_t d = pos - cbase;
    return d < cn ? cn - d : 0u;
  }
  // Pre-draw the next up-to-HOT_CACHE words in parallel, one per lane, for the next
  // step: issue() starts the loads, finish() (at the end of the step) lazily
  // twists, stores and tempers them -- the memory latency overlaps the step.
  uint32_t pa = 0, pnb = 0, pfar = 0;
  bool plazy = false, pmine = false;
  __device__ __forceinline__ void prefetch_issue(int lane) {
    if (pos >= (uint32_t)MT_N) wrap();
    cbase = pos;
    cn = (uint32_t)MT_N - pos < (uint32_t)HOT_CACHE ? (uint32_t)MT_N - pos : (uint32_t)HOT_CACHE;
    const uint32_t q = pos + (uint32_t)lane;
    pmine = (uint32_t)lane < cn;
    plazy = pmine && q >= tw;
    if (pmine) {
      pa = w[q];
      if (plazy) {
        // word q (< pos + 8 <= tw + 8) needs new[q - 227], twisted in an earlier step
        pnb = w[q == MT_N - 1 ? 0u : q + 1u];
        pfar = w[q < (uint32_t)(MT_N - MT_M) ? q + MT_M : q - (MT_N - MT_M)];
      }
    }
  }
  __device__ __forceinline__ void prefetch_finish(int lane) {
    const uint32_t q = cbase + (uint32_t)lane;
    uint32_t y = pa;
    if (plazy) {
      const uint32_t yy = (pa & 0x80000000u) | (pnb & 0x7fffffffu);
      y = pfar ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
      w[q] = y;  // after every lane's loads (data dependency)
    }
    if (cbase + cn > tw) tw = cbase + cn;
    cache = pmine ? mt_temper(y) : 0u;
  }
  __device__ __forceinline__ void prefetch(int lane) {
    prefetch_issue(lane);
    prefetch_finish(lane);
  }

  // Early pre-draw (the small kernels): the loads of the window [p0, p0 + 16)
  // at the position p0 the step starts from are issued right after the hot record is in,
  // before any of the step's stores -- their wait at the step's end then neither waits on
  // the memory latency nor, through the in-order vmcnt, on the step's own stores.  The step
  // draws d <= 8 words in practice; the next pre-drawn outputs are the window's lanes
  // d .. d + 7.  A lazily twisted word the step's slow path twisted meanwhile is twisted
  // again from the same old words (same value); a window the step outran (d > 8, or a
  // block wrap) falls back to the late pre-draw.
  static constexpr uint32_t kEarlyWin = 16;
  uint32_t ep0 = ~0u;  // the window's first position (~0u: none)
  __device__ __forceinline__ void early_issue(int lane) {
    // (pos <= tw always: the window's lazy words need old or already twisted words only)
    if (pos + kEarlyWin > (uint32_t)MT_N) return;
    ep0 = pos;
    const uint32_t q = pos + (uint32_t)lane;
    pmine = (uint32_t)lane < kEarlyWin;
    plazy = pmine && q >= tw;
    if (pmine) {
      pa = w[q];
      if (plazy) {
        pnb = w[q == MT_N - 1 ? 0u : q + 1u];
        pfar = w[q < (uint32_t)(MT_N - MT_M) ? q + MT_M : q - (MT_N - MT_M)];
      }
    }
  }
  __device__ __forceinline__ bool early_ok() const { return ep0 != ~0u && pos - ep0 <= kEarlyWin - 8u; }
  // The early window's outputs, or (outran: d > 8, a block wrap, no window) a late
  // pre-draw -- one tail for both, so that no field is stored on one branch only (LLVM
  // merges such stores through a pointer phi, and the object no longer fits registers).
  __device__ __forceinline__ void early_finish(int lane) {
    uint32_t base, n, d;
    if (early_ok()) {
      base = ep0; n = kEarlyWin; d = pos - ep0;
    } else {
      prefetch_issue(lane);  // (wraps if due; cbase = pos)
      base = cbase; n = cn; d = 0u;
    }
    const uint32_t q = base + (uint32_t)lane;
    uint32_t y = pa;
    if (plazy) {
      const uint32_t yy = (pa & 0x80000000u) | (pnb & 0x7fffffffu);
      y = pfar ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
      w[q] = y;  // (a word the step's slow path twisted meanwhile: the same value again)
    }
    if (base + n > tw) tw = base + n;
    const uint32_t t = pmine ? mt_temper(y) : 0u;
    cache = (uint32_t)__shfl((int)t, (int)(((uint32_t)lane + d) & 63u));
    cbase = pos;
    cn = n - d < (uint32_t)HOT_CACHE ? n - d : (uint32_t)HOT_CACHE;
  }

  __device__ __forceinline__ uint32_t next() {
    const uint32_t d = pos - cbase;
    if (d < cn) {
      ++pos;
      return rdl(cache, (int)d);  // d is wave-uniform: a scalar read, no LDS round trip
    }
    if (pos >= (uint32_t)MT_N) { wrap(); cn = 0; }
    uint32_t y;
    if (pos >= tw) {
      const uint32_t a = w[pos];
      const uint32_t nb = w[pos == MT_N - 1 ? 0u : pos + 1u];
      const uint32_t far = w[pos < (uint32_t)(MT_N - MT_M) ? pos + MT_M : pos - (MT_N - MT_M)];
      const uint32_t yy = (a & 0x80000000u) | (nb & 0x7fffffffu);
      y = far ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
      w[pos] = y;  // every lane stores the same word
      tw = pos + 1;
    } else {
      y = w[pos];
    }
    ++pos;
    return mt_temper(y);
  }
  __device__ __forceinline__ int64_t randbelow(int64_t n) {
    if (n <= 0) return 0;  // never reached on a valid board (guards against an unbounded loop)
    int k = 64 - __builtin_clzll((unsigned long long)n);
    uint32_t r = next() >> (32 - k);
    while ((int64_t)r >= n) r = next() >> (32 - k);
    return r;
  }
  __device__ __forceinline__ int64_t randint(int64_t a, int64_t b) { return a + randbelow(b - a + 1); }
  // numpy legacy RandomState.randint(lo, hi) (hi exclusive): masked rejection on 32-bit
  // outputs, no draw when hi - lo == 1; also shuffle's random_interval(i) = np_randint(0, i + 1)
  __device__ __forceinline__ int64_t np_randint(int64_t lo, int64_t hi) {
    if (hi <= lo + 1) return lo;
    const uint32_t rng = (uint32_t)(hi - lo - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v = next() & mask;
    while (v > rng) v = next() & mask;
    return lo + (int64_t)v;
  }
  __device__ __forceinline__ double random() {
    uint32_t x = next() >> 5, y = next() >> 6;
    return (x * 67108864.0 + y) * (1.0 / 9007199254740992.0);
  }
};

// The built-in opponents' random source (TDGymBasic.py:81-292).  random_agent=True
// (NP = false): the board's CPython stream.  random_agent=False (NP = true): the
// board's numpy layout stream (the one reset() draws roads from), except the destruct
// branch's tower index, which the reference still draws from CPython random (:191,
// :287).  Each method is one call site shape of the reference: ri(lo, hi) =
// random.randint(lo, hi) | np_random.randint(lo, hi + 1).  NP is a template argument,
// not a nullable pointer: a pointer chosen between two locals at run time would keep
// both streams in scratch memory.
template <bool NP>
struct OppRng {
  WaveMt& py;
  WaveMt& np;  // == py when !NP
  __device__ __forceinline__ int64_t ri(int64_t lo, int64_t hi) {
    if constexpr (NP) return np.np_randint(lo, hi + 1); else return py.randint(lo, hi);
  }
  __device__ __forceinline__ double rnd() {
    if constexpr (NP) return np.random(); else return py.random();
  }
  // random.shuffle's randbelow(i + 1) | np shuffle's random_interval(i)
  __device__ __forceinline__ int64_t shuffle_j(int64_t i) {
    if constexpr (NP) return np.np_randint(0, i + 1); else return py.randbelow(i + 1);
  }
  // random_enemy_lv0's cluster slot: random.randint(0, types) (:85) | np_random.randint(0, types) (:88)
  __device__ __forceinline__ int64_t slot(int64_t types) {
    if constexpr (NP) return np.np_randint(0, types); else return py.randint(0, types);
  }
};

// Runs f(OppRng<...>&) on the stream random_agent selects.  random_agent=False: board
// b's numpy layout stream, loaded from and stored back to its MT record (np_mt).
template <class F>
__device__ __forceinline__ void with_opp_rng(const StepArgs& a, int b, int lane, WaveMt& R, F&& f) {
  if (a.opp_np) {
    uint32_t* const npw = a.np_mt + (size_t)b * OPP_WORDS;
    WaveMt N{npw, npw[MT_N], npw[MT_N + 1]};
    N.cbase = N.pos;
    OppRng<true> G{R, N};
    f(G);
    if (lane == 0) { npw[MT_N] = N.pos; npw[MT_N + 1] = N.tw; }
  } else {
    OppRng<false> G{R, R};
    f(G);
  }
}

// ---------------------------------------------------------------------------
// defender operations (TDBoard.py:226-293), wave-uniform
// ---------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void diamond(Smem<NC>& S, const Ctx& x, int cell, int delta) {
  const int k = x.C.tower_distance, W = 2 * k + 1, L = x.L;
  const int r0 = div_side(cell, x.Lm), c0 = cell - r0 * L;
  for (int idx = x.lane; idx < W * W; idx += 64) {
    int i = idx / W - k, j = idx % W - k;
    int ai = i < 0 ? -i : i, aj = j < 0 ? -j : j;
    int r = r0 + i, c = c0 + j;
    if (ai + aj <= k && r >= 0 && r < L && c >= 0 && c < L) {
      uint32_t w = S.cell[r * L + c];
      int cnt = (int)(w >> 24) + delta;
      S.cell[r * L + c] = (w & 0x00ffffffu) | ((uint32_t)(cnt & 0xff) << 24);
    }
  }
  wsync();
}

template <int NC>
__device__ __forceinline__ int tower_build(Smem<NC>& S, U& u, const Ctx& x, int t, int cell) {
  const double price = x.C.t_price[t][0];
  if (u.cost_def < price) return FC_COST;                 // :228
  if (cw_block(S.cell[cell]) > 0) return FC_POS;          // :232
  if (u.nt >= TCAP) { u.flags |= FLAG_TW_OVERFLOW; return FC_CAP; }
  if (x.lane == 0) {
    S.tInf[u.nt] = tw_pack(cell, t, 0, x.ep, x.ep);
    S.tCd[u.nt] = 0.0;
    set_tower(S, cell, tw_nib(0, t));
  }
  u.nt += 1;
  u.cost_def = dsub(u.cost_def, price);                   // :238
  u.cells_dirty = true;
  u.tw_dirty = true;
  wsync();
  diamond(S, x, cell, +1);                                // :239-245
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int find_tower(Smem<NC>& S, const U& u, const Ctx& x, int cell) {
  bool hit = x.lane < u.nt && (int)(S.tInf[x.lane] & 0xfffu) == cell;
  uint64_t m = ballot(hit);
  return m ? ctz64(m) : -1;
}

template <int NC>
__device__ __forceinline__ int tower_lvup(Smem<NC>& S, U& u, const Ctx& x, int cell) {
  int k = find_tower(S, u, x, cell);
  if (k < 0) return FC_TARGET;                            // :269-271
  uint32_t ti = S.tInf[k];
  int t = (ti >> 12) & 3, lv = (ti >> 14) & 1;
  if (lv >= x.C.max_tower_lv) return FC_LVMAX;            // :252
  double price = x.C.t_price[t][lv + 1];                  // :256
  if (u.cost_def < price) return FC_COST;
  wsync();
  if (x.lane == 0) {
    S.tInf[k] = tw_pack(cell, t, lv + 1, tw_ec(ti), x.ep);
    set_tower(S, cell, tw_nib(lv + 1, t));
  }
  u.cost_def = dsub(u.cost_def, price);                   // :266
  u.tw_dirty = true;
  wsync();
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int tower_destruct(Smem<NC>& S, U& u, const Ctx& x, int cell) {
  int k = find_tower(S, u, x, cell);
  if (k < 0) return FC_TARGET;                            // :291-293
  uint32_t ti = S.tInf[k];
  int t = (ti >> 12) & 3, lv = (ti >> 14) & 1;
  // Tower.cost: tower_cost[t][0] when built, + tower_attack_interval[t][1] at the upgrade
  // (the upgrade_tower argument swap), each from the epoch it was captured in
  double value = captured(x, tw_ec(ti), [&](const TdDevCfg& c) { return c.t_price[t][0]; });
  if (lv >= 1) value = dadd(value, captured(x, tw_eu(ti), [&](const TdDevCfg& c) { return c.t_addcost[t][lv]; }));
  u.cost_def = dadd(u.cost_def, dmul(value, x.C.destruct_return));  // :276
  u.cost_def = pymin(u.cost_def, u.max_cost);                      // :277
  u.cells_dirty = true;
  u.tw_dirty = true;
  // towers.remove(t): keep the order of the rest (:278)
  uint32_t vi = 0;
  double vc = 0.0;
  int j = x.lane;
  if (j >= k && j + 1 < u.nt) { vi = S.tInf[j + 1]; vc = S.tCd[j + 1]; }
  wsync();
  if (j >= k && j + 1 < u.nt) { S.tInf[j] = vi; S.tCd[j] = vc; }
  if (x.lane == 0) set_tower(S, cell, 0u);
  u.nt -= 1;
  wsync();
  diamond(S, x, cell, -1);                                // :281-287
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int defender_op(Smem<NC>& S, U& u, const Ctx& x, int op, int cell) {
  if (op < 4) return tower_build(S, u, x, op, cell);
  if (op == 4) return tower_lvup(S, u, x, cell);
  return tower_destruct(S, u, x, cell);
}

// Multi-action defender: the serial (r, c, t) scan of TDDefense.py:42-60 /
// TDMulti.py:209-227.  The (6, L, L) int64 flags are read first with 16-B loads
// (8 in flight per lane) and folded into one 6-bit flag byte per cell in LDS (the
// group map grp[0], unused until enemy_stats).  Cells where no operation can change
// the board are skipped: per 64-cell chunk a ballot marks the cells whose flagged
// build / lvup / destruct would succeed in the CURRENT state, the first such cell
// runs the reference's exact serial sequence, and the ballot is recomputed.
// Skipped cells would only have produced failures, which leave no trace in
// multi-action mode.  The real actions (grp[1]) go out as int64 (6, L, L) in
// 128-B-aligned windows, like the observation.
// (In the two-wave kernel the second wave folds the flags while the first loads the
// board, and writes the real actions out after the step's actions: scan_fold /
// scan_write_real below, handed over at barriers.)
// The flags folded into grp[0] (grp[1] cleared); true when a flag is not 0 / 1 / 2.
template <int NC>
__device__ __forceinline__ bool scan_fold(Smem<NC>& S, int lane, int ncr, const int64_t* A) {
  const int n = 6 * ncr;
  uint8_t* flag = &S.grp[0][0];
  uint32_t* fw = reinterpret_cast<uint32_t*>(flag);
  for (int i = lane; i < (2 * NC) / 4; i += 64) fw[i] = 0u;  // grp[0] and grp[1]
  wsync();
  bool bad = false;
  if ((ncr & 1) == 0 && (reinterpret_cast<uintptr_t>(A) & 15u) == 0) {  // 16-B units of two cells of one plane
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
    const i64x2* A2 = reinterpret_cast<const i64x2*>(A);
    const int n2 = n / 2;
    constexpr int K = 8;  // 16-B loads in flight per lane
    // (not unrolled: with the trip count known (NC) the compiler unrolled this loop and
    // hoisted the next rounds' loads, 85-91 VGPRs at 20x20 and 182-188 at 30x30 in every
    // multi-action kernel; rolled, 62-63)
#pragma unroll 1
    for (int base = 0; base < n2; base += 64 * K) {
      i64x2 v[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = base + 64 * k + lane;
        v[k] = e < n2 ? __builtin_nontemporal_load(A2 + e) : i64x2{0, 0};
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = base + 64 * k + lane;
        if (e < n2) {
          const int pl = (2 * e) / ncr, c = 2 * e - pl * ncr;
          bad |= (unsigned long long)v[k].x > 2ull || (unsigned long long)v[k].y > 2ull;
          const uint32_t bits = ((v[k].x == 1 ? 1u : 0u) << (8 * (c & 3)) | (v[k].y == 1 ? 1u : 0u) << (8 * ((c + 1) & 3)))
                                << pl;
          if (bits) atomicOr(&fw[c >> 2], bits);
        }
      }
    }
  } else {
    for (int e = lane; e < n; e += 64) {
      const int64_t v = A[e];
      const int pl = e / ncr, c = e - pl * ncr;
      bad |= v < 0 || v > 2;
      if (v == 1) atomicOr(&fw[c >> 2], (1u << pl) << (8 * (c & 3)));
    }
  }
  const bool any_bad = ballot(bad) != 0ull;
  wsync();
  return any_bad;
}

// The real actions (grp[1]) out as int64 (6, L, L) in 128-B-aligned windows.
template <int NC>
__device__ __forceinline__ void scan_write_real(const Smem<NC>& S, int lane, int ncr, int64_t* R) {
  const int n = 6 * ncr;
  const uint8_t* real = &S.grp[1][0];
  if ((ncr & 1) == 0 && (reinterpret_cast<uintptr_t>(R) & 15u) == 0) {
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
    i64x2* R2 = reinterpret_cast<i64x2*>(R);
    const int n2 = n / 2, mis = (int)((reinterpret_cast<uintptr_t>(R2) >> 4) & 7u);
    for (int e = lane - mis; e < n2; e += 64) {
      if (e < 0) continue;
      const int pl = (2 * e) / ncr, c = 2 * e - pl * ncr;
      const uint32_t r2 = *reinterpret_cast<const uint16_t*>(real + c);
      __builtin_nontemporal_store(i64x2{(long long)((r2 >> pl) & 1u), (long long)((r2 >> (8 + pl)) & 1u)}, R2 + e);
    }
  } else {
    for (int e = lane; e < n; e += 64) {
      const int pl = e / ncr;
      R[e] = (real[e - pl * ncr] >> pl) & 1u;
    }
  }
}

// FOLD: the flags are folded here (else by the second wave, `bad` its verdict); WRITE:
// the real actions are written here (else by the second wave after barrier (A)).
template <int NC, bool FOLD = true, bool WRITE = true>
__device__ __forceinline__ void defender_scan(Smem<NC>& S, U& u, const Ctx& x, const int64_t* A, int64_t* R, bool active,
                                              bool bad = false) {
  const TdDevCfg& C = x.C;
  const int ncr = x.NCr;
  uint8_t* flag = &S.grp[0][0];
  uint8_t* real = &S.grp[1][0];
  if constexpr (FOLD) bad = scan_fold(S, x.lane, ncr, A);
  if (bad) u.flags |= FLAG_BAD_ACTION;
  for (int base = 0; base < ncr && active; base += 64) {
    const int cell = base + x.lane;
    const bool valid = cell < ncr;
    const uint32_t fl = valid ? flag[cell] : 0u;
    int last = -1;
    while (true) {
      bool cand = false;
      if (valid && fl && x.lane > last) {
        uint32_t w = S.cell[cell];
        uint32_t tw = twr_of(w);
        bool canb = false;
        if (cw_block(w) == 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (((fl >> t) & 1u) && !(u.cost_def < C.t_price[t][0])) canb = true;
        }
        bool hasT = (tw & 0x80u) != 0;
        int tlv = (tw >> 2) & 1, tty = tw & 3;
        bool canl = hasT && ((fl >> 4) & 1u) && tlv < C.max_tower_lv && !(u.cost_def < C.t_price[tty][tlv + 1]);
        bool cand_d = hasT && ((fl >> 5) & 1u);
        cand = canb || canl || cand_d;
      }
      uint64_t m = ballot(cand);
      if (!m) break;
      const int j = ctz64(m);
      const int c = base + j;
      const uint32_t f = rdl(fl, j);
      uint32_t rb = 0;
      for (int t = 0; t < 4; ++t)
        if ((f >> t) & 1u)
          if (tower_build(S, u, x, t, c) == FC_OK) { rb |= 1u << t; u.def_cd = C.def_interval; }
      if ((f >> 4) & 1u)
        if (tower_lvup(S, u, x, c) == FC_OK) { rb |= 16u; u.def_cd = C.def_interval; }
      if ((f >> 5) & 1u)
        if (tower_destruct(S, u, x, c) == FC_OK) { rb |= 32u; u.def_cd = C.def_interval; }
      if (x.lane == j) real[c] = (uint8_t)rb;
      last = j;
    }
  }
  wsync();
  if (WRITE && R) scan_write_real(S, x.lane, ncr, R);
}

// ---------------------------------------------------------------------------
// attacker: summon_cluster (TDBoard.py:199-224)
// ---------------------------------------------------------------------------
// Cluster types / real actions are packed 4 bits per slot (slot k at bits 4k..4k+3).
template <int NC>
__device__ __forceinline__ int summon_cluster(Smem<NC>& S, U& u, const Ctx& x, uint32_t types, int road, uint32_t* real) {
  const TdDevCfg& C = x.C;
  const int lv = u.progress >= C.enemy_upgrade_at ? 1 : 0;  // :201
  const int st = u.start(road);
  bool tried = false, summoned = false;
  uint32_t rp = 0;
  // the four types' cost (lanes 0-3) and max LP (lanes 4-7) at this level in ONE LDS read,
  // then read per slot from those lanes (8 dependent LDS round trips before, one per slot)
  const double tab = x.lane < 4 ? C.e_cost[x.lane & 3][lv] : C.e_lp[x.lane & 3][lv];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int t = (int)((types >> (4 * k)) & 0xfu);
    int r = t;
    if (t != 4) {                                           // :207-209
      tried = true;
      const double cost = rdl(tab, t);
      if (u.cost_atk < cost) {                              // :212-213
        r = 4;
      } else if (u.n >= ECAP) {
        u.flags |= FLAG_EN_OVERFLOW;
        r = 4;
      } else {
        u.cost_atk = dsub(u.cost_atk, cost);                // :215
        const double lp = rdl(tab, 4 + t);
        if (x.lane == 0) {
          S.eLP[u.n] = lp;
          S.eMg[u.n] = 0.0;
          S.eInf[u.n] = en_pack(st, t, lv, 0, x.ep);
        }
        u.n += 1;
        summoned = true;
      }
    }
    rp |= (uint32_t)r << (4 * k);
  }
  if (real) *real = rp;
  return (tried && !summoned) ? FC_COST : FC_OK;            // :219-224
}

// ---------------------------------------------------------------------------
// TDBoard.step (TDBoard.py:295-368) + enemy_LP statistics
// ---------------------------------------------------------------------------
// Enemy.defense as the enemy captured it (TDElements.py:33-43)
__device__ __forceinline__ double e_def(const Ctx& x, uint32_t inf) {
  const int t = en_type(inf), lv = en_lv(inf);
  return captured(x, en_ep(inf), [&](const TdDevCfg& c) { return c.e_def[t][lv]; });
}

// Enemies up to which the towers target in parallel (board_step; FEW = false: never --
// the large kernel, where it measured slower, and the two-wave 20x20 single-action
// kernel, which has no registers to spare for it).
constexpr int kFewEnemies = 16;

template <int NC, bool FEW = true>
__device__ __forceinline__ double board_step(Smem<NC>& S, U& u, const Ctx& x, const StepArgs& a, int b) {
  const TdDevCfg& C = x.C;
  const int L = x.L, lane = x.lane;
  double reward = dadd(0.0, C.reward_time);                 // :298-299
  u.steps += 1;                                             // :300
  u.progress = ddiv((double)u.steps, (double)C.max_episode_steps);  // :301

  // --- stable sort by f64 key dist - margin (:305): rank = #smaller + #equal-before
  const int n = u.n;
  double lp[2], mg[2];
  uint32_t inf[2];
  bool val[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int i = lane + 64 * s;
    val[s] = i < n;
    lp[s] = val[s] ? S.eLP[i] : 0.0;
    mg[s] = val[s] ? S.eMg[i] : 0.0;
    inf[s] = val[s] ? S.eInf[i] : 0u;
  }
  if (n > 1) {  // (a list of 0 or 1 enemies is sorted; most boards, most steps)
    double key[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) key[s] = val[s] ? dsub((double)pk_dist(S.cell[en_cell(inf[s])]), mg[s]) : 0.0;
    int rank[2] = {0, 0};
    for (int j = 0; j < n; ++j) {  // enemy j's key from the lane that holds it
      const double kj = j < 64 ? rdl(key[0], j) : rdl(key[1], j - 64);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        int i = lane + 64 * s;
        if (kj < key[s] || (kj == key[s] && j < i)) rank[s] += 1;
      }
    }
    wsync();
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (val[s]) { S.eLP[rank[s]] = lp[s]; S.eMg[rank[s]] = mg[s]; S.eInf[rank[s]] = inf[s]; }
    wsync();
    // lane owns sorted enemies lane and lane + 64
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int i = lane + 64 * s;
      lp[s] = val[s] ? S.eLP[i] : 0.0;
      mg[s] = val[s] ? S.eMg[i] : 0.0;
      inf[s] = val[s] ? S.eInf[i] : 0u;
    }
  }

  // --- towers fire in list order (:306-313); dead enemies stay targetable.
  // Tower k lives in lane k (cool-down in a register); a fired tower is read
  // with a wave-uniform lane index (v_readlane).
  double tcd = lane < u.nt ? S.tCd[lane] : 0.0;
  const uint32_t tinf_l = lane < u.nt ? S.tInf[lane] : 0u;
  if (n == 0) {
    // no enemy anywhere: every tower just cools down (cd -= 1; no target; clamp at 0)
    if (lane < u.nt) { const double cd = dsub(tcd, 1.0); tcd = cd > 0.0 ? cd : 0.0; }
  } else {
    // Targeting never depends on another tower's shot (dead enemies stay targetable), so
    // what the serial loop needs per tower -- range, interval, attack and splash as the
    // tower captured them -- is gathered once, one tower per lane, into the enemy
    // arrays' LDS (dead between the sorted load above and the compaction below): the
    // loop reads it with one uniform-address LDS load per value, no epoch branches.
    double* const tp = S.eLP;  // [TCAP][4]: rge, intv, atk, dmgrge
    static_assert(sizeof(S.eLP) >= TCAP * 4 * sizeof(double), "tower table in the enemy LP array");
    if (lane < u.nt) {
      const int tt = (tinf_l >> 12) & 3, tl = (tinf_l >> 14) & 1, te = tw_eu(tinf_l);
      tp[4 * lane + 0] = captured(x, te, [&](const TdDevCfg& c) { return c.t_rge[tt][tl]; });
      tp[4 * lane + 1] = captured(x, te, [&](const TdDevCfg& c) { return c.t_intv[tt][tl]; });
      tp[4 * lane + 2] = captured(x, te, [&](const TdDevCfg& c) { return c.t_atk[tt][tl]; });
      tp[4 * lane + 3] = captured(x, te, [&](const TdDevCfg& c) { return c.t_dmg[tt][tl]; });
    }
    wsync();
    if (FEW && n <= kFewEnemies) {
      // A few enemies (most boards that have any): the towers pick their targets in
      // parallel, lane k = tower k, each scanning the n enemies in list order; then the
      // shots land in tower order, each enemy (lane j) taking the hits of the towers that
      // fired, one tower after the other -- the reference's order of LP updates per enemy
      // (:306-313), without a dependent LDS round trip per tower.
      const bool tk = lane < u.nt;
      const int tt = (int)((tinf_l >> 12) & 3u), tc = (int)(tinf_l & 0xfffu);
      double cd = dsub(tcd, 1.0);                            // :307
      const bool tries = tk && !(cd > 0.0);
      const double rge = tries ? tp[4 * lane] : -1.0;
      int tgt = -1;
      for (int j = 0; j < n; ++j) {  // first enemy within range (list order)
        const int ec = en_cell(rdl(inf[0], j));
        if (tgt < 0 && (double)cheb(ec, tc, L, x.Lm) <= rge) tgt = j;
      }
      const int tgc = en_cell((uint32_t)__shfl((int)inf[0], tgt < 0 ? 0 : tgt));  // every lane shuffles
      const double dr = tt >= 2 && tgt >= 0 ? tp[4 * lane + 3] : -1.0;
      int frz = -1;  // TowerFrozen: the first enemy within splash of the target (:112-132)
      if (tt == 3)
        for (int j = 0; j < n; ++j) {
          const int ec = en_cell(rdl(inf[0], j));
          if (frz < 0 && (double)cheb(tgc, ec, L, x.Lm) <= dr) frz = j;
        }
      if (tgt >= 0) cd = dadd(cd, tp[4 * lane + 1]);         // cd += intv
      if (tries && cd < 0.0) cd = 0.0;                       // :311-312
      if (tk) tcd = cd;
      const uint32_t slow = (uint32_t)C.frozen_time << 16;   // config.frozen_time, read live (:126)
      for (uint64_t fm = ballot(tgt >= 0); fm; fm &= fm - 1) {  // the towers that fired, in order
        const int k = ctz64(fm);
        const int kt = (int)((rdl(tinf_l, k) >> 12) & 3u);
        const double atk = tp[4 * k + 2];
        if (kt <= 1) {  // TowerArrow / TowerMagic (TDElements.py:71-93)
          if (lane == (int)rdl((uint32_t)tgt, k)) lp[0] = damage(lp[0], atk, e_def(x, inf[0]), kt == 1);
        } else if (kt == 2) {  // TowerBomb splash (:95-110)
          const int kc = (int)rdl((uint32_t)tgc, k);
          if (val[0] && (double)cheb(kc, en_cell(inf[0]), L, x.Lm) <= tp[4 * k + 3])
            lp[0] = damage(lp[0], atk, e_def(x, inf[0]), false);
        } else if (lane == (int)rdl((uint32_t)frz, k)) {
          lp[0] = damage(lp[0], atk, 0.0, true);
          inf[0] = (inf[0] & 0xff00ffffu) | slow;
        }
      }
    } else
    for (int k = 0; k < u.nt; ++k) {
      double cd = dsub(rdl(tcd, k), 1.0);                    // :307
      if (!(cd > 0.0)) {
        const uint32_t ti = rdl(tinf_l, k);
        const int tt = (ti >> 12) & 3, tc = ti & 0xfff;
        const double rge = tp[4 * k];
        bool in0 = val[0] && (double)cheb(en_cell(inf[0]), tc, L, x.Lm) <= rge;
        bool in1 = val[1] && (double)cheb(en_cell(inf[1]), tc, L, x.Lm) <= rge;
        uint64_t m0 = ballot(in0), m1 = ballot(in1);
        if (m0 | m1) {
          const int tgt = m0 ? ctz64(m0) : 64 + ctz64(m1);
          cd = dadd(cd, tp[4 * k + 1]);  // cd += intv
          const double atk = tp[4 * k + 2];
          if (tt <= 1) {  // TowerArrow / TowerMagic (TDElements.py:71-93)
            if (lane == (tgt & 63)) {
              if (tgt < 64) lp[0] = damage(lp[0], atk, e_def(x, inf[0]), tt == 1);
              else lp[1] = damage(lp[1], atk, e_def(x, inf[1]), tt == 1);
            }
          } else {
            const uint32_t tinf = (tgt >> 6) ? rdl(inf[1], tgt & 63) : rdl(inf[0], tgt & 63);
            const int tgc = en_cell(tinf);
            const double dr = tp[4 * k + 3];
            if (tt == 2) {  // TowerBomb splash (:95-110)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                if (val[s] && (double)cheb(tgc, en_cell(inf[s]), L, x.Lm) <= dr)
                  lp[s] = damage(lp[s], atk, e_def(x, inf[s]), false);
            } else {  // TowerFrozen: first enemy within splash of the target (:112-132)
              bool h0 = val[0] && (double)cheb(tgc, en_cell(inf[0]), L, x.Lm) <= dr;
              bool h1 = val[1] && (double)cheb(tgc, en_cell(inf[1]), L, x.Lm) <= dr;
              uint64_t q0 = ballot(h0), q1 = ballot(h1);
              if (q0 | q1) {
                const int f = q0 ? ctz64(q0) : 64 + ctz64(q1);
                if (lane == (f & 63)) {
                  const uint32_t slow = (uint32_t)C.frozen_time << 16;  // config.frozen_time, read live (:126)
                  if (f < 64) { lp[0] = damage(lp[0], atk, 0.0, true); inf[0] = (inf[0] & 0xff00ffffu) | slow; }
                  else { lp[1] = damage(lp[1], atk, 0.0, true); inf[1] = (inf[1] & 0xff00ffffu) | slow; }
                }
              }
            }
          }
        }
        if (cd < 0.0) cd = 0.0;                              // :311-312
      }
      if (lane == k) tcd = cd;
    }
  }
  if (lane < u.nt) S.tCd[lane] = tcd;

  // --- kills (:313-317): every enemy at LP 0 was hit this step
  bool dead0 = val[0] && lp[0] == 0.0, dead1 = val[1] && lp[1] == 0.0;
  const int nk = popc64(ballot(dead0)) + popc64(ballot(dead1));
  reward = dadd(reward, dmul(C.reward_kill, (double)nk));  // :315

  // --- march (:319-344)
  bool alive[2] = {val[0] && !dead0, val[1] && !dead1};
  bool leak[2] = {false, false};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (!alive[s]) continue;
    const uint32_t e = inf[s];
    const int t = en_type(e), lv = en_lv(e);
    int slow = en_slow(e), cell = en_cell(e);
    const double sp = captured(x, en_ep(e), [&](const TdDevCfg& c) { return c.e_speed[t][lv]; });
    if (slow > 0) { mg[s] = dadd(mg[s], dmul(sp, C.frozen_ratio)); slow -= 1; }
    else mg[s] = dadd(mg[s], sp);
    while (mg[s] >= 1.0) {
      mg[s] = dsub(mg[s], 1.0);
      const int d = pk_dir(S.cell[cell]);
      // map[5] codes (TDBoard.py:319): 0:+c 1:-c 2:+r 3:-r
      const int r1 = div_side(cell, x.Lm);
      int r = r1 + (d == 2) - (d == 3), c = cell - r1 * L + (d == 0) - (d == 1);
      if (r < 0 || r >= L || c < 0 || c >= L) { u.flags |= FLAG_BAD_MOVE; break; }
      cell = r * L + c;
      if (cell == u.end_cell) { leak[s] = true; break; }
    }
    inf[s] = en_pack(cell, t, lv, slow, en_ep(e));
  }
  // a bad move is rare and lane-local: fold the flag into the uniform copy
  if (ballot((u.flags & FLAG_BAD_MOVE) != 0)) u.flags |= FLAG_BAD_MOVE;
  const int nl = popc64(ballot(leak[0])) + popc64(ballot(leak[1]));
  for (int p = 0; p < nl; ++p) {                            // :336-343, in list order
    if (u.base_LP > 0) reward = dsub(reward, C.penalty_leak);
    u.base_LP = u.base_LP - 1 > 0 ? u.base_LP - 1 : 0;
  }
  // --- compact survivors, list order kept (:316-317, :345-346)
  bool keep0 = alive[0] && !leak[0], keep1 = alive[1] && !leak[1];
  const uint64_t k0 = ballot(keep0), k1 = ballot(keep1);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int n2 = popc64(k0) + popc64(k1);
  wsync();
  if (keep0) { int d = popc64(k0 & lt); S.eLP[d] = lp[0]; S.eMg[d] = mg[0]; S.eInf[d] = inf[0]; }
  if (keep1) { int d = popc64(k0) + popc64(k1 & lt); S.eLP[d] = lp[1]; S.eMg[d] = mg[1]; S.eInf[d] = inf[1]; }
  u.n = n2;

  // --- costs (:348-353)
  double rate;
  if (u.progress >= 0.5) rate = C.atk_final_rate;
  else rate = dadd(dmul(C.atk_init_rate, dsub(1.0, u.progress)), dmul(C.atk_final_rate, u.progress));
  u.cost_atk = pymin(dadd(u.cost_atk, rate), u.max_cost);  // self.max_cost (:352-353)
  u.cost_def = pymin(dadd(u.cost_def, C.def_rate), u.max_cost);
  wsync();
  return reward;  // the caller writes the enemy list back (store_enemies)
}

// The enemy list after board_step, back to HBM (before enemy_stats reuses its LDS).
template <int NC>
__device__ __forceinline__ void store_enemies(const Smem<NC>& S, const U& u, const Ctx& x, const StepArgs& a, int b) {
  const size_t eb = (size_t)b * ECAP;
  for (int i = x.lane; i < u.n; i += 64) {
    sst(&a.en_lp[eb + i], S.eLP[i]);
    sst(&a.en_mg[eb + i], S.eMg[i]);
    sst(&a.en_inf[eb + i], S.eInf[i]);
  }
}

// enemy_LP planes (TDBoard.py:355-365): per (type, cell) min / max / sum in list
// order / count, all in numpy float32.  The first enemy of each group (its
// "head") walks the list and owns the group's stats.
template <int NC>
__device__ __forceinline__ void enemy_stats(Smem<NC>& S, const U& u, const Ctx& x) {
  const TdDevCfg& C = x.C;
  const int n = u.n;
  if (n == 0) return;  // write_obs emits zero planes without reading grp
  static_assert((4 * NC) % 16 == 0 && offsetof(Smem<NC>, grp) % 16 == 0, "grp cleared in 16-B units");
  for (int i = x.lane; i < 4 * NC / 16; i += 64)
    reinterpret_cast<uint4*>(&S.grp[0][0])[i] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t key[2];
  float r[2] = {0.0f, 0.0f};
  bool val[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int i = x.lane + 64 * s;
    val[s] = i < n;
    key[s] = 0;
    if (val[s]) {
      uint32_t e = S.eInf[i];
      key[s] = e & 0x3fffu;  // cell | type << 12
      const int t = en_type(e), lv = en_lv(e);
      r[s] = f32(ddiv(S.eLP[i], captured(x, en_ep(e), [&](const TdDevCfg& c) { return c.e_lp[t][lv]; })));  // LP / maxLP (:358)
    }
  }
  float mn[2] = {1.0f, 1.0f}, mx[2] = {0.0f, 0.0f}, sm[2] = {0.0f, 0.0f};
  int cnt[2] = {0, 0};
  bool head[2] = {val[0], val[1]};
  for (int j = 0; j < n; ++j) {  // enemy j's group key and ratio from the lane that holds it
    const uint32_t kj = j < 64 ? rdl(key[0], j) : rdl(key[1], j - 64);
    const float rj = j < 64 ? rdl(r[0], j) : rdl(r[1], j - 64);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int i = x.lane + 64 * s;
      if (val[s] && kj == key[s]) {
        if (j < i) head[s] = false;
        else {
          mn[s] = rj < mn[s] ? rj : mn[s];
          mx[s] = rj > mx[s] ? rj : mx[s];
          sm[s] = __fadd_rn(sm[s], rj);
          cnt[s] += 1;
        }
      }
    }
  }
  const float mcl = (float)C.max_cluster_length;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int i = x.lane + 64 * s;
    if (head[s]) {
      S.gst[i][0] = mn[s];
      S.gst[i][1] = mx[s];
      S.gst[i][2] = __fdiv_rn(sm[s], (float)cnt[s]);
      S.gst[i][3] = __fdiv_rn((float)cnt[s], mcl);
      S.grp[key[s] >> 12][key[s] & 0xfffu] = (uint8_t)i;
    }
  }
  wsync();
}

// Channel 9 by distance (per episode): s[9] = map[4] / (max(map[4]) + 1), an
// int32 scalar divisor promotes to f64, rounded once to f32 (TDBoard.py:121).
template <int NC>
__device__ __forceinline__ void d9_table(Smem<NC>& S, int maxdist, int lane) {
  if (lane <= maxdist) S.d9[lane] = f32(ddiv((double)lane, (double)(maxdist + 1)));
}

// Broadcast channels and the channel-9 table (TDBoard.py:115-142).  (The same divisions
// as two uniform passes over all lanes instead of a branch per channel measured slower:
// 219 vs 214 us at 65,536 boards, profiles/r03/s24.)
template <int NC>
__device__ __forceinline__ void channel_scalars(Smem<NC>& S, const U& u, const Ctx& x) {
  const TdDevCfg& C = x.C;
  const int l = x.lane;
  if (l < 48) {
    float v = 0.0f;
    if (l == 5) v = f32(ddiv((double)u.base_LP, (double)u.max_base_LP));
    else if (l == 11) v = f32(ddiv(u.cost_def, u.max_cost));
    else if (l == 12) v = f32(ddiv(u.cost_atk, u.max_cost));
    else if (l == 13) v = f32(u.progress);
    else if (l >= 21 && l < 25) v = (u.cost_def >= C.t_price[l - 21][0]) ? 1.0f : 0.0f;
    else if (l >= 41 && l < 45) v = f32(ddiv(ddiv(u.cost_def, C.e_cost[l - 41][0]), (double)C.max_cluster_length));
    S.chv[l] = v;
  }
  d9_table(S, u.maxdist, l);
  wsync();
}


// Once the step's actions are done (the towers and map[6] are final), the cell words
// are replaced in LDS by what the rest of the step reads of a cell: the binary
// observation bits (cell_bits, bits 0-20), the march direction map[5] (bits 21-22)
// and the distance to the end map[4] (bits 24-31; channel 9 and the sort key).  The
// board's own cell words must have been written back first (store_cells).
template <int NC>
__device__ __forceinline__ void pack_obs_cells(Smem<NC>& S, const Ctx& x) {
  for (int i = x.lane; i < x.NCr; i += 64) {
    const uint32_t w = S.cell[i];
    S.cell[i] = cell_bits(w, twr_of(w)) | ((uint32_t)cw_dir(w) << 21) | ((uint32_t)cw_dist(w) << 24);
  }
  wsync();
}

template <int NC>
__device__ __forceinline__ float obs_value(const Smem<NC>& S, int ch, int cell, bool any_enemy) {
  const uint32_t w = S.cell[cell];  // packed by pack_obs_cells
  switch (obs_kind(ch)) {
    case OK_BIN: return bitf(w, ch);
    case OK_D9: return S.d9[w >> 24];
    case OK_ENEMY: {
      if (!any_enemy) return 0.0f;
      const int e = ch - 25;
      const uint32_t g = S.grp[e & 3][cell];
      return g == 0xFFu ? 0.0f : S.gst[g][e >> 2];
    }
    default: return S.chv[ch];
  }
}

// Observation stores are non-temporal: 1.2 GB per launch written once and never
// read back by the kernel; as plain stores the dirty lines fill the XCD L2s and
// every state load behind them waits on a write-back (measured: 16 % slower).
__device__ __forceinline__ void obs_store(f32x4* p, f32x4 v) { __builtin_nontemporal_store(v, p); }
// The two lines a board shares with its neighbours (written half by this wave, half
// by a wave on another XCD) are stored write-through (sc1) instead: two non-temporal
// partial writes of one line cost ~7 % of the whole stream (scripts/storepol.hip:
// 234 us with nt partial lines, 218 us with sc1 ones = the whole-lines-only bound).
__device__ __forceinline__ void obs_store_shared(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);  // aux 16 = sc1
}

// The (45, L, L) float32 observation of one board.  The wave writes the batch's
// observation stream in 128-B-aligned 1-KB windows: store k covers the 16-B units
// [A + 64k, A + 64k + 64) of the stream, A = the board's first unit rounded down to
// a 128-B line, and lanes outside the board are masked off.  Every line is then
// written whole by one instruction except the two the board shares with its
// neighbours (a board is 18,000 B at L = 10, not a multiple of 128).  Non-temporal
// stores of partial lines run at ~0.85x the rate of whole ones
// (scripts/membench.hip: 4.3 vs 5.0-5.1 TB/s), so the channel-major walk of the
// planes (800-B runs per store) is not line-aligned enough.  Lane unit i of the board
// is channel i / Q, quad i % Q (Q = L*L/4 quads of 4 cells per plane).
template <int NC, int LT>
__device__ __forceinline__ void write_obs(const Smem<NC>& S, const Ctx& x, float* out, bool any_enemy) {
  const int ncr = LT ? LT * LT : x.NCr;
  if ((ncr & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {  // else: caller buffer not 16-B aligned
    const int Q = ncr / 4, n4 = NCH * Q;
    f32x4* o4 = reinterpret_cast<f32x4*>(out);
    const int mis = (int)((reinterpret_cast<uintptr_t>(o4) >> 4) & 7u);  // units of the line before the board
    // units [0, head) and [tail, n4) lie in lines shared with the neighbouring boards
    const int head = mis ? 8 - mis : 0, tail = ((n4 + mis) & ~7) - mis;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o4, 0, n4 * 16, 0x00020000);
    const uint4* cell4 = reinterpret_cast<const uint4*>(S.cell);
    for (int i = x.lane - mis; i < n4; i += 64) {
      if (i < 0) continue;
      const int ch = i / Q, q = i - ch * Q;
      const int kind = obs_kind(ch);
      f32x4 v;
      if (kind == OK_BIN) {
        const uint4 w = cell4[q];
        const uint32_t c = (uint32_t)ch;
        v = f32x4{(float)((w.x >> c) & 1u), (float)((w.y >> c) & 1u), (float)((w.z >> c) & 1u),
                  (float)((w.w >> c) & 1u)};
      } else if (kind == OK_CONST) {
        const float c = S.chv[ch];
        v = f32x4{c, c, c, c};
      } else if (kind == OK_D9) {
        const uint4 w = cell4[q];
        v = f32x4{S.d9[w.x >> 24], S.d9[w.y >> 24], S.d9[w.z >> 24], S.d9[w.w >> 24]};
      } else if (any_enemy) {  // wave-uniform
        const int e = ch - 25, st = e >> 2, t = e & 3;
        const uint32_t g4 = *reinterpret_cast<const uint32_t*>(&S.grp[t][4 * q]);
        const uint32_t g0 = g4 & 0xffu, g1 = (g4 >> 8) & 0xffu, g2 = (g4 >> 16) & 0xffu, g3 = g4 >> 24;
        // branch-free: read a clamped slot, keep it only where the cell has a group
        const float f0 = S.gst[g0 & (ECAP - 1)][st], f1 = S.gst[g1 & (ECAP - 1)][st];
        const float f2 = S.gst[g2 & (ECAP - 1)][st], f3 = S.gst[g3 & (ECAP - 1)][st];
        v = f32x4{g0 != 0xffu ? f0 : 0.0f, g1 != 0xffu ? f1 : 0.0f, g2 != 0xffu ? f2 : 0.0f, g3 != 0xffu ? f3 : 0.0f};
      } else {
        v = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (i < head || i >= tail) obs_store_shared(rs, i * 16, v);
      else obs_store(o4 + i, v);
    }
  } else {
    const int nf = NCH * ncr;
    for (int f = x.lane; f < nf; f += 64) {
      const int ch = f / ncr;
      out[f] = obs_value(S, ch, f - ch * ncr, any_enemy);
    }
  }
}

// The class of every observation window, by the board's misalignment `mis` (units of
// the 128-B line before the board) and window k, as a compile-time table read with one
// scalar load per 8 windows (instead of the window's channel range, channel mask and
// edge test in ~20 SALU per window): bits 0-1 the channel class (0 binary planes only,
// 1 broadcast channels only, 2 enemy planes only, 3 mixed), bit 2 the window holds a
// line shared with a neighbouring board.
template <int LT>
struct ObsWinTab {
  static constexpr int Q = LT * LT / 4, N4 = NCH * Q, K = (N4 + 7 + 63) / 64, W = (K + 7) / 8;
  struct T { uint32_t w[8][W]; };
  static constexpr uint32_t cls(int mis, int k) {
    const int head = mis ? 8 - mis : 0, tail = ((N4 + mis) & ~7) - mis;
    const int ulo = 64 * k - mis, uhi = ulo + 63;
    const int clo = (ulo < 0 ? 0 : ulo) / Q, chi = (uhi > N4 - 1 ? N4 - 1 : uhi) / Q;
    uint64_t chm = 0;
    for (int c = clo; c <= chi; ++c) chm |= 1ull << c;
    chm &= kChAll;
    const uint32_t c = (chm & ~kChBin) == 0 ? 0u : (chm & ~kChConst) == 0 ? 1u : (chm & ~kChEnemy) == 0 ? 2u : 3u;
    return c | ((ulo < head || uhi >= tail) ? 4u : 0u);
  }
  static constexpr T make() {
    T t{};
    for (int m = 0; m < 8; ++m)
      for (int k = 0; k < K; ++k) t.w[m][k / 8] |= cls(m, k) << (4 * (k % 8));
    return t;
  }
  static constexpr T tab = make();
};

// The (45, L, L) float32 observation of one board for compile-time L, into a
// 16-B-aligned buffer: the 128-B-aligned 1-KB windows of write_obs (store k covers
// stream units [A + 64k, A + 64k + 64), A = the board's first unit rounded down to a
// line), software-pipelined.  For G windows at a time every lane first issues its
// two LDS reads -- the 16-B packed cell quad and one word that is the broadcast value
// (chv) or the enemy group quad (grp) -- then the windows are computed and stored.
// The window's channel mix is wave-uniform (SALU): a window of one class takes a
// short path, the per-cell tables (channel 9, enemy stats) are read only where the
// window holds such channels.  Stores are buffer stores whose lanes outside the board
// get an out-of-range offset: the hardware drops them, so no lane is masked off by a
// branch.  wt: every line write-through (sc1) instead of non-temporal, where the
// batch's observation fits the 256-MiB Infinity Cache (scripts/storepol.hip at 8,192
// boards, 147 MB: 21.8 us sc1, 30.0 us nt; at 65,536 boards, 1.18 GB, nt whole lines
// are the fastest form, with the two lines shared with the neighbours sc1).
//
// PASS: 0 every window; 1 only the windows of binary planes alone (ObsWinTab class 0:
// roads, end, starts, buildable, tower level / type -- final once the step's actions
// are, td_step_kernel_small2 writes them early); 2 every other window.
// edge_wt: how the two lines the board shares with its neighbours are stored.  2 (default):
// plain write-back stores -- with the XCD-contiguous board map (StepArgs::xcd_map) the
// neighbours' waves run on this XCD and its L2 merges the two halves into one line write
// (a pair split across two XCDs is written back byte-masked by both L2s); 1: write-through
// (sc1).  2 vs 1 at 65,536 boards: 1.088x vs 1.093x the algorithmic bytes, step time +-0
// (profiles/r04/s20); non-temporal partial lines measured 233 vs 212 us (r04/s4).
template <int NC, int LT, int KB = 0, int KE = -1, int G = 4, int PASS = 0>
__device__ __forceinline__ void write_obs_lines(const Smem<NC>& S, int lane, float* out, bool any_enemy, bool wt,
                                                int edge_wt = 1) {
  static_assert(LT >= 8, "a 128-B line spans at most two channel planes");
  constexpr int Q = LT * LT / 4, N4 = NCH * Q;
  constexpr int K = KE >= 0 ? KE : (N4 + 7 + 63) / 64;  // windows [KB, K) of the board's (N4 + 7 + 63) / 64
  constexpr uint32_t OOB = 0x80000000u;  // beyond the buffer's num_records: store dropped
  const char* const sb = reinterpret_cast<const char*>(&S);
  const int o_cell = (int)(reinterpret_cast<const char*>(S.cell) - sb);  // packed cell words (pack_obs_cells)
  const int o_grp = (int)(reinterpret_cast<const char*>(&S.grp[0][0]) - sb);
  const int o_chv = (int)(reinterpret_cast<const char*>(S.chv) - sb);
  const int o_d9 = (int)(reinterpret_cast<const char*>(S.d9) - sb);
  const int o_gst = (int)(reinterpret_cast<const char*>(&S.gst[0][0]) - sb);
  const int mis = (int)((reinterpret_cast<uintptr_t>(out) >> 4) & 7u);  // units of the line before the board
  const int head = mis ? 8 - mis : 0, tail = ((N4 + mis) & ~7) - mis;   // [0, head), [tail, N4): shared lines
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, N4 * 16, 0x00020000);
  const int i0 = lane - mis;
  typedef Div24<Q, N4 + 64> DivQ;  // unit -> channel (every unit read is in [0, N4))
  // the window's channel class and edge bit (wave-uniform, ObsWinTab)
  auto wclass = [&](int k) { return (ObsWinTab<LT>::tab.w[mis][k >> 3] >> (4 * (k & 7))) & 7u; };
  // only a window at either end of the board holds lanes outside it (i < 0, i >= N4):
  // clamp there, so every lane reads LDS inside the board image
  auto unit = [&](int i, uint32_t wc) { return (wc & 4u) ? (i < 0 ? 0 : (i > N4 - 1 ? N4 - 1 : i)) : i; };
  for (int k0 = KB; k0 < K; k0 += G) {
    uint4 A[G];
    uint32_t W[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int k = k0 + j;
      if ((K - KB) % G == 0 || k < K) {
        const uint32_t wc = wclass(k);
        if (PASS != 0 && (((wc & 3u) == 0) != (PASS == 1))) continue;  // wave-uniform
        const int i = unit(i0 + 64 * k, wc);
        const int ch = DivQ::div(i), q = i - ch * Q;
        A[j] = *reinterpret_cast<const uint4*>(sb + o_cell + 16 * q);
        if ((wc & 3u) == 1) {  // broadcast channels only: the channel's value
          W[j] = *reinterpret_cast<const uint32_t*>(sb + o_chv + 4 * ch);
        } else if ((wc & 3u) >= 2) {
          // enemy plane: the cell quad's group bytes; else the channel's broadcast value
          // (bit select: a ternary here compiled to a divergent branch)
          const int e = ch - 25;
          const int wa = o_grp + (e & 3) * NC + 4 * q, wb = o_chv + 4 * ch, m = -(int)((unsigned)e < 16u);
          const int wo = wb ^ ((wa ^ wb) & m);
          W[j] = *reinterpret_cast<const uint32_t*>(sb + wo);
        } else {
          W[j] = 0u;  // binary planes only: the cell quad is all
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int k = k0 + j;
      if (!((K - KB) % G == 0 || k < K)) continue;
      const uint32_t wc = wclass(k);
      if (PASS != 0 && (((wc & 3u) == 0) != (PASS == 1))) continue;
      const bool edge = (wc & 4u) != 0;  // the window holds a line shared with a neighbour
      const int i = i0 + 64 * k;
      const int ch = DivQ::div(unit(i, wc));
      const int e = ch - 25;
      const bool isen = (unsigned)e < 16u, isd9 = ch == 9, isbin = ((kChBin >> ch) & 1ull) != 0;
      const uint32_t a4[4] = {A[j].x, A[j].y, A[j].z, A[j].w};
      float v[4];
      if ((wc & 3u) == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (float)((a4[c] >> ch) & 1u);
      } else if ((wc & 3u) == 1) {
        const float cv = __uint_as_float(W[j]);
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = cv;
      } else if ((wc & 3u) == 2 && !any_enemy) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = 0.0f;
      } else {
        // a window of several channel kinds: each lane takes its own channel's path
        // (a select over every kind's value measured 1.5 % slower at 8,192 boards)
        if (isbin) {
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = (float)((a4[c] >> (ch & 31)) & 1u);
        } else if (isd9) {  // channel 9 by distance
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const float*>(sb + o_d9 + 4 * (int)(a4[c] >> 24));
        } else if (isen && any_enemy) {  // enemy stats by the cell's group head
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t g = (W[j] >> (8 * c)) & 0xffu;
            const float f = *reinterpret_cast<const float*>(sb + o_gst + 16 * (int)(g & 0x7fu) + 4 * ((e >> 2) & 3));
            v[c] = g != 0xffu ? f : 0.0f;
          }
        } else {
          const float cv = isen ? 0.0f : __uint_as_float(W[j]);
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = cv;
        }
      }
      const f32x4 val = f32x4{v[0], v[1], v[2], v[3]};
      const uint32_t off = (uint32_t)i * 16u;  // i < 0 or i >= N4: out of range already
      if (wt) {  // wave-uniform
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, off, 0, 16 /* sc1 */);
      } else if (!edge) {  // whole lines of this board only
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, off, 0, 2 /* nt */);
      } else {
        const bool shared = i < head || i >= tail;  // a line shared with a neighbouring board
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, shared ? OOB : off, 0, 2 /* nt */);
        if (edge_wt == 2)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, shared ? off : OOB, 0, 0 /* plain */);
        else
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, shared ? off : OOB, 0, 16 /* sc1 */);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// board load / reset / store
// ---------------------------------------------------------------------------
// The inputs of one board step, all loads issued before any is waited on.
// Lane l holds enemy slot l (l < PFE), tower slot l (l < PFT), cells l and l + 64, and one word
// of `w`: lanes 0-23 the header, 24-25 the discrete defender action, 26-37 the
// opponent stream's hot record.
struct Prefetch {
  double lp, mg, tcd;
  uint4 c4;  // cells 4 lane .. 4 lane + 3 (board of L*L % 4 == 0), else cells lane and lane + 64 in .x / .y
  uint32_t inf, tinf, w;
};
// PFE / PFT: enemy / tower slots fetched speculatively with the header (template
// arguments below).  The small-batch kernel (latency-bound) takes 16 of each up front;
// the large-batch kernel (HBM-bound) takes none and loads exactly the live slots once
// the header's counts are in (one dependent round trip, hidden by the other waves).
constexpr int PF_ACT = 24, PF_HOT = 26, PF_SMALL = 16, PF_LARGE = 0;
// (Four enemy slots instead of 16 in TD-def, where 0.02 % of bench.py's steady-state boards
// hold more than 4, read the same bytes -- each slot array's first 128-B line is fetched
// whole either way: PMC 1,534 vs 1,535 B read per board -- in the same time, r06/s5.)
static_assert(offsetof(TdHdr, steps) == 24 && offsetof(TdHdr, start_cell) == 56 && offsetof(TdHdr, episodes) == 76 &&
                  offsetof(TdHdr, max_cost) == 80 && offsetof(TdHdr, max_base_LP) == 88,
              "Prefetch header word map");

template <int PFE, int PFT>
__device__ __forceinline__ void prefetch_issue(Prefetch& P, const StepArgs& a, int b, int lane, int ncr,
                                               bool want_act) {
  const size_t eb = (size_t)b * ECAP, tb = (size_t)b * TCAP, cb = (size_t)b * ncr;
  if (lane < PFE) {  // enemy slots beyond PFE load after the header
    P.lp = a.en_lp[eb + lane];
    P.mg = a.en_mg[eb + lane];
    P.inf = a.en_inf[eb + lane];
  }
  if (lane < PFT) {  // tower slots beyond PFT load after the header
    P.tcd = a.tw_cd[tb + lane];
    P.tinf = a.tw_inf[tb + lane];
  }
  if ((ncr & 3) == 0) {
    P.c4 = lane < (ncr >> 2) ? reinterpret_cast<const uint4*>(a.cells + cb)[lane] : uint4{0u, 0u, 0u, 0u};
  } else {  // (assigned whole: member-wise stores kept P.c4 in scratch in the generic-L build)
    P.c4 = uint4{lane < ncr ? a.cells[cb + lane] : 0u, lane + 64 < ncr ? a.cells[cb + lane + 64] : 0u, 0u, 0u};
  }
  const uint32_t* src;
  if (lane < PF_ACT) src = reinterpret_cast<const uint32_t*>(a.hdr + b) + lane;
  else if (lane < PF_HOT) src = want_act ? reinterpret_cast<const uint32_t*>(a.def_act + b) + (lane - PF_ACT) : nullptr;
  else if (lane < PF_HOT + HOT_WORDS) src = a.opp_hot + (size_t)b * HOT_WORDS + (lane - PF_HOT);
  else src = nullptr;
  P.w = src ? *src : 0u;
}

__device__ __forceinline__ uint32_t lane_word(uint32_t v, int l) { return rdl(v, l); }
// The f64 whose low / high words are held by lanes l / l + 1.
__device__ __forceinline__ double lane_f64(uint32_t v, int l) {
  return __hiloint2double((int)lane_word(v, l + 1), (int)lane_word(v, l));
}

// Commit the prefetched inputs of board b into the LDS image and the scalar state.
template <int NC, int PFE, int PFT>
__device__ __forceinline__ void load_board(Smem<NC>& S, U& u, const Ctx& x, const StepArgs& a, int b, const Prefetch& P) {
  const size_t eb = (size_t)b * ECAP, cb = (size_t)b * x.NCr;
  if ((x.NCr & 3) == 0) {
    // 16-B cell loads: the first 256 cells came with the prefetch, the rest (L > 16)
    // are all issued before any is stored to LDS
    const int n4 = x.NCr >> 2;
    const uint4* g4 = reinterpret_cast<const uint4*>(a.cells + cb);
    uint4* s4 = reinterpret_cast<uint4*>(S.cell);
    constexpr int NR = (NC / 4 + 63) / 64 - 1;  // further 16-B loads per lane: 0 (L <= 16) .. 3 (NC = 1024)
    uint4 r[NR > 0 ? NR : 1];
#pragma unroll
    for (int k = 0; k < NR; ++k) {  // every element assigned (clamped index): the array stays in registers
      const int i = 64 * (k + 1) + x.lane;
      r[k] = g4[i < n4 ? i : n4 - 1];
    }
    if (x.lane < n4) s4[x.lane] = P.c4;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int i = 64 * (k + 1) + x.lane;
      if (i < n4) s4[i] = r[k];
    }
  } else {
    if (x.lane < x.NCr) S.cell[x.lane] = P.c4.x;
    if (x.lane + 64 < x.NCr) S.cell[x.lane + 64] = P.c4.y;
    for (int i = 128 + x.lane; i < x.NCr; i += 64) S.cell[i] = a.cells[cb + i];
  }
  // TdHdr words (td_common.h): 0-5 cost_def, cost_atk, ep_return; 6 steps, 7 base_LP,
  // 8 atk_cd, 9 def_cd, 10 n_en, 11 n_tw, 12 num_roads, 13 end_cell, 14-16 start_cell,
  // 17 maxdist, 18 flags, 19 episodes, 20-21 max_cost, 22 max_base_LP
  u.cost_def = lane_f64(P.w, 0); u.cost_atk = lane_f64(P.w, 2); u.ep_ret = lane_f64(P.w, 4);
  u.steps = (int)lane_word(P.w, 6); u.base_LP = (int)lane_word(P.w, 7);
  u.atk_cd = (int)lane_word(P.w, 8); u.def_cd = (int)lane_word(P.w, 9);
  u.n = (int)lane_word(P.w, 10); u.nt = (int)lane_word(P.w, 11);
  u.num_roads = (int)lane_word(P.w, 12); u.end_cell = (int)lane_word(P.w, 13);
  u.set_starts((int)lane_word(P.w, 14), (int)lane_word(P.w, 15), (int)lane_word(P.w, 16));
  u.maxdist = (int)lane_word(P.w, 17); u.flags = (int)lane_word(P.w, 18); u.episodes = (int)lane_word(P.w, 19);
  if (x.lane == 0) S.flags0 = u.flags;
  u.max_cost = lane_f64(P.w, 20); u.max_base_LP = (int)lane_word(P.w, 22);
  u.progress = ddiv((double)u.steps, (double)x.C.max_episode_steps);
  u.cells_dirty = false;
  u.tw_dirty = false;
  if (x.lane < u.n && x.lane < PFE) { S.eLP[x.lane] = P.lp; S.eMg[x.lane] = P.mg; S.eInf[x.lane] = P.inf; }
  for (int i = PFE + x.lane; i < u.n; i += 64) { S.eLP[i] = a.en_lp[eb + i]; S.eMg[i] = a.en_mg[eb + i]; S.eInf[i] = a.en_inf[eb + i]; }
  uint32_t tinf = P.tinf;
  if (x.lane < u.nt) {
    double tcd = P.tcd;
    if (x.lane >= PFT) {
      const size_t tb = (size_t)b * TCAP;
      tcd = a.tw_cd[tb + x.lane];
      tinf = a.tw_inf[tb + x.lane];
    }
    S.tCd[x.lane] = tcd;
    S.tInf[x.lane] = tinf;
  }
  wsync();
  if (x.lane < u.nt)  // (one tower per cell: no two lanes share a word)
    S.cell[tinf & 0xfffu] |= tw_nib((int)((tinf >> 14) & 1u), (int)((tinf >> 12) & 3u));
  wsync();
}

// Fresh board from a layout record (TDGymBasic.reset :43-53, TDBoard.__init__ :14-79).
template <int NC>
__device__ __forceinline__ void reset_board(Smem<NC>& S, U& u, const Ctx& x, const uint32_t* rec) {
  const TdDevCfg& C = x.C;
  // vector loads only (lane-indexed, then readlane): a record handed over by a
  // concurrently running refill must not come through the scalar cache
  const uint32_t hw = rec[x.lane & (LAYOUT_HDR - 1)];
  for (int i = x.lane; i < x.NCr; i += 64) S.cell[i] = rec[LAYOUT_HDR + i];
  u.num_roads = (int)rdl(hw, 1); u.end_cell = (int)rdl(hw, 2); u.maxdist = (int)rdl(hw, 3);
  u.set_starts(rdl(hw, 4), rdl(hw, 5), rdl(hw, 6));
  u.cost_def = C.def_init_cost; u.cost_atk = C.atk_init_cost;
  u.base_LP = C.base_LP; u.steps = 0; u.progress = 0.0;
  u.max_cost = C.max_cost; u.max_base_LP = C.base_LP;  // TDBoard(max_cost, base_LP) from config at reset
  u.atk_cd = 0; u.def_cd = 0; u.n = 0; u.nt = 0; u.ep_ret = 0.0;
  u.cells_dirty = true;
  u.tw_dirty = true;
  wsync();
}

// Cell words back to HBM when map[6] changed or a new layout was loaded (before
// pack_obs_cells reuses the LDS copy).
template <int NC>
__device__ __forceinline__ void store_cells(const Smem<NC>& S, const U& u, const Ctx& x, const StepArgs& a, int b) {
  const size_t cb = (size_t)b * x.NCr;
  if (u.cells_dirty)
    for (int i = x.lane; i < x.NCr; i += 64) sst(&a.cells[cb + i], S.cell[i] & ~kTwBits);
}

__device__ __forceinline__ TdHdr hdr_of(const U& u) {
  TdHdr h;
  h.cost_def = u.cost_def; h.cost_atk = u.cost_atk; h.ep_return = u.ep_ret;
  h.steps = u.steps; h.base_LP = u.base_LP; h.atk_cd = u.atk_cd; h.def_cd = u.def_cd;
  h.n_en = u.n; h.n_tw = u.nt; h.num_roads = u.num_roads; h.end_cell = u.end_cell;
  h.start_cell[0] = u.start(0); h.start_cell[1] = u.start(1); h.start_cell[2] = u.start(2);
  h.maxdist = u.maxdist; h.flags = u.flags; h.episodes = u.episodes;
  h.max_cost = u.max_cost; h.max_base_LP = u.max_base_LP; h.format = kHdrFormat;
  return h;
}

// The towers' words (cool-downs every step, the rest only when the list changed).
template <int NC>
__device__ __forceinline__ void store_towers(const Smem<NC>& S, int nt, bool dirty, int lane, const StepArgs& a, int b) {
  const size_t tb = (size_t)b * TCAP;
  if (lane < nt) {
    sst(&a.tw_cd[tb + lane], S.tCd[lane]);
    if (dirty) sst(&a.tw_inf[tb + lane], S.tInf[lane]);
  }
}

// The header's second half (words 12-23: layout, flags, episodes, the captured max_cost /
// max_base_LP) changes only at an episode end, a reset or a new flag: a step that did none
// of these stores the first 48 B only (hdr_hi false; -48 B written per board and step).
template <int NC>
__device__ __forceinline__ void store_board(const Smem<NC>& S, const U& u, const Ctx& x, const StepArgs& a, int b,
                                            bool hdr_hi = true) {
  if (x.lane == 0) {
    static_assert(sizeof(TdHdr) == 6 * 16, "header stored as 6 x 16 B");
    const TdHdr h = hdr_of(u);
    const uint4* src = reinterpret_cast<const uint4*>(&h);
    uint4* dst = reinterpret_cast<uint4*>(a.hdr + b);
    dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2];
    if (hdr_hi) { dst[3] = src[3]; dst[4] = src[4]; dst[5] = src[5]; }
  }
  // cells were written back by store_cells, enemies at the end of board_step
  store_towers(S, u.nt, u.tw_dirty, x.lane, a, b);
}

// The per-board outputs of a step (td_step_io) and the board after it: in
// td_step_kernel_small2 the stepping wave hands them to the second wave in LDS, which
// stores them (store_board, store_outputs) while the stepping wave computes the group
// statistics and broadcast channels -- off the board's critical path.
struct alignas(16) StepOut {
  TdHdr hdr;           // the board's header after the step (6 lanes copy it out, 16 B each)
  int32_t nt, tw_dirty;
  double reward, ep_ret;
  int64_t real_def;
  int32_t ep_steps, fail_def;
  uint32_t done, win, allow, cool;
  uint32_t scan_bad;  // second wave, multi-action scan: a flag was not 0 / 1 / 2 (scan_fold)
  uint32_t go;   // second wave: 0 nothing (a board never reset wrote its own outputs), 1 store and write
                 // half of the late windows, 2 store only (an auto-reset board: the stepping wave writes every window)
  uint32_t any;  // the board has enemies (enemy windows read the group statistics)
  uint32_t hdr_hi;  // the header's second half changed (store_board): 6 lanes store it, else 3
};

__device__ __forceinline__ void store_outputs(const StepArgs& a, int b, double reward, double ep_ret, int64_t real_def,
                                              int32_t ep_steps, int32_t fail_def, bool done, int win, uint32_t allow,
                                              uint32_t cool, int lane) {
  if (lane != 0) return;
  sst(&a.reward[b], reward);
  sst(&a.done[b], (uint8_t)(done ? 1 : 0));
  if (a.win) sst(&a.win[b], (int8_t)win);
  if (a.allow_next) sst(&a.allow_next[b], (uint8_t)allow);
  if (a.cooldowns) sst(&a.cooldowns[b], (uint8_t)cool);
  if (a.fail_def) sst(&a.fail_def[b], fail_def);
  if (a.real_def && !a.multi) sst(&a.real_def[b], real_def);
  if (a.ep_return) sst(&a.ep_return[b], ep_ret);
  if (a.ep_len) sst(&a.ep_len[b], ep_steps);
  if (done && a.last_ep) {  // the board's last finished episode (td_episode_records)
    td_episode_record r;
    r.ret = ep_ret;
    r.length = ep_steps;
    r.win = win;
    a.last_ep[b] = r;
  }
  if (done && a.ep_stats) {  // device-side episode accounting (SURVEY §8(b) td_episode_stats)
    atomicAdd(&a.ep_stats[0], 1.0);
    atomicAdd(&a.ep_stats[1], ep_ret);
  }
}
__device__ __forceinline__ void store_outputs(const StepArgs& a, int b, const StepOut& o, int lane) {
  store_outputs(a, b, o.reward, o.ep_ret, o.real_def, o.ep_steps, o.fail_def, o.done != 0u, (int)(int32_t)o.win, o.allow,
                o.cool, lane);
}

// ---------------------------------------------------------------------------
// built-in opponents
// ---------------------------------------------------------------------------
template <int NC, class Rng>
__device__ __forceinline__ void opponent_enemy(Smem<NC>& S, U& u, const Ctx& x, Rng& R, int difficulty) {
  // random_enemy_lv0 / lv1 (TDGymBasic.py:81-108)
  if (u.atk_cd != 0) return;
  uint32_t types = 0;
  int road;
  if (difficulty == 0) {
    for (int k = 0; k < 8; ++k) types |= (uint32_t)R.slot(4) << (4 * k);
    road = (int)R.ri(0, u.num_roads - 1);
  } else {
    const uint32_t t = (uint32_t)R.ri(0, 3);
    road = (int)R.ri(0, u.num_roads - 1);
    types = t * 0x11111111u;
  }
  summon_cluster(S, u, x, types, road, nullptr);
  wsync();
  u.atk_cd = x.C.atk_interval;  // the (ok, real) tuple is always truthy
}

template <int NC, class Rng>
__device__ __forceinline__ void opponent_tower_lv0(Smem<NC>& S, U& u, const Ctx& x, Rng& R) {
  // random_tower_lv0 (TDGymBasic.py:111-122)
  if (u.def_cd != 0) return;
  int r = (int)R.ri(0, x.L - 1);
  int c = (int)R.ri(0, x.L - 1);
  int t = (int)R.ri(0, 3);
  if (tower_build(S, u, x, t, r * x.L + c) == FC_OK) u.def_cd = x.C.def_interval;
}

// random_tower_lv1 / lv2 (TDGymBasic.py:124-292).
template <int NC, class Rng>
__device__ __forceinline__ void build_near_road(Smem<NC>& S, U& u, const Ctx& x, Rng& R, int t, bool draw_type) {
  // road cells in row-major order, then random.shuffle (Fisher-Yates on randbelow)
  // The list lives in the sort-key scratch as cell indices (<= L*L <= 4096 > 4*ECAP,
  // so it is kept in the group map instead: grp has 4*NC bytes -> store u16 cells).
  uint16_t* cells = reinterpret_cast<uint16_t*>(&S.grp[0][0]);
  int nroad = 0;
  for (int base = 0; base < x.NCr; base += 64) {
    int c = base + x.lane;
    bool isr = c < x.NCr && (S.cell[c] & 1u);
    uint64_t m = ballot(isr);
    const uint64_t lt = (x.lane == 0) ? 0ull : (~0ull >> (64 - x.lane));
    if (isr) cells[nroad + popc64(m & lt)] = (uint16_t)c;
    nroad += popc64(m);
  }
  wsync();
  for (int i = nroad - 1; i >= 1; --i) {
    int j = (int)R.shuffle_j(i);
    if (x.lane == 0) { uint16_t tmp = cells[i]; cells[i] = cells[j]; cells[j] = tmp; }
    wsync();
  }
  if (draw_type) t = (int)R.ri(0, 3);
  for (int i = 0; i < nroad; ++i) {
    int k = (int)R.ri(0, 24);
    int dr = k / 5 - 2, dc = k % 5 - 2;
    int cc = cells[i];
    const int rc = div_side(cc, x.Lm);
    int r = rc + dr, c = cc - rc * x.L + dc;
    if (r < 0 || r >= x.L || c < 0 || c >= x.L) continue;
    int fc = tower_build(S, u, x, t, r * x.L + c);
    if (fc == FC_OK) { u.def_cd = x.C.def_interval; return; }
    if (fc == FC_COST) return;
  }
}

template <int NC, class Rng>
__device__ __forceinline__ void upgrade_or_destruct(Smem<NC>& S, U& u, const Ctx& x, Rng& R, int act) {
  if (u.nt == 0) return;
  if (act == 1) {
    int id = (int)R.ri(0, u.nt - 1);
    int cell = (int)(S.tInf[id] & 0xfffu);
    if (tower_lvup(S, u, x, cell) == FC_OK) u.def_cd = x.C.def_interval;
  } else {
    if (R.rnd() > 0.01) return;
    int id = (int)R.py.randint(0, u.nt - 1);  // CPython random whatever random_agent is (:187, :191)
    int cell = (int)(S.tInf[id] & 0xfffu);
    if (tower_destruct(S, u, x, cell) == FC_OK) u.def_cd = x.C.def_interval;
  }
}

template <int NC, class Rng>
__device__ __forceinline__ void opponent_tower(Smem<NC>& S, U& u, const Ctx& x, Rng& R, int difficulty) {
  if (difficulty == 0) { opponent_tower_lv0(S, u, x, R); return; }
  if (u.def_cd != 0) return;
  int act = (int)R.ri(0, 2);
  if (act != 0) { upgrade_or_destruct(S, u, x, R, act); return; }
  if (difficulty == 1) { build_near_road(S, u, x, R, 0, true); return; }
  // lv2: tower type from the enemy type mix (TDGymBasic.py:217-240)
  if (u.n == 0) return;
  int cnt[4] = {0, 0, 0, 0};
  for (int i = 0; i < u.n; ++i) cnt[en_type(S.eInf[i])] += 1;
  // np.unique -> present types ascending; ratio = nums.astype(float32) / np.sum(nums):
  // float32 array / int64 scalar promotes to float64 (NEP 50), so the ratio is an f64 quotient
  int types[4], nt = 0;
  for (int t = 0; t < 4; ++t) if (cnt[t]) types[nt++] = t;
  double p = R.rnd();
  int chosen = -1;
  for (int i = 0; i < 4; ++i) {
    if (i >= nt) { u.flags |= FLAG_BAD_ACTION; break; }  // the reference raises IndexError here
    double ratio = ddiv((double)cnt[types[i]], (double)u.n);
    if (p < ratio) { chosen = types[i]; break; }
    p = dsub(p, ratio);
  }
  if (chosen < 0) return;
  const int remap[4] = {2, 0, 1, 0};
  int t = remap[chosen];
  if (R.rnd() < 0.2) t = 3;
  build_near_road(S, u, x, R, t, false);
}

// Attacker clusters of TD-atk (TDAttack.py:36-46) and TD-2p (TDMulti.py:199-206, 229-241).
template <int NC, int MODE>
__device__ __forceinline__ void attacker_actions(Smem<NC>& S, U& u, const Ctx& x, const StepArgs& a, int b) {
  const TdDevCfg& C = x.C;
  if (x.lane < 24) {
    int64_t v = a.atk_act[(size_t)b * 24 + x.lane];
    const bool bad = v < 0 || v > 4;
    S.atk[x.lane] = bad ? 4 : (int)v;
    S.real_atk[x.lane] = bad ? 4 : (int)v;
  }
  if (x.lane < 4) S.fail_atk[x.lane] = -1;
  {
    bool bad = false;
    if (x.lane < 24) { int64_t v = a.atk_act[(size_t)b * 24 + x.lane]; bad = v < 0 || v > 4; }
    if (ballot(bad)) u.flags |= FLAG_BAD_ACTION;
  }
  wsync();
  if (u.atk_cd != 0) return;
  for (int i = 0; i < u.num_roads; ++i) {
    uint32_t cl = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) cl |= (uint32_t)S.atk[8 * i + k] << (4 * k);
    const bool all4 = cl == 0x44444444u;
    uint32_t real = cl;
    if (MODE == MODE_2P && a.multi) {  // TDMulti multi: every road, always truthy (:201-206)
      summon_cluster(S, u, x, cl, i, &real);
      u.atk_cd = C.atk_interval;
    } else if (all4) {
      if (x.lane == 0) S.fail_atk[i] = 0;               // TDAttack.py:40-42, TDMulti.py:234-236
    } else {
      const int fc = summon_cluster(S, u, x, cl, i, &real);
      if (MODE == MODE_ATK) {
        if (fc == FC_OK) u.atk_cd = C.atk_interval;     // res is a real bool here (TDAttack.py:43-44)
        if (x.lane < 8) S.real_atk[8 * i + x.lane] = (int)((real >> (4 * x.lane)) & 0xfu);
      } else {
        u.atk_cd = C.atk_interval;                      // tuple truthiness (TDMulti.py:237-238)
      }
      if (x.lane == 0) S.fail_atk[i] = fc;
    }
    wsync();
  }
}


// SCAN: the multi-action defender scan is compiled in (launched only when a.multi).
// Its 16-B staging buffers raise the 30x30 kernel from 55 to 148 VGPRs, and the
// discrete kernel should not pay for them in occupancy.
// SMALL: the batch runs as one round of waves (td_step_kernel_small); with a.obs_wt
// the observation lines are stored write-through (write_obs_lines).  (Storing the
// layout and tower planes at the start of the step, before the step logic, was
// measured slower at 4,096 and 8,192 boards: 36.3 / 53.1 vs 25.7 / 38.3 us.)

// Observation windows written by the stepping wave of a two-wave board (the first half).
template <int LT>
__host__ __device__ constexpr int obs_half() { return ((NCH * LT * LT / 4 + 7 + 63) / 64 + 1) / 2; }
// After the second wave's early pass over the binary-plane windows: the first window of
// the second wave's share of the rest, so both waves write half of the remaining
// windows (counted at a line-aligned board; ObsWinTab class != 0).
template <int LT>
constexpr int obs_late_half() {
  constexpr int K = (NCH * LT * LT / 4 + 7 + 63) / 64;
  int late = 0;
  for (int k = 0; k < K; ++k) late += (ObsWinTab<LT>::cls(0, k) & 3u) != 0u;
  int seen = 0;
  for (int k = 0; k < K; ++k) {
    if (2 * seen >= late) return k;
    seen += (ObsWinTab<LT>::cls(0, k) & 3u) != 0u;
  }
  return K;
}

// SPLIT: the board's workgroup has a second wave (td_step_kernel_small2) that waits at
// the one workgroup barrier of this path and then writes the second half of the
// observation windows.
template <int NC, int LT, int MODE, bool SCAN, bool SMALL, bool SPLIT = false>
__device__ __forceinline__ void step_board(Smem<NC>& S, const Ctx& x, const StepArgs& a, int b, const Prefetch& P,
                                           StepOut* so = nullptr) {
  const TdDevCfg& C = x.C;
  uint32_t* const opp = a.opp_mt + (size_t)b * OPP_WORDS;
  uint32_t* const hot = a.opp_hot + (size_t)b * HOT_WORDS;
  U u;
  constexpr int PF = SMALL ? PF_SMALL : PF_LARGE;
  load_board<NC, PF, PF>(S, u, x, a, b, P);
  const int64_t act_in = (int64_t)(((uint64_t)lane_word(P.w, PF_ACT + 1) << 32) | lane_word(P.w, PF_ACT));
  // built-in opponent stream: position, lazy-twist boundary and the next draws
  // (pre-computed by the previous step) come from the board's hot record
  WaveMt R{opp, lane_word(P.w, PF_HOT + 0), lane_word(P.w, PF_HOT + 1)};
  // The large kernel refills the pre-drawn outputs only when they run short (lazy); the
  // small kernels (no SGPR to spare at 8 waves per SIMD) refill every step and use a cache
  // only if it starts at the current position.
  constexpr bool LAZY_HOT = !SMALL;
  if constexpr (LAZY_HOT) {
    R.cn = lane_word(P.w, PF_HOT + 2);
    R.cbase = lane_word(P.w, PF_HOT + 3);
  } else {
    R.cn = lane_word(P.w, PF_HOT + 3) == R.pos ? lane_word(P.w, PF_HOT + 2) : 0u;
    R.cbase = R.pos;
  }
  R.cache = __shfl(P.w, PF_HOT + 4 + (x.lane < HOT_CACHE ? x.lane : 0));
  // (the early window in the large kernel too: +-0, reads +29 B per board, r04/s18)
  constexpr bool EARLY_MT = SMALL && !SCAN && MODE != MODE_2P;
  if constexpr (EARLY_MT) R.early_issue(x.lane);
  constexpr bool SCAN2 = SPLIT && SCAN;
  if (u.num_roads < 1 || u.num_roads > 3) {
    // never reset (its road generation failed): nothing to step
    const int nf = NCH * x.NCr;
    float* o = a.obs + (size_t)b * nf;
    for (int i = x.lane; i < nf; i += 64) o[i] = 0.0f;
    if (x.lane == 0) {  // every output defined: done, no reward, no action taken
      a.hdr[b].flags = u.flags | FLAG_NO_LAYOUT;
      a.reward[b] = 0.0;
      a.done[b] = 1;
      if (a.win) a.win[b] = -1;
      if (a.allow_next) a.allow_next[b] = 0;
      if (a.cooldowns) a.cooldowns[b] = 0;
      if (a.fail_def) a.fail_def[b] = 0;
      if (a.real_def && !a.multi) a.real_def[b] = (int64_t)6 * x.NCr;
      if (a.ep_return) a.ep_return[b] = 0.0;
      if (a.ep_len) a.ep_len[b] = 0;
    }
    if (a.real_def && a.multi)
      for (int i = x.lane; i < 6 * x.NCr; i += 64) a.real_def[(size_t)b * 6 * x.NCr + i] = 0;
    if (a.fail_atk && x.lane < 3) a.fail_atk[(size_t)b * 3 + x.lane] = -1;
    if (a.real_atk && x.lane < 24) a.real_atk[(size_t)b * 24 + x.lane] = 4;
    if constexpr (SPLIT) {
      if (x.lane == 0) { S.early_go = 0u; so->go = 0u; }
      if constexpr (SCAN2) __syncthreads();  // (A0)
      __syncthreads();  // (A)
      __syncthreads();  // (B)
      __syncthreads();  // (C)
    }
    return;
  }
  float* const obs = a.obs + (size_t)b * NCH * x.NCr;
  const bool wt = a.obs_wt != 0;

  u.atk_cd = u.atk_cd - 1 > 0 ? u.atk_cd - 1 : 0;
  u.def_cd = u.def_cd - 1 > 0 ? u.def_cd - 1 : 0;
  const int64_t empty_def = (int64_t)6 * x.NCr;
  int fail_def = 0;
  int64_t real_def = empty_def;

  // ---- defender
  if (MODE != MODE_ATK) {
    if constexpr (SCAN2) {
      __syncthreads();  // (A0) the second wave has folded the flags
      defender_scan<NC, false, false>(S, u, x, nullptr, nullptr, u.def_cd == 0, so->scan_bad != 0u);
    } else if (SCAN) {
      defender_scan(S, u, x, a.def_act + (size_t)b * 6 * x.NCr,
                    a.real_def ? a.real_def + (size_t)b * 6 * x.NCr : nullptr, u.def_cd == 0);
    } else {
      int64_t act = act_in;
      if (act < 0 || act > empty_def) { u.flags |= FLAG_BAD_ACTION; act = empty_def; }
      if (u.def_cd == 0 && act != empty_def) {
        // op = act // L^2, row = (act // L) % L, column = act % L (TDDefense.py:65-67)
        const int a32 = (int)act, ncr = LT ? LT * LT : x.NCr;
        const int op = a32 / ncr;
        fail_def = defender_op(S, u, x, op, a32 - op * ncr);
        if (fail_def == FC_OK) { u.def_cd = C.def_interval; real_def = act; }
      }
    }
  }
  // ---- attacker
  if (MODE == MODE_DEF) {
    with_opp_rng(a, b, x.lane, R, [&](auto& G) { opponent_enemy(S, u, x, G, a.difficulty); });
  } else {
    attacker_actions<NC, MODE>(S, u, x, a, b);
    // info of the attacker now: its LDS arrays share space with the observation tables
    if (a.fail_atk && x.lane < 3) a.fail_atk[(size_t)b * 3 + x.lane] = S.fail_atk[x.lane];
    if (a.real_atk && x.lane < 24) a.real_atk[(size_t)b * 24 + x.lane] = S.real_atk[x.lane];
    if (MODE == MODE_ATK)
      with_opp_rng(a, b, x.lane, R, [&](auto& G) { opponent_tower(S, u, x, G, a.difficulty); });
  }
  // the towers and map[6] are final: cell words back to HBM if they changed, then
  // packed for the rest of the step (board_step reads the packed direction and distance)
  store_cells(S, u, x, a, b);
  u.cells_dirty = false;
  pack_obs_cells(S, x);
  // pre-draw the next step's words: loads issued now, consumed at the end of the step
  // (the step's draws are done: refill the pre-drawn outputs if the next step may run short)
  const bool refill = MODE != MODE_2P && (EARLY_MT || !LAZY_HOT || R.cached_left() < (uint32_t)HOT_REFILL);
  // (the multi-action kernels have no registers to carry the loads across the step: at once)
  if (refill && !EARLY_MT) {
    if constexpr (SCAN) R.prefetch(x.lane);
    else R.prefetch_issue(x.lane);
  }
  wsync();
  if constexpr (SPLIT) {  // (A): the second wave writes the binary-plane windows while this one steps
    if (x.lane == 0) S.early_go = 1u;
    __syncthreads();
  }

  // ---- TDBoard.step
  // (parallel targeting: +1.1-1.4 % at 8,192 / 4,096 boards, -0.7 % in the large kernel at 65,536, profiles/r03/s29)
  double reward = board_step<NC, SMALL && !(SPLIT && LT == 20 && MODE == MODE_DEF && !SCAN)>(S, u, x, a, b);
  // The next step's opponent words, loaded since the attacker phase, are consumed here,
  // before this step's state stores: gfx950 counts loads and stores in one vmcnt, so
  // after the stores the wait for these loads became a wait for every store's
  // acknowledgement (s_waitcnt vmcnt(0)).  (Holding every state store back to the end
  // of the step, next to the observation, measured slower: 219 vs 216 us at 65,536
  // boards, 35.8 vs 34.9 at 8,192, profiles/r03/s16.)
  // (consumed here rather than before the board step: 8,192 boards 32.6-32.7 vs 33.2-33.3 us, r04/s13)
  if constexpr (EARLY_MT) {
    R.early_finish(x.lane);
  } else if (!SCAN && refill) R.prefetch_finish(x.lane);
  if (MODE == MODE_ATK) reward = -reward;                   // TDAttack.py:50
  const bool done = (u.base_LP <= 0) || (u.steps >= C.max_episode_steps);  // :384-385
  u.ep_ret = dadd(u.ep_ret, reward);
  const int ep_steps = u.steps;
  int8_t win = -1;
  if (done) {
    if (MODE == MODE_ATK) win = u.base_LP <= 0 ? 1 : 0;
    else win = u.base_LP > 0 ? 1 : 0;
  }
  // info['AllowNextMove'] (bits 0-1), and the env's attacker_cd / defender_cd attributes
  // after the step, saturated at 15 (td_step_io.cooldowns)
  const uint8_t allow = (uint8_t)((u.atk_cd <= 1 ? 1 : 0) | (u.def_cd <= 1 ? 2 : 0));
  const int acd = u.atk_cd < 15 ? u.atk_cd : 15, dcd = u.def_cd < 15 ? u.def_cd : 15;
  const uint8_t cool = (uint8_t)(acd | (dcd << 4));
  const double ep_ret = u.ep_ret;

  if (done) u.episodes += 1;
  bool was_reset = false;
  uint32_t lay_head = 0;
  if (done && a.autoreset && !a.opp_np) {  // random_agent=False: td_autoreset_kernel follows
    // consume staged layout number lay_head, published by a refill kernel on a side
    // stream while this grid may be running: relaxed sc1 poll of its tag, then one
    // agent-scope acquire before the plain vector loads of the record
    // (MI355X_MICROARCH.md § visibility, "Valid forms"; producer side: wave_layout)
    lay_head = a.lay_head[b];
    const uint32_t* rec = a.nxt + ((size_t)b * NSLOT + lay_head % NSLOT) * a.slot_words;
    const uint32_t want = slot_tag(lay_head);
    bool ready = ld_relaxed(rec) == want;
    // a dry ring: wait for the refill drawing this layout, or draw it now
    if (!ready) ready = take_dry_ring(a, b, lay_head, &u.flags);
    if (ready) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      reset_board(S, u, x, rec);
      was_reset = true;
    } else {
      u.flags |= FLAG_NO_LAYOUT;  // 65 failing draws in a row (the reference raises): the board keeps its finished episode
    }
  }
  // The enemy list back to HBM (after the layout poll's loads, whose wait would
  // otherwise wait for these stores too; a reset board has none).
  store_enemies(S, u, x, a, b);
  if constexpr (SPLIT) {
    // the new episode's layout first (the second wave stores the board next)
    if (was_reset) {
      store_cells(S, u, x, a, b);
      pack_obs_cells(S, x);
    }
  }
  if (x.lane == 0) {
    if (was_reset)  // the record has been read into LDS: its slot may be redrawn
      st_relaxed(a.lay_head + b, lay_head + 1u);
    sst(&hot[0], R.pos);
    sst(&hot[1], R.tw);
    sst(&hot[2], R.cn);
    sst(&hot[3], R.cbase);
  }
  if (refill && x.lane < HOT_CACHE) sst(&hot[4 + x.lane], R.cache);
  if constexpr (SPLIT) {
    // (B) the second wave's early pass has landed; it takes the board and the outputs
    // and stores them while this wave computes the statistics and broadcast channels;
    // (C) both are in LDS: each wave writes half of the windows the early pass left -- a
    // board that auto-reset this step has a new layout, and this wave rewrites every window.
    if (x.lane == 0) {  // field by field: no second register copy of the board
      so->hdr = hdr_of(u);
      so->nt = u.nt; so->tw_dirty = u.tw_dirty ? 1 : 0;
      so->reward = reward; so->ep_ret = ep_ret; so->real_def = real_def;
      so->ep_steps = ep_steps; so->fail_def = fail_def;
      so->done = done ? 1u : 0u; so->win = (uint32_t)(int32_t)win; so->allow = allow; so->cool = cool;
      so->go = was_reset ? 2u : 1u; so->any = u.n > 0 ? 1u : 0u;
      so->hdr_hi = (was_reset || done || u.flags != S.flags0) ? 1u : 0u;
    }
    __syncthreads();
    enemy_stats(S, u, x);  // no-op for a board without enemies (e.g. just reset)
    channel_scalars(S, u, x);
    __syncthreads();
    if (was_reset) write_obs_lines<NC, LT>(S, x.lane, obs, u.n > 0, wt, a.edge_wt);
    else write_obs_lines<NC, LT, 0, obs_late_half<LT>(), 4, 2>(S, x.lane, obs, u.n > 0, wt, a.edge_wt);
  } else {
    enemy_stats(S, u, x);  // no-op for a board without enemies (e.g. just reset)
    channel_scalars(S, u, x);
    if (was_reset) {  // the new episode's layout
      store_cells(S, u, x, a, b);
      pack_obs_cells(S, x);
    }
    store_board(S, u, x, a, b, was_reset || done || u.flags != S.flags0);
    store_outputs(a, b, reward, ep_ret, real_def, ep_steps, fail_def, done, win, allow, cool, x.lane);
    // the observation last: nothing of the step is live any more, the writer has the registers
    if constexpr (LT != 0) {
      if ((reinterpret_cast<uintptr_t>(a.obs) & 15u) == 0) {
        write_obs_lines<NC, LT>(S, x.lane, obs, u.n > 0, wt, a.edge_wt);
      } else {
        write_obs<NC, LT>(S, x, obs, u.n > 0);
      }
    } else {
      write_obs<NC, LT>(S, x, obs, u.n > 0);
    }
  }
}

// One workgroup (one wave) per board.  (A persistent variant that prefetched the
// next board while stepping the current one measured slower: its static board
// assignment leaves a one-board tail, and the step is bound by HBM writes.)
// The kernel arguments a step needs before its board's loads go out, read together at the
// top: read where each is used they were six dependent scalar loads, each waited for, in
// front of every board's first load.
__device__ __forceinline__ void prologue_args(const StepArgs& a) {
  asm volatile("" ::"s"(a.B), "s"(a.xcd_map), "s"(a.multi), "s"(a.cfg), "s"(a.hdr), "s"(a.en_lp), "s"(a.en_mg),
               "s"(a.en_inf), "s"(a.tw_cd), "s"(a.tw_inf), "s"(a.cells), "s"(a.opp_hot), "s"(a.def_act));
}

template <int LT, int MODE, bool SCAN, bool SMALL>
__device__ __forceinline__ void step_kernel_body(const StepArgs& a) {
  constexpr int NC = LT ? LT * LT : MAX_KERNEL_L * MAX_KERNEL_L;
  __shared__ Smem<NC> S;
  const int i = (int)blockIdx.x;
  prologue_args(a);
  if (i >= a.B) return;
  const int b = a.xcd_map ? xcd_board(i, a.B) : i;
  const int L = LT ? LT : a.L;
  const Ctx x{S.cfg, L, L * L, (int)(threadIdx.x & 63), a.cfgs, a.epoch};
  const uint4 cfgv = load_cfg(a.cfg, x.lane);
  Prefetch P;
  constexpr int PF = SMALL ? PF_SMALL : PF_LARGE;
  prefetch_issue<PF, PF>(P, a, b, x.lane, x.NCr, MODE != MODE_ATK && !a.multi);
  store_cfg(S, cfgv, x.lane);  // (its load issued first: this wait leaves the board's loads in flight)
  wsync();  // every lane reads the block: no LDS access may move above its store
  step_board<NC, LT, MODE, SCAN, SMALL>(S, x, a, b, P);
}

// Large batches (several rounds of waves, HBM-write bound): 6 waves per SIMD at
// L = 10 (106 SGPRs), no register pressure beyond the step's own.
template <int LT, int MODE, bool SCAN>
__global__ __launch_bounds__(64) void td_step_kernel(StepArgs a) {
  step_kernel_body<LT, MODE, SCAN, false>(a);  // by value (see kargs)
}

// Batches that fit one round of waves.  8 waves per SIMD where LDS allows it (L = 10:
// 5,072 B per board): the compiler then keeps the kernel at <= 80 SGPRs, the gfx950
// limit for 8 resident waves (MI355X_MICROARCH.md, residency), so 8,192 boards -- 8
// GPUs' share of BASELINE's 65,536 -- run as ONE round instead of 6,144 + 2,048.  At
// 65,536 boards the same build is 7 % slower (SGPR spill code), hence two kernels.
// The two-wave 20x20 TD-atk kernel does not fit 64 VGPRs: at 8 waves per SIMD it spilled
// (8 B of scratch per lane), so 6.  (The multi-action scan kernels ran at 5 until the
// flag fold's loop was kept rolled, scan_fold.)
template <int LT, int MODE, bool SCAN>
constexpr int small2_cap() { return LT == 20 && MODE == MODE_ATK && !SCAN ? 6 : 8; }
#define TD_SMALL_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#define TD_SMALL2_ATTR __attribute__((amdgpu_waves_per_eu(small2_cap<LT, MODE, SCAN>(), small2_cap<LT, MODE, SCAN>())))
template <int LT, int MODE, bool SCAN>
__global__ __launch_bounds__(64) TD_SMALL_ATTR void td_step_kernel_small(StepArgs a) {
  step_kernel_body<LT, MODE, SCAN, true>(kargs(a));
}

// Batches up to half the resident waves: two waves per board.  The first steps the board
// as in td_step_kernel_small; the second waits at one barrier and writes the second half
// of the observation windows beside it, which shortens a board's critical path where the
// batch leaves issue slots free (4,096 boards: 8,192 waves, 8 per SIMD).
template <int LT, int MODE, bool SCAN>
__global__ __launch_bounds__(128) TD_SMALL2_ATTR void td_step_kernel_small2(StepArgs a_) {
  const StepArgs& a = kargs(a_);
  constexpr int NC = LT * LT;
  __shared__ Smem<NC> S;
  __shared__ StepOut SO;
  prologue_args(a);
  if ((int)blockIdx.x >= a.B) return;
  const int b = a.xcd_map ? xcd_board((int)blockIdx.x, a.B) : (int)blockIdx.x;
  const int lane = (int)threadIdx.x & 63;
  if (threadIdx.x < 64) {
    const Ctx x{S.cfg, LT, NC, lane, a.cfgs, a.epoch};
    const uint4 cfgv = load_cfg(a.cfg, lane);
    Prefetch P;
    prefetch_issue<PF_SMALL, PF_SMALL>(P, a, b, lane, NC, MODE != MODE_ATK && !a.multi);
    store_cfg(S, cfgv, lane);  // (see load_cfg)
    wsync();  // every lane reads the block: no LDS access may move above its store
    step_board<NC, LT, MODE, SCAN, true, true>(S, x, a, b, P, &SO);
  } else {
    float* const obs = a.obs + (size_t)b * NCH * NC;
    constexpr bool SCAN2 = SCAN;
    if constexpr (SCAN2) {  // the multi-action flags, folded while the first wave loads the board
      const bool bad = scan_fold(S, lane, NC, a.def_act + (size_t)b * 6 * NC);
      if (lane == 0) SO.scan_bad = bad ? 1u : 0u;
      __syncthreads();  // (A0)
    }
    __syncthreads();  // (A) actions and towers final, cells packed
    if constexpr (SCAN2) {  // the real actions, beside the step (grp[1] is not touched before (B))
      if (S.early_go && a.real_def) scan_write_real(S, lane, NC, a.real_def + (size_t)b * 6 * NC);
    }
    if (S.early_go) {
      write_obs_lines<NC, LT, 0, -1, 4, 1>(S, lane, obs, false, a.obs_wt != 0, a.edge_wt);
      // landed before (B): after an auto-reset the first wave rewrites these windows
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // (B) the board after the step and its outputs are in SO
    const uint32_t go = SO.go;
    if (go) {
      static_assert(sizeof(TdHdr) == 6 * 16 && offsetof(StepOut, hdr) == 0 && alignof(StepOut) >= 16,
                    "header copied as 6 x 16-B LDS reads");
      if (lane < (SO.hdr_hi ? 6 : 3)) reinterpret_cast<uint4*>(a.hdr + b)[lane] = reinterpret_cast<const uint4*>(&SO.hdr)[lane];
      store_towers(S, SO.nt, SO.tw_dirty != 0, lane, a, b);
      store_outputs(a, b, SO, lane);
    }
    __syncthreads();  // (C) statistics and broadcast channels in LDS
    if (go == 1u)
      write_obs_lines<NC, LT, obs_late_half<LT>(), -1, 4, 2>(S, lane, obs, SO.any != 0u, a.obs_wt != 0,
                                                            a.edge_wt);
  }
}

// The built-in opponents called on their own, between steps (TDGymBasic.py:81-292,
// called directly by demo.py:78-79): random_enemy_lv{0,1} (side 0) or
// random_tower_lv{0,1,2} (side 1) for every masked board, on the board's opponent
// stream, with the reference's cool-down check and update.  No observation.
template <int LT>
__global__ __launch_bounds__(64) void td_opponent_kernel(StepArgs a, int side, int level) {
  constexpr int NC = LT ? LT * LT : MAX_KERNEL_L * MAX_KERNEL_L;
  __shared__ Smem<NC> S;
  const int b = blockIdx.x;
  if (b >= a.B) return;
  if (a.reset_mask && !a.reset_mask[b]) return;
  stage_cfg(S, a.cfg);
  const int L = LT ? LT : a.L;
  const Ctx x{S.cfg, L, L * L, (int)threadIdx.x, a.cfgs, a.epoch};
  Prefetch P;
  prefetch_issue<PF_SMALL, PF_SMALL>(P, a, b, x.lane, x.NCr, false);
  U u;
  load_board<NC, PF_SMALL, PF_SMALL>(S, u, x, a, b, P);
  if (u.num_roads < 1 || u.num_roads > 3) return;  // never reset: nothing to act on
  uint32_t* const hot = a.opp_hot + (size_t)b * HOT_WORDS;
  WaveMt R{a.opp_mt + (size_t)b * OPP_WORDS, lane_word(P.w, PF_HOT + 0), lane_word(P.w, PF_HOT + 1)};
  R.cn = lane_word(P.w, PF_HOT + 2);
  R.cbase = lane_word(P.w, PF_HOT + 3);
  R.cache = __shfl(P.w, PF_HOT + 4 + (x.lane < HOT_CACHE ? x.lane : 0));
  with_opp_rng(a, b, x.lane, R, [&](auto& G) {
    if (side == 0) opponent_enemy(S, u, x, G, level);
    else opponent_tower(S, u, x, G, level);
  });
  __syncthreads();
  R.prefetch(x.lane);  // the next step expects the hot record primed
  const size_t eb = (size_t)b * ECAP;
  for (int i = x.lane; i < u.n; i += 64) {
    sst(&a.en_lp[eb + i], S.eLP[i]);
    sst(&a.en_mg[eb + i], S.eMg[i]);
    sst(&a.en_inf[eb + i], S.eInf[i]);
  }
  store_cells(S, u, x, a, b);
  store_board(S, u, x, a, b);
  if (x.lane == 0) { hot[0] = R.pos; hot[1] = R.tw; hot[2] = R.cn; hot[3] = R.cbase; }
  if (x.lane < HOT_CACHE) hot[4 + x.lane] = R.cache;
}

template <int LT>
static hipError_t launch_opponent2(const StepArgs& a, int side, int level, hipStream_t s) {
  hipLaunchKernelGGL(td_opponent_kernel<LT>, dim3(a.B), dim3(64), 0, s, a, side, level);
  return hipGetLastError();
}

hipError_t launch_opponent(const StepArgs& a, int side, int level, hipStream_t s) {
  switch (a.L) {
    case 10: return launch_opponent2<10>(a, side, level, s);
    case 20: return launch_opponent2<20>(a, side, level, s);
    case 30: return launch_opponent2<30>(a, side, level, s);
    default: return launch_opponent2<0>(a, side, level, s);
  }
}

// Layout draws are resumable (RoadGen::draw): a refill gives each board a budget of
// walks per launch, and a draw that runs out (in practice one the reference never
// finishes, ~1,000 walks per retry loop) keeps its state in the board's HBM scratch
// -- the RoadResume header, then the generator's arrays -- with the partial record
// in the ring slot (its tag still the old one) and the stream position in np_mt.
// The next refill continues it draw for draw.  So a refill launch runs at most
// ~a.refill_walks walks per board -- except for a board whose ring is empty, whose
// draw runs to the end at once (rare: the initial fill, or episodes shorter than the
// refill can follow).
__device__ __forceinline__ RoadResume* resume_hdr(const StepArgs& a, int b) {
  return reinterpret_cast<RoadResume*>(a.scratch + (size_t)b * a.scratch_stride);
}

// TDGymBasic.reset's draws (:42-51) for board b into slot `slot` of its ring, as
// layout number `n` of the stream: failing draws are skipped up to ``retries``
// times, at most ``budget`` walks are run (ROAD_PENDING: continued by a later call).
// A finished record is published for a step grid that may be running on another
// stream: plain stores, every lane's vmcnt(0), the barrier, ONE agent-scope
// release, then the tag by an sc1 store (MI355X_MICROARCH.md § visibility, "Valid
// forms", producer bullet).  Returns the road status of the last draw.
template <int NC, bool SBP = false>
__device__ int wave_layout(LayoutSmem<NC>& G, const StepArgs& a, int b, int retries, uint32_t* slot, uint32_t n,
                           int budget) {
  const int lane = (int)threadIdx.x, L = a.L, lw = LAYOUT_HDR + L * L;
  const int sbytes = (int)road_scratch_bytes(L);
  // (the walk budget and the retry count bound the draw's loop: wave-uniform, SGPRs)
  budget = (int)__builtin_amdgcn_readfirstlane((uint32_t)budget);
  retries = (int)__builtin_amdgcn_readfirstlane((uint32_t)retries);
  uint32_t* gmt = a.np_mt + (size_t)b * OPP_WORDS;
  RoadResume* ghdr = resume_hdr(a, b);
  uint8_t* gscr = a.scratch + (size_t)b * a.scratch_stride + sizeof(RoadResume);
  for (int i = lane; i < OPP_WORDS; i += 64) G.mt[i] = gmt[i];
  if (lane < 16) reinterpret_cast<uint32_t*>(&G.res)[lane] = reinterpret_cast<const uint32_t*>(ghdr)[lane];
  __syncthreads();
  const bool resumed = G.res.phase != RP_NEW;  // wave-uniform
  if (resumed) {
    for (int i = lane; i < sbytes / 4; i += 64) reinterpret_cast<uint32_t*>(G.scratch)[i] = reinterpret_cast<const uint32_t*>(gscr)[i];
    for (int i = 1 + lane; i < lw; i += 64) G.rec[i] = slot[i];
    __syncthreads();
  }
  int st = ROAD_ERR_BOUND;
  {
    WaveRoadGen<NC, SBP> g;
    g.carve(G.scratch, L * L);
    g.mt = G.mt; g.rec = G.rec; g.L = L; g.lane = lane;
    // the stream position and the resume state are wave-uniform: SGPRs
    g.pos = __builtin_amdgcn_readfirstlane(G.mt[MT_N]);
    g.tw = __builtin_amdgcn_readfirstlane(G.mt[MT_N + 1]);
    g.base = g.pos; g.n = 0; g.win = 0;
    RoadResume res;
    for (int i = 0; i < 16; ++i)
      reinterpret_cast<uint32_t*>(&res)[i] = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(&G.res)[i]);
    g.load_maps(resumed);  // the draw's field / turn bitmaps
    st = g.draw(res, budget, kRoadAttempts, retries);
    __syncthreads();
    g.save_maps();
    if (lane == 0) { G.mt[MT_N] = g.pos; G.mt[MT_N + 1] = g.tw; G.res = res; }
  }
  __syncthreads();
  // every store below is write-through (st_relaxed = sc1): the claim release and the
  // tag store publish them without a release fence (see claim_board)
  for (int i = lane; i < OPP_WORDS; i += 64) st_relaxed(gmt + i, G.mt[i]);
  if (lane < 16) st_relaxed(reinterpret_cast<uint32_t*>(ghdr) + lane, reinterpret_cast<const uint32_t*>(&G.res)[lane]);
  if (st == ROAD_PENDING) {  // keep the draw for the next call (published by the caller's claim release)
    for (int i = lane; i < sbytes / 4; i += 64)
      st_relaxed(reinterpret_cast<uint32_t*>(gscr) + i, reinterpret_cast<const uint32_t*>(G.scratch)[i]);
    for (int i = 1 + lane; i < lw; i += 64) st_relaxed(slot + i, G.rec[i]);
  } else if (st == ROAD_OK) {
    for (int i = 1 + lane; i < lw; i += 64) st_relaxed(slot + i, G.rec[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's record stores have landed
    __syncthreads();
    if (lane == 0) st_relaxed(slot, slot_tag(n));
  }
  return st;
}

// TDGymBasic.reset of board b, by one wave (the device is idle for this board: no refill
// holds it).  The layout is the caller's record (td_reset_layouts), else the board's
// next staged layout, else a draw from its numpy stream now -- skipping up to `retries`
// failing draws.  A draw that still fails leaves the board unchanged and returns its
// road status (the reference raises); else the board is reset, its first observation
// written, and ROAD_OK returned.  keep_flags: an auto-reset keeps the board's flags,
// an explicit reset clears them.
template <int NC, int LT>
__device__ int reset_one(Smem<NC>& S, LayoutSmem<NC>& gen, const StepArgs& a, int b, int retries, bool keep_flags) {
  const int L = LT ? LT : a.L;
  const uint32_t* rec;
  bool from_ring = false;
  uint32_t head = 0;
  const int ov = a.ovr_idx ? a.ovr_idx[b] : -1;
  if (ov >= 0) {
    rec = a.ovr_rec + (size_t)ov * (LAYOUT_HDR + L * L);
  } else {
    head = a.lay_head[b];
    const uint32_t tail = a.lay_tail[b];
    uint32_t* slot = a.nxt + ((size_t)b * NSLOT + head % NSLOT) * a.slot_words;
    if (tail == head) {  // nothing staged: draw now
      const int st = wave_layout(gen, a, b, retries, slot, head, 0x7fffffff);
      __syncthreads();
      if (st != ROAD_OK) return st;
      if (threadIdx.x == 0) a.lay_tail[b] = tail + 1u;
    }
    rec = slot;
    from_ring = true;
  }
  stage_cfg(S, a.cfg);
  __syncthreads();
  const Ctx x{S.cfg, L, L * L, (int)threadIdx.x, a.cfgs, a.epoch};
  U u;
  u.episodes = a.hdr[b].episodes;
  u.flags = keep_flags ? a.hdr[b].flags : 0;
  reset_board(S, u, x, rec);
  channel_scalars(S, u, x);
  store_cells(S, u, x, a, b);
  pack_obs_cells(S, x);
  if (a.obs) {
    float* const o = a.obs + (size_t)b * NCH * x.NCr;
    if constexpr (LT != 0) {
      if ((reinterpret_cast<uintptr_t>(a.obs) & 15u) == 0) write_obs_lines<NC, LT>(S, x.lane, o, false, false);
      else write_obs<NC, LT>(S, x, o, false);
    } else {
      write_obs<NC, LT>(S, x, o, false);
    }
  }
  store_board(S, u, x, a, b);
  if (x.lane == 0 && from_ring) a.lay_head[b] = head + 1u;
  return ROAD_OK;
}

template <int NC>
union ResetSmem {
  Smem<NC> board;
  LayoutSmem<NC> gen;
};

// TDGymBasic.reset for the boards in reset_mask (td_reset / td_reset_layouts: the
// device is idle, td_capi synchronises first).  A failing draw (no retry) is reported
// in reset_fail and leaves the board unchanged, as the reference raises.
template <int LT>
__global__ __launch_bounds__(64) void td_reset_kernel(StepArgs a) {
  constexpr int NC = LT ? LT * LT : MAX_KERNEL_L * MAX_KERNEL_L;
  __shared__ ResetSmem<NC> sh;
  const int b = blockIdx.x;
  if (b >= a.B) return;
  if (a.reset_mask && !a.reset_mask[b]) return;
  const int st = reset_one<NC, LT>(sh.board, sh.gen, a, b, 0, false);
  if (threadIdx.x == 0) a.reset_fail[b] = (uint8_t)st;
}

// Auto-reset with random_agent=False (TDGymBasic.py:87-89,101-103 under gym 0.21's
// AsyncVectorEnv, which calls reset() right after the step that ends an episode): the
// built-in opponent and reset() draw from the same numpy stream, so the next layout
// cannot be drawn ahead of play.  Launched right behind each step kernel on its
// stream: a wave scans 64 boards' done flags (written by that step) and resets the
// finished boards in turn, drawing each layout from the board's stream now, exactly
// where the reference's reset() would -- failing draws skipped as in every auto-reset.
// The step kernel left those boards finished (no staged layout is consumed in this
// mode); their observation is overwritten with the new episode's first one.  Boards
// flagged FLAG_NO_LAYOUT are skipped: a board never reset (its first road generation
// failed, done every step) or whose auto-reset already failed 65 draws in a row stays
// as it is until an explicit reset, as under random_agent=True -- it neither stalls
// the step stream with 65 draws every step nor consumes its stream.
template <int LT>
__global__ __launch_bounds__(64) void td_autoreset_kernel(StepArgs a) {
  constexpr int NC = LT ? LT * LT : MAX_KERNEL_L * MAX_KERNEL_L;
  __shared__ ResetSmem<NC> sh;
  const int lane = (int)threadIdx.x;
  const int b0 = (int)blockIdx.x * 64;
  const bool mine = b0 + lane < a.B && a.done[b0 + lane] != 0 && !(a.hdr[b0 + lane].flags & FLAG_NO_LAYOUT);
  uint64_t m = ballot(mine);
  while (m) {
    const int b = b0 + ctz64(m);
    m &= m - 1;
    const int st = reset_one<NC, LT>(sh.board, sh.gen, a, b, kLayoutRetries, true);
    __syncthreads();
    if (st != ROAD_OK && lane == 0) a.hdr[b].flags |= FLAG_NO_LAYOUT;  // keeps stepping its finished episode
  }
}

// Keep every board's ring of staged layouts full: lanes check G boards at once
// (layouts drawn minus consumed < NSLOT), then the wave draws the missing layouts
// of those boards one by one with the whole-wave generator (WaveRoadGen).
//
// guard = 0 (refill): runs on a side stream concurrently with the step grids, which
// never wait for it; a board another refill holds is skipped, and a draw gets at most
// a.refill_walks walks unless the ring is empty.
//
// guard = G > 0 (ring guard): runs ON the step stream, between two steps, before every
// G-th step (td_capi.hip td_step): every ring holding fewer than G complete layouts is
// filled to G -- draws run to the end, a board a side refill holds is waited for (its
// wave is resident and gives the claim back after its walk budget).  A board consumes
// at most one layout per step, so none of the next G steps finds its ring empty: an
// episode end never depends on the refill cadence (TDGymBasic.py:37-55 resets at every
// end).  The one exception is the reference's own failure, 65 failing draws in a row
// (it raises): the ring stays short and the step flags the board no_layout.  Rings
// below G are rare when the side refills keep up (a board would have to finish
// NSLOT - G + 1 episodes between two refills), so a guard launch is mostly a scan.
template <int LT>
__global__ __launch_bounds__(64) void td_refill_kernel(StepArgs a, int guard) {
  constexpr int NC = LT ? LT * LT : MAX_KERNEL_L * MAX_KERNEL_L;
  __shared__ LayoutSmem<NC> G;
  const int lane = (int)threadIdx.x;
  const int grp = a.refill_grp;
  const uint32_t level = guard ? (uint32_t)guard : (uint32_t)NSLOT;  // layouts wanted per ring
  for (int base = (int)blockIdx.x * grp; base < a.B; base += (int)gridDim.x * grp) {
    const int b = base + lane;
    const bool mine = lane < grp && b < a.B;
    uint32_t head = 0, tail = 0;
    if (mine) {
      head = ld_relaxed(a.lay_head + b);  // a step grid may be advancing it right now
      tail = ld_relaxed(a.lay_tail + b);
    }
    uint64_t m = ballot(mine && tail - head < level);
    while (m) {
      const int l = ctz64(m);
      m &= m - 1;
      const int bb = base + l;
      if (!claim_board(a.lay_claim + bb, lane)) {  // another refill is drawing its layouts
        if (!guard) continue;
        // a board whose claim wait already gave up is not waited for again (a claim never
        // given back would stall every guard launch 1 s); it is not counted twice either
        if (ld_relaxed((const uint32_t*)&a.hdr[bb].flags) & FLAG_CLAIM_TIMEOUT) continue;
        // the holder is a resident side-refill wave that gives the claim back after its
        // walk budget; bounded all the same (1 s, as take_dry_ring): a claim never given
        // back leaves this board's ring short -- its episode end is then flagged
        // no_layout by the step -- instead of hanging the step stream
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool got = false;
        while (!got && __builtin_amdgcn_s_memrealtime() - t0 < kTakeSpinTicks) {
          __builtin_amdgcn_s_sleep(8);
          got = claim_board(a.lay_claim + bb, lane);
        }
        if (!got) {  // visible: the board's flag and the engine's counter (td_guard_timeouts)
          if (lane == 0) {
            atomicOr(&a.hdr[bb].flags, FLAG_CLAIM_TIMEOUT);
            if (a.guard_to) atomicAdd(a.guard_to, 1u);
          }
          continue;
        }
      }
      uint32_t t = __builtin_amdgcn_readfirstlane(ld_relaxed(a.lay_tail + bb));  // (wave-uniform: SGPRs)
      const uint32_t h = __builtin_amdgcn_readfirstlane(ld_relaxed(a.lay_head + bb));
#pragma nounroll
      while (t - h < level) {
        uint32_t* slot = a.nxt + ((size_t)bb * NSLOT + t % NSLOT) * a.slot_words;
        // an empty ring is urgent (the board needs this layout at its next episode end):
        // its draw runs to the end; otherwise at most a.refill_walks walks this launch
        const int st = wave_layout<NC, kGenSBProof && NC <= 128>(
            G, a, bb, kLayoutRetries, slot, t, t == h || guard ? 0x7fffffff : a.refill_walks);
        __syncthreads();
        if (st != ROAD_OK) break;  // out of walks (continued next launch), or 65 failing draws in a row
        ++t;
      }
      if (lane == 0) st_relaxed(a.lay_tail + bb, t);
      release_board(a.lay_claim + bb, lane);
    }
  }
}

// The step kernel of a mode: K<LT, MODE, SCAN> for K = td_step_kernel or td_step_kernel_small.
#define TD_STEP_DISPATCH(K, LT, a, CALL)                                   \
  do {                                                                     \
    if ((a).mode == MODE_DEF && (a).multi) CALL((K<LT, MODE_DEF, true>));  \
    else if ((a).mode == MODE_DEF) CALL((K<LT, MODE_DEF, false>));         \
    else if ((a).mode == MODE_ATK) CALL((K<LT, MODE_ATK, false>));         \
    else if ((a).multi) CALL((K<LT, MODE_2P, true>));                      \
    else CALL((K<LT, MODE_2P, false>));                                    \
  } while (0)

// ev0 / ev1 (optional): timing events bound to the step kernel's own dispatch
// (hipExtLaunchKernelGGL), so their interval is the kernel's start-to-end as the
// dispatch packet timestamps it -- no marker packets around the launch.
template <int LT>
static hipError_t launch2(const StepArgs& a, hipStream_t s, bool reset, hipEvent_t ev0, hipEvent_t ev1) {
#define TD_LAUNCH(k)                                                                    \
  do {                                                                                  \
    if (ev0) hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64), 0, s, ev0, ev1, 0, a);       \
    else hipLaunchKernelGGL(k, dim3(a.B), dim3(64), 0, s, a);                           \
  } while (0)
#define TD_LAUNCH2(k)                                                                    \
  do {                                                                                   \
    if (ev0) hipExtLaunchKernelGGL(k, dim3(a.B), dim3(128), 0, s, ev0, ev1, 0, a);       \
    else hipLaunchKernelGGL(k, dim3(a.B), dim3(128), 0, s, a);                           \
  } while (0)
  const bool aligned = (reinterpret_cast<uintptr_t>(a.obs) & 15u) == 0;
  if (reset) {
    hipLaunchKernelGGL(td_reset_kernel<LT>, dim3(a.B), dim3(64), 0, s, a);
  } else if constexpr (LT != 0) {
    if (a.small == 2 && aligned) TD_STEP_DISPATCH(td_step_kernel_small2, LT, a, TD_LAUNCH2);
    else if (a.small && aligned) TD_STEP_DISPATCH(td_step_kernel_small, LT, a, TD_LAUNCH);
    else TD_STEP_DISPATCH(td_step_kernel, LT, a, TD_LAUNCH);
  } else {
    TD_STEP_DISPATCH(td_step_kernel, LT, a, TD_LAUNCH);
  }
#undef TD_LAUNCH
#undef TD_LAUNCH2
  return hipGetLastError();
}

// Step-kernel workgroups (boards) resident at once on the device: the batch size up
// to which a step runs as one round of waves (td_step_kernel_small).
template <int LT>
static int resident3(const StepArgs& a, int cus, int waves) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
#define TD_OCC(k) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64, 0)
#define TD_OCC2(k) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 128, 0)
  if (waves == 2) TD_STEP_DISPATCH(td_step_kernel_small2, LT, a, TD_OCC2);
  else TD_STEP_DISPATCH(td_step_kernel_small, LT, a, TD_OCC);
#undef TD_OCC
#undef TD_OCC2
  return e == hipSuccess ? n * cus : 0;
}

int step_resident_boards(const StepArgs& a, int cus, int waves) {
  switch (a.L) {
    case 10: return resident3<10>(a, cus, waves);
    case 20: return resident3<20>(a, cus, waves);
    case 30: return resident3<30>(a, cus, waves);
    default: return 0;  // generic-L kernels: no small-batch build
  }
}

hipError_t launch_step(const StepArgs& a, hipStream_t s, bool reset, hipEvent_t ev0, hipEvent_t ev1) {
  switch (a.L) {
    case 10: return launch2<10>(a, s, reset, ev0, ev1);
    case 20: return launch2<20>(a, s, reset, ev0, ev1);
    case 30: return launch2<30>(a, s, reset, ev0, ev1);
    default: return launch2<0>(a, s, reset, ev0, ev1);
  }
}

// The paramConfig epochs live enemies and towers still refer to (td_set_config
// recycles the others): one wave per board, bits OR-ed into used[NCFG / 32].
__global__ __launch_bounds__(64) void td_cfg_usage_kernel(StepArgs a, uint32_t* used) {
  const int b = blockIdx.x, l = (int)threadIdx.x;
  if (b >= a.B) return;
  const int n = a.hdr[b].n_en, nt = a.hdr[b].n_tw;
  for (int i = l; i < n; i += 64) {
    const int e = en_ep(a.en_inf[(size_t)b * ECAP + i]);
    atomicOr(&used[e >> 5], 1u << (e & 31));
  }
  if (l < nt) {
    const uint32_t ti = a.tw_inf[(size_t)b * TCAP + l];
    atomicOr(&used[tw_ec(ti) >> 5], 1u << (tw_ec(ti) & 31));
    atomicOr(&used[tw_eu(ti) >> 5], 1u << (tw_eu(ti) & 31));
  }
}

hipError_t launch_cfg_usage(const StepArgs& a, uint32_t* used, hipStream_t s) {
  hipLaunchKernelGGL(td_cfg_usage_kernel, dim3(a.B), dim3(64), 0, s, a, used);
  return hipGetLastError();
}

template <int LT>
static void launch_autoreset2(const StepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(td_autoreset_kernel<LT>, dim3((a.B + 63) / 64), dim3(64), 0, s, a);
}

hipError_t launch_autoreset(const StepArgs& a, hipStream_t s) {
  switch (a.L) {
    case 10: launch_autoreset2<10>(a, s); break;
    case 20: launch_autoreset2<20>(a, s); break;
    case 30: launch_autoreset2<30>(a, s); break;
    default: launch_autoreset2<0>(a, s); break;
  }
  return hipGetLastError();
}

template <int LT>
static void launch_refill2(const StepArgs& a_, hipStream_t s, int guard) {
  StepArgs a = a_;
  if (guard) a.refill_grp = 64;  // the guard mostly scans: one ballot of 64 boards per wave, one wave per 64 boards
  const int grp = a.refill_grp;
  const int groups = (a.B + grp - 1) / grp;  // a wave walks the groups grid-stride
  const int waves = guard || groups < a.refill_waves ? groups : a.refill_waves;
  hipLaunchKernelGGL(td_refill_kernel<LT>, dim3(waves), dim3(64), 0, s, a, guard);
}

hipError_t launch_refill(const StepArgs& a, hipStream_t s, int guard) {
  switch (a.L) {
    case 10: launch_refill2<10>(a, s, guard); break;
    case 20: launch_refill2<20>(a, s, guard); break;
    case 30: launch_refill2<30>(a, s, guard); break;
    default: launch_refill2<0>(a, s, guard); break;
  }
  return hipGetLastError();
}

}  // namespace td
