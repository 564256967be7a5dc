// td_step_half.hip -- the batched gym-TD step with one HALF-wave (32 lanes) per board.
//
// td_step.hip gives every board a 64-lane wave.  At small batches (8,192 boards = the
// N = 8 share of BASELINE's 65,536, and 4,096 = configs[1]) that grid is one round of
// waves, and its kernel time is the launch ramp plus the last-started wave's step: the
// dispatcher starts a one-wave workgroup per board over 7.6-9.5 us while the started
// waves keep the VALU busy, but a grid of half as many waves starts in ~2 us under the
// same load (scripts/launch_ramp.hip, profiles/r04/s13-s15).  Here wave w steps the two
// NEIGHBOURING boards 2w' and 2w' + 1 (w' its XCD-mapped pair), one per half, in lockstep:
//   * lane l works for board 2w' + (l >> 5) as lane hl = l & 31 of that board: the
//     serial phases of the reference run half-uniform, ballots are split by half, and a
//     lane's broadcast of a half-uniform index reads two v_readlane (one per half);
//   * the board images sit side by side in LDS (PairSmem, one constant block for both);
//   * the two boards' observations are ONE contiguous 36,000-B stretch of the batch's
//     (B, 45, L, L) output, written by the whole wave in 128-B-aligned 1-KB windows:
//     the line the two boards share is written whole by one store, so only the two
//     lines at the ends of the pair are shared with other waves.
// Same step, same results as td_step_kernel_small (bit for bit: every parity test runs
// on this kernel too); the rules and encodings come from td_board.h.
//
// Reference order of one env step: cool-downs (TDDefense.py:38-39),
// the defender action (:40-77), the built-in attacker (TDGymBasic.py:81-108), TDBoard.step
// (TDBoard.py:295-368), done / get_states / info (TDBoard.py:370-385, 85-144,
// TDDefense.py:81-87).  Built for TD-def discrete at L = 10 (the metric's boards).
#include <hip/hip_runtime.h>

#include <hip/hip_ext.h>

#include <climits>

#include "td_board.h"
#include "td_kernels.h"
#include "td_layout.h"
#include "td_rng.h"
#include "td_wave.h"

namespace td {

#ifdef TD_STAMPS  // diagnostic builds: per-phase s_memtime stamps of each board (td_step.hip STAMP slots)
#define HSTAMP(i) do { if (a.stamps && x.hl == 0) a.stamps[(size_t)b * 16 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
#define HSTAMP_AT(bb, i, clk) do { if (a.stamps) a.stamps[(size_t)(bb) * 16 + (i)] = (clk); } while (0)
#else
#define HSTAMP(i) do { } while (0)
#define HSTAMP_AT(bb, i, clk) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// the pair's LDS image
// ---------------------------------------------------------------------------
template <int NC>
struct alignas(16) HalfBoard {
  static_assert(NC % 4 == 0 && NC / 4 <= 32, "cells move as one 16-B unit per lane of a half");
  uint32_t cell[NC];  // cell words (td_layout.h) + the tower nibble (td_board.h tw_nib)
  uint8_t grp[4][NC];  // enemy group (head enemy index) per (type, cell), 0xFF none
  union {
    struct {           // load .. march: the enemy list
      double eLP[ECAP];
      double eMg[ECAP];
    };
    float gst[ECAP][4];  // stats .. obs: group min, max, avg, count/8 by head enemy
  };
  uint32_t eInf[ECAP];
  double tCd[TCAP];
  uint32_t tInf[TCAP];
  union alignas(16) {
    uint32_t stg[48];  // load: header (24 words), discrete action (2), opponent hot record (12)
    struct {           // observation
      float chv[48];   // broadcast channel values
      float d9[32];    // channel 9 by distance (road length < 2L <= 32)
    };
  };
};

template <int NC>
struct alignas(16) PairSmem {
  HalfBoard<NC> hb[2];
  TdDevCfg cfg;  // the current constant block, staged once for both boards
};

// ---------------------------------------------------------------------------
// half-wave lane helpers
// ---------------------------------------------------------------------------
// The 32 bits of a wave ballot that belong to half h.
__device__ __forceinline__ uint32_t half_bits(uint64_t m, int h) { return (uint32_t)(m >> (h << 5)); }
__device__ __forceinline__ uint32_t hballot(bool p, int h) { return half_bits(__ballot(p), h); }
__device__ __forceinline__ int ctz32(uint32_t m) { return __builtin_ctz(m); }
__device__ __forceinline__ int popc32(uint32_t m) { return __popc(m); }

// The larger of a half-uniform value over the halves active here (0 for none): the
// wave-uniform bound of a loop both halves run in lockstep.
__device__ __forceinline__ int wmax(int v) {
  const uint64_t ex = __ballot(true);
  const int a = (ex & 1ull) ? (int)__builtin_amdgcn_readlane((uint32_t)v, 0) : 0;
  const int b = ((ex >> 32) & 1ull) ? (int)__builtin_amdgcn_readlane((uint32_t)v, 32) : 0;
  return a > b ? a : b;
}
// Lane j of this lane's half, j wave-uniform (0 <= j < 32): two scalar reads.
__device__ __forceinline__ uint32_t hru(uint32_t v, int j, int h) {
  const uint32_t a = __builtin_amdgcn_readlane(v, j), b = __builtin_amdgcn_readlane(v, j + 32);
  return h ? b : a;
}
__device__ __forceinline__ double hru(double v, int j, int h) {
  return __hiloint2double((int)hru((uint32_t)__double2hiint(v), j, h), (int)hru((uint32_t)__double2loint(v), j, h));
}
__device__ __forceinline__ float hru(float v, int j, int h) {
  return __uint_as_float(hru(__float_as_uint(v), j, h));
}
// Lane j of this lane's half, j half-uniform (each half its own index, 0 <= j < 32).
__device__ __forceinline__ uint32_t hrd(uint32_t v, int j, int h) {
  const int j0 = (int)(__builtin_amdgcn_readlane((uint32_t)j, 0) & 31u);
  const int j1 = (int)(__builtin_amdgcn_readlane((uint32_t)j, 32) & 31u);
  const uint32_t a = __builtin_amdgcn_readlane(v, j0), b = __builtin_amdgcn_readlane(v, j1 + 32);
  return h ? b : a;
}
__device__ __forceinline__ double hrd(double v, int j, int h) {
  return __hiloint2double((int)hrd((uint32_t)__double2hiint(v), j, h), (int)hrd((uint32_t)__double2loint(v), j, h));
}
// Lane j of this lane's half, j per lane (an LDS permute).
__device__ __forceinline__ uint32_t hshfl(uint32_t v, int j, int lane) {
  return (uint32_t)__shfl((int)v, (lane & 32) | (j & 31));
}

// Half-uniform board state (U of td_step.hip, held per lane).
struct HU {
  double cost_def, cost_atk, ep_ret, progress, max_cost;
  int steps, base_LP, atk_cd, def_cd, n, nt, num_roads, end_cell, maxdist, flags, episodes, max_base_LP;
  uint64_t starts;  // start cells of roads 0-2, 16 bits each (a shift, not a select of fields: keeps HU in registers)
  bool cells_dirty, tw_dirty;
  __device__ __forceinline__ int start(int road) const { return (int)((starts >> (16 * road)) & 0xffffu); }
  __device__ __forceinline__ void set_starts(uint32_t s0, uint32_t s1, uint32_t s2) {
    starts = (uint64_t)s0 | ((uint64_t)s1 << 16) | ((uint64_t)s2 << 32);
  }
};

struct HCtx {
  const TdDevCfg& C;  // the current constant block (epoch ep), staged in LDS
  int L, NCr, lane, hl, h;
  const TdDevCfg* tab;  // every epoch's block (HBM)
  int ep;
};

template <class F>
__device__ __forceinline__ double hcaptured(const HCtx& x, int ep, F f) {
  double v = f(x.C);
  if (ep != x.ep) v = f(x.tab[ep]);
  return v;
}

__device__ __forceinline__ double h_e_def(const HCtx& x, uint32_t inf) {
  const int t = en_type(inf), lv = en_lv(inf);
  return hcaptured(x, en_ep(inf), [&](const TdDevCfg& c) { return c.e_def[t][lv]; });
}

template <int NC>
__device__ __forceinline__ void h_set_tower(HalfBoard<NC>& S, int cell, uint32_t nib) {
  S.cell[cell] = (S.cell[cell] & ~kTwBits) | nib;
}

// ---------------------------------------------------------------------------
// CPython MT19937 of the built-in opponent, one stream per half (td_step.hip WaveMt)
// ---------------------------------------------------------------------------
struct HalfMt {
  uint32_t* w;        // the board's stream words (per half)
  uint32_t pos, tw;   // position, lazy-twist boundary: words [tw, 624) hold the previous block
  int hl, h, lane;
  uint32_t cache = 0, cbase = 0, cn = 0;  // lane hl: tempered output for position cbase + hl (hl < cn)
  uint32_t pa = 0, pnb = 0, pfar = 0;
  bool plazy = false, pmine = false;
  uint32_t ep0 = ~0u;  // the early window's first position (~0u: none)
  static constexpr uint32_t kWin = 16;

  static __device__ __forceinline__ uint32_t twist1(uint32_t a, uint32_t b, uint32_t far) {
    const uint32_t yy = (a & 0x80000000u) | (b & 0x7fffffffu);
    return far ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
  }
  __device__ __forceinline__ void load3(uint32_t q) {
    pa = w[q];
    if (plazy) {
      pnb = w[q == MT_N - 1 ? 0u : q + 1u];
      pfar = w[q < (uint32_t)(MT_N - MT_M) ? q + MT_M : q - (MT_N - MT_M)];
    }
  }
  // the late pre-draw of the next HOT_CACHE words (a window the step outran)
  __device__ __forceinline__ void prefetch_issue() {
    if (pos >= (uint32_t)MT_N) { tw = 0; pos = 0; }
    cbase = pos;
    cn = (uint32_t)MT_N - pos < (uint32_t)HOT_CACHE ? (uint32_t)MT_N - pos : (uint32_t)HOT_CACHE;
    const uint32_t q = pos + (uint32_t)hl;
    pmine = (uint32_t)hl < cn;
    plazy = pmine && q >= tw;
    if (pmine) load3(q);
  }
  // The early window [p0, p0 + 16) at the step's starting position, loaded before any
  // of the step's stores (td_step.hip WaveMt::early_issue).
  __device__ __forceinline__ void early_issue() {
    ep0 = ~0u;
    if (pos + kWin > (uint32_t)MT_N) return;
    ep0 = pos;
    const uint32_t q = pos + (uint32_t)hl;
    pmine = (uint32_t)hl < kWin;
    plazy = pmine && q >= tw;
    if (pmine) load3(q);
  }
  __device__ __forceinline__ void early_finish() {
    uint32_t base, n, d;
    if (ep0 != ~0u && pos - ep0 <= kWin - 8u) {
      base = ep0; n = kWin; d = pos - ep0;
    } else {
      prefetch_issue();
      base = cbase; n = cn; d = 0u;
    }
    const uint32_t q = base + (uint32_t)hl;
    uint32_t y = pa;
    if (plazy) {
      y = twist1(pa, pnb, pfar);
      w[q] = y;  // (a word the step's slow path twisted meanwhile: the same value again)
    }
    if (base + n > tw) tw = base + n;
    const uint32_t t = pmine ? mt_temper(y) : 0u;
    cache = hshfl(t, (int)(((uint32_t)hl + d) & 31u), lane);
    cbase = pos;
    cn = n - d < (uint32_t)HOT_CACHE ? n - d : (uint32_t)HOT_CACHE;
  }
  __device__ __forceinline__ uint32_t next() {
    const uint32_t d = pos - cbase;
    const uint32_t c = hrd(cache, (int)(d & 31u), h);  // (read outside the branch: every lane takes part)
    if (d < cn) {
      ++pos;
      return c;
    }
    if (pos >= (uint32_t)MT_N) { tw = 0; pos = 0; cn = 0; }
    uint32_t y;
    if (pos >= tw) {
      const uint32_t a = w[pos];
      const uint32_t nb = w[pos == MT_N - 1 ? 0u : pos + 1u];
      const uint32_t far = w[pos < (uint32_t)(MT_N - MT_M) ? pos + MT_M : pos - (MT_N - MT_M)];
      y = twist1(a, nb, far);
      w[pos] = y;  // every lane of the half stores the same word
      tw = pos + 1;
    } else {
      y = w[pos];
    }
    ++pos;
    return mt_temper(y);
  }
  __device__ __forceinline__ int64_t randbelow(int64_t n) {
    if (n <= 0) return 0;
    const int k = 64 - __builtin_clzll((unsigned long long)n);
    uint32_t r = next() >> (32 - k);
    while ((int64_t)r >= n) r = next() >> (32 - k);
    return r;
  }
  __device__ __forceinline__ int64_t randint(int64_t a, int64_t b) { return a + randbelow(b - a + 1); }
  __device__ __forceinline__ int64_t np_randint(int64_t lo, int64_t hi) {
    if (hi <= lo + 1) return lo;
    const uint32_t rng = (uint32_t)(hi - lo - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v = next() & mask;
    while (v > rng) v = next() & mask;
    return lo + (int64_t)v;
  }
};

// The TD-def opponent's random source (td_step.hip OppRng): the board's CPython stream,
// or (random_agent=False) its numpy layout stream.
template <bool NP>
struct HOppRng {
  HalfMt& py;
  HalfMt& np;
  __device__ __forceinline__ int64_t ri(int64_t lo, int64_t hi) {
    if constexpr (NP) return np.np_randint(lo, hi + 1); else return py.randint(lo, hi);
  }
  __device__ __forceinline__ int64_t slot(int64_t types) {
    if constexpr (NP) return np.np_randint(0, types); else return py.randint(0, types);
  }
};

template <class F>
__device__ __forceinline__ void h_with_opp_rng(const StepArgs& a, int b, const HCtx& x, HalfMt& R, F&& f) {
  if (a.opp_np) {
    uint32_t* const npw = a.np_mt + (size_t)b * OPP_WORDS;
    HalfMt N{npw, npw[MT_N], npw[MT_N + 1], x.hl, x.h, x.lane};
    N.cbase = N.pos;
    HOppRng<true> G{R, N};
    f(G);
    if (x.hl == 0) { npw[MT_N] = N.pos; npw[MT_N + 1] = N.tw; }
  } else {
    HOppRng<false> G{R, R};
    f(G);
  }
}

// ---------------------------------------------------------------------------
// defender operations (TDBoard.py:226-293), half-uniform
// ---------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void h_diamond(HalfBoard<NC>& S, const HCtx& x, int cell, int delta) {
  const int k = x.C.tower_distance, W = 2 * k + 1, L = x.L;
  const int r0 = cell / L, c0 = cell % L;
  for (int idx = x.hl; idx < W * W; idx += 32) {
    const int i = idx / W - k, j = idx % W - k;
    const int ai = i < 0 ? -i : i, aj = j < 0 ? -j : j;
    const int r = r0 + i, c = c0 + j;
    if (ai + aj <= k && r >= 0 && r < L && c >= 0 && c < L) {
      const uint32_t w = S.cell[r * L + c];
      const int cnt = (int)(w >> 24) + delta;
      S.cell[r * L + c] = (w & 0x00ffffffu) | ((uint32_t)(cnt & 0xff) << 24);
    }
  }
  wsync();
}

template <int NC>
__device__ __forceinline__ int h_tower_build(HalfBoard<NC>& S, HU& u, const HCtx& x, int t, int cell) {
  const double price = x.C.t_price[t][0];
  if (u.cost_def < price) return FC_COST;                 // :228
  if (cw_block(S.cell[cell]) > 0) return FC_POS;          // :232
  if (u.nt >= TCAP) { u.flags |= FLAG_TW_OVERFLOW; return FC_CAP; }
  if (x.hl == 0) {
    S.tInf[u.nt] = tw_pack(cell, t, 0, x.ep, x.ep);
    S.tCd[u.nt] = 0.0;
    h_set_tower(S, cell, tw_nib(0, t));
  }
  u.nt += 1;
  u.cost_def = dsub(u.cost_def, price);                   // :238
  u.cells_dirty = true;
  u.tw_dirty = true;
  wsync();
  h_diamond(S, x, cell, +1);                              // :239-245
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int h_find_tower(HalfBoard<NC>& S, const HU& u, const HCtx& x, int cell) {
  const bool hit = x.hl < u.nt && (int)(S.tInf[x.hl] & 0xfffu) == cell;
  const uint32_t m = hballot(hit, x.h);
  return m ? ctz32(m) : -1;
}

template <int NC>
__device__ __forceinline__ int h_tower_lvup(HalfBoard<NC>& S, HU& u, const HCtx& x, int cell) {
  const int k = h_find_tower(S, u, x, cell);
  if (k < 0) return FC_TARGET;                            // :269-271
  const uint32_t ti = S.tInf[k];
  const int t = (ti >> 12) & 3, lv = (ti >> 14) & 1;
  if (lv >= x.C.max_tower_lv) return FC_LVMAX;            // :252
  const double price = x.C.t_price[t][lv + 1];            // :256
  if (u.cost_def < price) return FC_COST;
  wsync();
  if (x.hl == 0) {
    S.tInf[k] = tw_pack(cell, t, lv + 1, tw_ec(ti), x.ep);
    h_set_tower(S, cell, tw_nib(lv + 1, t));
  }
  u.cost_def = dsub(u.cost_def, price);                   // :266
  u.tw_dirty = true;
  wsync();
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int h_tower_destruct(HalfBoard<NC>& S, HU& u, const HCtx& x, int cell) {
  const int k = h_find_tower(S, u, x, cell);
  if (k < 0) return FC_TARGET;                            // :291-293
  const uint32_t ti = S.tInf[k];
  const int t = (ti >> 12) & 3, lv = (ti >> 14) & 1;
  // Tower.cost: tower_cost[t][0] when built, + tower_attack_interval[t][1] at the upgrade
  double value = hcaptured(x, tw_ec(ti), [&](const TdDevCfg& c) { return c.t_price[t][0]; });
  if (lv >= 1) value = dadd(value, hcaptured(x, tw_eu(ti), [&](const TdDevCfg& c) { return c.t_addcost[t][lv]; }));
  u.cost_def = dadd(u.cost_def, dmul(value, x.C.destruct_return));  // :276
  u.cost_def = pymin(u.cost_def, u.max_cost);                      // :277
  u.cells_dirty = true;
  u.tw_dirty = true;
  // towers.remove(t): the order of the rest is kept (:278)
  uint32_t vi = 0;
  double vc = 0.0;
  const int j = x.hl;
  if (j >= k && j + 1 < u.nt) { vi = S.tInf[j + 1]; vc = S.tCd[j + 1]; }
  wsync();
  if (j >= k && j + 1 < u.nt) { S.tInf[j] = vi; S.tCd[j] = vc; }
  if (x.hl == 0) h_set_tower(S, cell, 0u);
  u.nt -= 1;
  wsync();
  h_diamond(S, x, cell, -1);                              // :281-287
  return FC_OK;
}

template <int NC>
__device__ __forceinline__ int h_defender_op(HalfBoard<NC>& S, HU& u, const HCtx& x, int op, int cell) {
  if (op < 4) return h_tower_build(S, u, x, op, cell);
  if (op == 4) return h_tower_lvup(S, u, x, cell);
  return h_tower_destruct(S, u, x, cell);
}

// ---------------------------------------------------------------------------
// attacker: summon_cluster (TDBoard.py:199-224) and random_enemy_lv0/lv1
// ---------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void h_summon_cluster(HalfBoard<NC>& S, HU& u, const HCtx& x, uint32_t types, int road) {
  const TdDevCfg& C = x.C;
  const int lv = u.progress >= C.enemy_upgrade_at ? 1 : 0;  // :201
  const int st = u.start(road);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int t = (int)((types >> (4 * k)) & 0xfu);
    if (t != 4) {                                           // :207-209
      const double cost = C.e_cost[t & 3][lv];
      if (u.cost_atk < cost) {                              // :212-213
      } else if (u.n >= ECAP) {
        u.flags |= FLAG_EN_OVERFLOW;
      } else {
        u.cost_atk = dsub(u.cost_atk, cost);                // :215
        const double lp = C.e_lp[t & 3][lv];
        if (x.hl == 0) {
          S.eLP[u.n] = lp;
          S.eMg[u.n] = 0.0;
          S.eInf[u.n] = en_pack(st, t, lv, 0, x.ep);
        }
        u.n += 1;
      }
    }
  }
}

template <int NC, class Rng>
__device__ __forceinline__ void h_opponent_enemy(HalfBoard<NC>& S, HU& u, const HCtx& x, Rng& R, int difficulty) {
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
  h_summon_cluster(S, u, x, types, road);
  wsync();
  u.atk_cd = x.C.atk_interval;  // the (ok, real) tuple is always truthy
}

// ---------------------------------------------------------------------------
// TDBoard.step (TDBoard.py:295-368): enemy slot s of lane hl is list index hl + 32 s
// ---------------------------------------------------------------------------
constexpr int HS = ECAP / 32;   // enemy slots per lane
constexpr int kHalfFew = 16;    // enemies up to which the towers target in parallel (td_step.hip kFewEnemies)

template <int NC>
__device__ __forceinline__ double h_board_step(HalfBoard<NC>& S, HU& u, const HCtx& x, const StepArgs& a, int b) {
  const TdDevCfg& C = x.C;
  const int L = x.L, hl = x.hl, h = x.h;
  double reward = dadd(0.0, C.reward_time);                 // :298-299
  u.steps += 1;                                             // :300
  u.progress = ddiv((double)u.steps, (double)C.max_episode_steps);  // :301

  // --- stable sort by the f64 key dist - margin (:305): rank = #smaller + #equal-before
  const int n = u.n;
  double lp[HS], mg[HS];
  uint32_t inf[HS];
  bool val[HS];
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    const int i = hl + 32 * s;
    val[s] = i < n;
    lp[s] = val[s] ? S.eLP[i] : 0.0;
    mg[s] = val[s] ? S.eMg[i] : 0.0;
    inf[s] = val[s] ? S.eInf[i] : 0u;
  }
  if (n > 1) {  // (0 or 1 enemies: already sorted)
    double key[HS];
    int rank[HS];
#pragma unroll
    for (int s = 0; s < HS; ++s) {
      key[s] = val[s] ? dsub((double)pk_dist(S.cell[en_cell(inf[s])]), mg[s]) : 0.0;
      rank[s] = 0;
    }
    const int nm = wmax(n);
#pragma unroll
    for (int s2 = 0; s2 < HS; ++s2) {  // enemy j = 32 s2 + jj, read from lane jj of the half
      if (32 * s2 >= nm) break;
      const int jn = nm - 32 * s2 < 32 ? nm - 32 * s2 : 32;
      for (int jj = 0; jj < jn; ++jj) {
        const int j = 32 * s2 + jj;
        const double kj = hru(key[s2], jj, h);
        const bool jv = j < n;
#pragma unroll
        for (int s = 0; s < HS; ++s) {
          const int i = hl + 32 * s;
          if (jv && (kj < key[s] || (kj == key[s] && j < i))) rank[s] += 1;
        }
      }
    }
    wsync();
#pragma unroll
    for (int s = 0; s < HS; ++s)
      if (val[s]) { S.eLP[rank[s]] = lp[s]; S.eMg[rank[s]] = mg[s]; S.eInf[rank[s]] = inf[s]; }
    wsync();
#pragma unroll
    for (int s = 0; s < HS; ++s) {
      const int i = hl + 32 * s;
      lp[s] = val[s] ? S.eLP[i] : 0.0;
      mg[s] = val[s] ? S.eMg[i] : 0.0;
      inf[s] = val[s] ? S.eInf[i] : 0u;
    }
  }

  HSTAMP(3);
  // --- towers fire in list order (:306-313); dead enemies stay targetable.  Tower k
  // lives in lane k of the half (cool-down in a register).
  double tcd = hl < u.nt ? S.tCd[hl] : 0.0;
  const uint32_t tinf_l = hl < u.nt ? S.tInf[hl] : 0u;
  if (n == 0) {
    if (hl < u.nt) { const double cd = dsub(tcd, 1.0); tcd = cd > 0.0 ? cd : 0.0; }
  } else {
    // each tower's range, interval, attack and splash as it captured them, one tower per
    // lane, into the enemy LP array's LDS (dead between the sorted load and the compaction)
    double* const tp = S.eLP;  // [TCAP][4]
    static_assert(sizeof(S.eLP) >= TCAP * 4 * sizeof(double), "tower table in the enemy LP array");
    if (hl < u.nt) {
      const int tt = (tinf_l >> 12) & 3, tl = (tinf_l >> 14) & 1, te = tw_eu(tinf_l);
      tp[4 * hl + 0] = hcaptured(x, te, [&](const TdDevCfg& c) { return c.t_rge[tt][tl]; });
      tp[4 * hl + 1] = hcaptured(x, te, [&](const TdDevCfg& c) { return c.t_intv[tt][tl]; });
      tp[4 * hl + 2] = hcaptured(x, te, [&](const TdDevCfg& c) { return c.t_atk[tt][tl]; });
      tp[4 * hl + 3] = hcaptured(x, te, [&](const TdDevCfg& c) { return c.t_dmg[tt][tl]; });
    }
    wsync();
    if (n <= kHalfFew) {
      // few enemies: lane k = tower k picks its target in parallel, then the shots land
      // per enemy in tower order (td_step.hip board_step, FEW)
      const bool tk = hl < u.nt;
      const int tt = (int)((tinf_l >> 12) & 3u), tc = (int)(tinf_l & 0xfffu);
      double cd = dsub(tcd, 1.0);                            // :307
      const bool tries = tk && !(cd > 0.0);
      const double rge = tries ? tp[4 * hl] : -1.0;
      int tgt = -1;
      const int jn = wmax(n);
      for (int j = 0; j < jn; ++j) {  // first enemy within range, list order
        const int ec = en_cell(hru(inf[0], j, h));
        if (j < n && tgt < 0 && (double)cheb(ec, tc, L) <= rge) tgt = j;
      }
      const int tgc = en_cell(hshfl(inf[0], tgt < 0 ? 0 : tgt, x.lane));
      const double dr = tt >= 2 && tgt >= 0 ? tp[4 * hl + 3] : -1.0;
      int frz = -1;  // TowerFrozen: the first enemy within splash of the target (:112-132)
      for (int j = 0; j < jn; ++j) {
        const int ec = en_cell(hru(inf[0], j, h));
        if (tt == 3 && j < n && frz < 0 && (double)cheb(tgc, ec, L) <= dr) frz = j;
      }
      if (tgt >= 0) cd = dadd(cd, tp[4 * hl + 1]);          // cd += intv
      if (tries && cd < 0.0) cd = 0.0;                       // :311-312
      if (tk) tcd = cd;
      const uint32_t slow = (uint32_t)C.frozen_time << 16;   // config.frozen_time, read live (:126)
      uint32_t fm = hballot(tgt >= 0, h);                     // the towers that fired, in order
      while (__ballot(fm != 0u)) {
        const bool on = fm != 0u;
        const int k = on ? ctz32(fm) : 0;
        const uint32_t kinf = hrd(tinf_l, k, h);
        const int kt = (int)((kinf >> 12) & 3u);
        const int ktg = (int)hrd((uint32_t)tgt, k, h), kgc = (int)hrd((uint32_t)tgc, k, h);
        const int kfz = (int)hrd((uint32_t)frz, k, h);
        if (on) {
          const double atk = tp[4 * k + 2];
          if (kt <= 1) {  // TowerArrow / TowerMagic (TDElements.py:71-93)
            if (hl == ktg) lp[0] = damage(lp[0], atk, h_e_def(x, inf[0]), kt == 1);
          } else if (kt == 2) {  // TowerBomb splash (:95-110)
            if (val[0] && (double)cheb(kgc, en_cell(inf[0]), L) <= tp[4 * k + 3])
              lp[0] = damage(lp[0], atk, h_e_def(x, inf[0]), false);
          } else if (hl == kfz) {
            lp[0] = damage(lp[0], atk, 0.0, true);
            inf[0] = (inf[0] & 0xff00ffffu) | slow;
          }
          fm &= fm - 1u;
        }
      }
    } else {
      const int ktn = wmax(u.nt);
      for (int k = 0; k < ktn; ++k) {
        const bool kon = k < u.nt;
        double cd = dsub(hru(tcd, k, h), 1.0);                 // :307
        const uint32_t ti = hru(tinf_l, k, h);
        const bool fire = kon && !(cd > 0.0);
        const int tt = (ti >> 12) & 3, tc = ti & 0xfff;
        const double rge = fire ? tp[4 * k] : -1.0;
        uint32_t m[HS];
#pragma unroll
        for (int s = 0; s < HS; ++s) m[s] = hballot(val[s] && (double)cheb(en_cell(inf[s]), tc, L) <= rge, h);
        const bool any = (m[0] | m[1] | m[2] | m[3]) != 0u;
        if (fire && any) {
          const int tgt = m[0] ? ctz32(m[0]) : m[1] ? 32 + ctz32(m[1]) : m[2] ? 64 + ctz32(m[2]) : 96 + ctz32(m[3]);
          cd = dadd(cd, tp[4 * k + 1]);                          // cd += intv
          const double atk = tp[4 * k + 2];
          if (tt <= 1) {  // TowerArrow / TowerMagic (TDElements.py:71-93)
            if (hl == (tgt & 31)) {
#pragma unroll
              for (int s = 0; s < HS; ++s)
                if ((tgt >> 5) == s) lp[s] = damage(lp[s], atk, h_e_def(x, inf[s]), tt == 1);
            }
          } else {
            const int tgc = en_cell(S.eInf[tgt]);  // (the sorted list's cell; a slowdown changes no cell)
            const double dr = tp[4 * k + 3];
            if (tt == 2) {  // TowerBomb splash (:95-110)
#pragma unroll
              for (int s = 0; s < HS; ++s)
                if (val[s] && (double)cheb(tgc, en_cell(inf[s]), L) <= dr)
                  lp[s] = damage(lp[s], atk, h_e_def(x, inf[s]), false);
            } else {  // TowerFrozen: the first enemy within splash of the target (:112-132)
              uint32_t q[HS];
#pragma unroll
              for (int s = 0; s < HS; ++s) q[s] = hballot(val[s] && (double)cheb(tgc, en_cell(inf[s]), L) <= dr, h);
              if (q[0] | q[1] | q[2] | q[3]) {
                const int f = q[0] ? ctz32(q[0]) : q[1] ? 32 + ctz32(q[1]) : q[2] ? 64 + ctz32(q[2]) : 96 + ctz32(q[3]);
                if (hl == (f & 31)) {
                  const uint32_t slow = (uint32_t)C.frozen_time << 16;  // config.frozen_time, read live (:126)
#pragma unroll
                  for (int s = 0; s < HS; ++s)
                    if ((f >> 5) == s) { lp[s] = damage(lp[s], atk, 0.0, true); inf[s] = (inf[s] & 0xff00ffffu) | slow; }
                }
              }
            }
          }
        }
        if (fire && cd < 0.0) cd = 0.0;                      // :311-312
        if (hl == k && kon) tcd = cd;
      }
    }
  }
  if (hl < u.nt) S.tCd[hl] = tcd;
  HSTAMP(4);

  // --- kills (:313-317): every enemy at LP 0 was hit this step
  bool alive[HS];
  int nk = 0;
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    const bool dead = val[s] && lp[s] == 0.0;
    nk += popc32(hballot(dead, h));
    alive[s] = val[s] && !dead;
  }
  reward = dadd(reward, dmul(C.reward_kill, (double)nk));  // :315

  // --- march (:319-344)
  bool leak[HS];
  bool bad = false;
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    leak[s] = false;
    if (!alive[s]) continue;
    const uint32_t e = inf[s];
    const int t = en_type(e), lv = en_lv(e);
    int slow = en_slow(e), cell = en_cell(e);
    const double sp = hcaptured(x, en_ep(e), [&](const TdDevCfg& c) { return c.e_speed[t][lv]; });
    if (slow > 0) { mg[s] = dadd(mg[s], dmul(sp, C.frozen_ratio)); slow -= 1; }
    else mg[s] = dadd(mg[s], sp);
    while (mg[s] >= 1.0) {
      mg[s] = dsub(mg[s], 1.0);
      const int d = pk_dir(S.cell[cell]);
      // map[5] codes (TDBoard.py:319): 0:+c 1:-c 2:+r 3:-r
      const int r = cell / L + (d == 2) - (d == 3), c = cell % L + (d == 0) - (d == 1);
      if (r < 0 || r >= L || c < 0 || c >= L) { bad = true; break; }
      cell = r * L + c;
      if (cell == u.end_cell) { leak[s] = true; break; }
    }
    inf[s] = en_pack(cell, t, lv, slow, en_ep(e));
  }
  if (hballot(bad, h)) u.flags |= FLAG_BAD_MOVE;  // rare and lane-local: folded into the half's copy
  int nl = 0;
#pragma unroll
  for (int s = 0; s < HS; ++s) nl += popc32(hballot(leak[s], h));
  for (int p = 0; p < nl; ++p) {                            // :336-343, in list order
    if (u.base_LP > 0) reward = dsub(reward, C.penalty_leak);
    u.base_LP = u.base_LP - 1 > 0 ? u.base_LP - 1 : 0;
  }
  // --- compact the survivors, list order kept (:316-317, :345-346)
  const uint32_t lt = (1u << hl) - 1u;
  int d0 = 0;
  uint32_t km[HS];
#pragma unroll
  for (int s = 0; s < HS; ++s) km[s] = hballot(alive[s] && !leak[s], h);
  wsync();
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    if (alive[s] && !leak[s]) {
      const int d = d0 + popc32(km[s] & lt);
      S.eLP[d] = lp[s]; S.eMg[d] = mg[s]; S.eInf[d] = inf[s];
    }
    d0 += popc32(km[s]);
  }
  u.n = d0;

  // --- costs (:348-353)
  double rate;
  if (u.progress >= 0.5) rate = C.atk_final_rate;
  else rate = dadd(dmul(C.atk_init_rate, dsub(1.0, u.progress)), dmul(C.atk_final_rate, u.progress));
  u.cost_atk = pymin(dadd(u.cost_atk, rate), u.max_cost);  // self.max_cost (:352-353)
  u.cost_def = pymin(dadd(u.cost_def, C.def_rate), u.max_cost);
  wsync();
  return reward;
}

// enemy_LP planes (TDBoard.py:355-365): per (type, cell) min / max / sum in list order /
// count in numpy float32, owned by the group's first ("head") enemy.
template <int NC>
__device__ __forceinline__ void h_enemy_stats(HalfBoard<NC>& S, const HU& u, const HCtx& x) {
  const int n = u.n, hl = x.hl, h = x.h;
  if (n == 0) return;  // the writer emits zero planes without reading grp
  static_assert((4 * NC) % 16 == 0 && (4 * NC) / 16 <= 32, "grp cleared as one 16-B unit per lane of a half");
  if (hl < 4 * NC / 16)
    reinterpret_cast<uint4*>(&S.grp[0][0])[hl] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t key[HS];
  float r[HS];
  bool val[HS], head[HS];
  float mn[HS], mx[HS], sm[HS];
  int cnt[HS];
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    const int i = hl + 32 * s;
    val[s] = i < n;
    key[s] = 0u;
    r[s] = 0.0f;
    if (val[s]) {
      const uint32_t e = S.eInf[i];
      key[s] = e & 0x3fffu;  // cell | type << 12
      const int t = en_type(e), lv = en_lv(e);
      r[s] = f32(ddiv(S.eLP[i], hcaptured(x, en_ep(e), [&](const TdDevCfg& c) { return c.e_lp[t][lv]; })));  // :358
    }
    head[s] = val[s];
    mn[s] = 1.0f; mx[s] = 0.0f; sm[s] = 0.0f; cnt[s] = 0;
  }
  const int nm = wmax(n);
#pragma unroll
  for (int s2 = 0; s2 < HS; ++s2) {
    if (32 * s2 >= nm) break;
    const int jn = nm - 32 * s2 < 32 ? nm - 32 * s2 : 32;
    for (int jj = 0; jj < jn; ++jj) {
      const int j = 32 * s2 + jj;
      const uint32_t kj = hru(key[s2], jj, h);
      const float rj = hru(r[s2], jj, h);
      const bool jv = j < n;
#pragma unroll
      for (int s = 0; s < HS; ++s) {
        const int i = hl + 32 * s;
        if (jv && val[s] && kj == key[s]) {
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
  }
  const float mcl = (float)x.C.max_cluster_length;
  wsync();
#pragma unroll
  for (int s = 0; s < HS; ++s) {
    const int i = hl + 32 * s;
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

// Broadcast channels (TDBoard.py:115-142), two per lane, and channel 9 by distance.
template <int NC>
__device__ __forceinline__ void h_channel_scalars(HalfBoard<NC>& S, const HU& u, const HCtx& x) {
  const TdDevCfg& C = x.C;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int l = x.hl + 32 * r;
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
  }
  // s[9] = map[4] / (max(map[4]) + 1): an int32 divisor promotes to f64, rounded once (:121)
  if (x.hl <= u.maxdist) S.d9[x.hl] = f32(ddiv((double)x.hl, (double)(u.maxdist + 1)));
  wsync();
}

template <int NC>
__device__ __forceinline__ void h_pack_obs_cells(HalfBoard<NC>& S, const HCtx& x) {
  for (int i = x.hl; i < x.NCr; i += 32) {
    const uint32_t w = S.cell[i];
    S.cell[i] = cell_bits(w, twr_of(w)) | ((uint32_t)cw_dir(w) << 21) | ((uint32_t)cw_dist(w) << 24);
  }
  wsync();
}

template <int NC>
__device__ __forceinline__ void h_store_cells(const HalfBoard<NC>& S, const HU& u, const HCtx& x, const StepArgs& a,
                                              int b) {
  const size_t cb = (size_t)b * x.NCr;
  if (u.cells_dirty)
    for (int i = x.hl; i < x.NCr; i += 32) sst(&a.cells[cb + i], S.cell[i] & ~kTwBits);
}

// Fresh board from a layout record (TDGymBasic.reset :43-53, TDBoard.__init__ :14-79);
// vector loads only (the record may have been published by a concurrently running refill).
template <int NC>
__device__ __forceinline__ void h_reset_board(HalfBoard<NC>& S, HU& u, const HCtx& x, const uint32_t* rec) {
  const TdDevCfg& C = x.C;
  const uint32_t hw = rec[x.hl & (LAYOUT_HDR - 1)];
  for (int i = x.hl; i < x.NCr; i += 32) S.cell[i] = rec[LAYOUT_HDR + i];
  u.num_roads = (int)hru(hw, 1, x.h); u.end_cell = (int)hru(hw, 2, x.h); u.maxdist = (int)hru(hw, 3, x.h);
  u.set_starts(hru(hw, 4, x.h), hru(hw, 5, x.h), hru(hw, 6, x.h));
  u.cost_def = C.def_init_cost; u.cost_atk = C.atk_init_cost;
  u.base_LP = C.base_LP; u.steps = 0; u.progress = 0.0;
  u.max_cost = C.max_cost; u.max_base_LP = C.base_LP;  // TDBoard(max_cost, base_LP) from config at reset
  u.atk_cd = 0; u.def_cd = 0; u.n = 0; u.nt = 0; u.ep_ret = 0.0;
  u.cells_dirty = true;
  u.tw_dirty = true;
  wsync();
}

__device__ __forceinline__ TdHdr h_hdr_of(const HU& u) {
  TdHdr hd;
  hd.cost_def = u.cost_def; hd.cost_atk = u.cost_atk; hd.ep_return = u.ep_ret;
  hd.steps = u.steps; hd.base_LP = u.base_LP; hd.atk_cd = u.atk_cd; hd.def_cd = u.def_cd;
  hd.n_en = u.n; hd.n_tw = u.nt; hd.num_roads = u.num_roads; hd.end_cell = u.end_cell;
  hd.start_cell[0] = u.start(0); hd.start_cell[1] = u.start(1); hd.start_cell[2] = u.start(2);
  hd.maxdist = u.maxdist; hd.flags = u.flags; hd.episodes = u.episodes;
  hd.max_cost = u.max_cost; hd.max_base_LP = u.max_base_LP; hd.format = kHdrFormat;
  return hd;
}

// ---------------------------------------------------------------------------
// load: every input of a board issued at once, then committed to LDS
// ---------------------------------------------------------------------------
constexpr int PF_HALF = 16;  // enemy and tower slots fetched with the header
struct HPrefetch {
  double lp, mg, tcd;
  uint4 c4;
  uint32_t inf, tinf, w, w2;
};

template <int NC>
__device__ __forceinline__ void h_prefetch(HPrefetch& P, const StepArgs& a, int b, int hl) {
  const size_t eb = (size_t)b * ECAP, tb = (size_t)b * TCAP, cb = (size_t)b * NC;
  if (hl < PF_HALF) {
    P.lp = a.en_lp[eb + hl];
    P.mg = a.en_mg[eb + hl];
    P.inf = a.en_inf[eb + hl];
    P.tcd = a.tw_cd[tb + hl];
    P.tinf = a.tw_inf[tb + hl];
  }
  P.c4 = hl < NC / 4 ? reinterpret_cast<const uint4*>(a.cells + cb)[hl] : uint4{0u, 0u, 0u, 0u};
  const uint32_t* src;
  if (hl < 24) src = reinterpret_cast<const uint32_t*>(a.hdr + b) + hl;  // TdHdr words
  else if (hl < 26) src = reinterpret_cast<const uint32_t*>(a.def_act + b) + (hl - 24);
  else src = nullptr;
  P.w = src ? *src : 0u;
  P.w2 = hl < HOT_WORDS ? a.opp_hot[(size_t)b * HOT_WORDS + hl] : 0u;
}

constexpr int STG_ACT = 24, STG_HOT = 26;

template <int NC>
__device__ __forceinline__ void h_load_board(HalfBoard<NC>& S, HU& u, const HCtx& x, const StepArgs& a, int b,
                                             const HPrefetch& P) {
  const int hl = x.hl;
  if (hl < STG_HOT) S.stg[hl] = P.w;
  if (hl < HOT_WORDS) S.stg[STG_HOT + hl] = P.w2;
  if (hl < NC / 4) reinterpret_cast<uint4*>(S.cell)[hl] = P.c4;
  wsync();
  static_assert(STG_HOT + HOT_WORDS <= 48, "staging words");
  const TdHdr H = *reinterpret_cast<const TdHdr*>(S.stg);
  u.cost_def = H.cost_def; u.cost_atk = H.cost_atk; u.ep_ret = H.ep_return;
  u.steps = H.steps; u.base_LP = H.base_LP; u.atk_cd = H.atk_cd; u.def_cd = H.def_cd;
  u.n = H.n_en; u.nt = H.n_tw; u.num_roads = H.num_roads; u.end_cell = H.end_cell;
  u.set_starts(H.start_cell[0], H.start_cell[1], H.start_cell[2]);
  u.maxdist = H.maxdist; u.flags = H.flags; u.episodes = H.episodes;
  u.max_cost = H.max_cost; u.max_base_LP = H.max_base_LP;
  u.progress = ddiv((double)u.steps, (double)x.C.max_episode_steps);
  u.cells_dirty = false;
  u.tw_dirty = false;
  const size_t eb = (size_t)b * ECAP;
  if (hl < u.n && hl < PF_HALF) { S.eLP[hl] = P.lp; S.eMg[hl] = P.mg; S.eInf[hl] = P.inf; }
  for (int i = PF_HALF + hl; i < u.n; i += 32) { S.eLP[i] = a.en_lp[eb + i]; S.eMg[i] = a.en_mg[eb + i]; S.eInf[i] = a.en_inf[eb + i]; }
  uint32_t tinf = P.tinf;
  if (hl < u.nt) {
    double tcd = P.tcd;
    if (hl >= PF_HALF) {
      const size_t tb = (size_t)b * TCAP;
      tcd = a.tw_cd[tb + hl];
      tinf = a.tw_inf[tb + hl];
    }
    S.tCd[hl] = tcd;
    S.tInf[hl] = tinf;
  }
  wsync();
  if (hl < u.nt)  // (one tower per cell: no two lanes share a word)
    S.cell[tinf & 0xfffu] |= tw_nib((int)((tinf >> 14) & 1u), (int)((tinf >> 12) & 3u));
  wsync();
}

// ---------------------------------------------------------------------------
// one board's step (td_step.hip step_board, MODE_DEF, small-batch schedule), in two parts
// around the pair's early observation pass
// ---------------------------------------------------------------------------
// What a board's step carries from part A to part B.
struct HStep {
  HU u;
  int fail_def;
  int64_t real_def;
  bool live;     // the board has a layout (else: never reset, nothing stepped)
  bool enemies;  // enemies on the board after the actions (the enemy planes and channel 5 wait for the step)
};

// The broadcast channels as they will read after the step, computed before it: the step
// changes the costs only by its closing cost update (TDBoard.py:348-353), which depends on
// nothing the step decides, and base_LP only when an enemy leaks (channel 5: exact for a
// board without enemies; written late for the others).
template <int NC>
__device__ __forceinline__ void h_early_scalars(HalfBoard<NC>& S, const HU& u, const HCtx& x) {
  const TdDevCfg& C = x.C;
  HU v = u;
  v.steps = u.steps + 1;
  v.progress = ddiv((double)v.steps, (double)C.max_episode_steps);
  double rate;
  if (v.progress >= 0.5) rate = C.atk_final_rate;
  else rate = dadd(dmul(C.atk_init_rate, dsub(1.0, v.progress)), dmul(C.atk_final_rate, v.progress));
  v.cost_atk = pymin(dadd(u.cost_atk, rate), u.max_cost);
  v.cost_def = pymin(dadd(u.cost_def, C.def_rate), u.max_cost);
  h_channel_scalars(S, v, x);
}

// Part A: load, cool-downs, the defender's action and the built-in attacker; the cell words
// packed for the observation and the broadcast channels as they will read after the step.
template <int NC, int LT>
__device__ __forceinline__ void h_step_a(HalfBoard<NC>& S, const HCtx& x, const StepArgs& a, int b, const HPrefetch& P,
                                         HStep& T, HalfMt& R) {
  const TdDevCfg& C = x.C;
  const int hl = x.hl;
  HU& u = T.u;
  HSTAMP(0);
  h_load_board(S, u, x, a, b, P);
  const int64_t act_in = (int64_t)(((uint64_t)S.stg[STG_ACT + 1] << 32) | S.stg[STG_ACT]);
  // the opponent stream: position, lazy-twist boundary and the pre-drawn outputs (used
  // only when they start at the current position) from the hot record
  R.w = a.opp_mt + (size_t)b * OPP_WORDS;
  R.pos = S.stg[STG_HOT + 0];
  R.tw = S.stg[STG_HOT + 1];
  R.cn = S.stg[STG_HOT + 3] == R.pos ? S.stg[STG_HOT + 2] : 0u;
  R.cbase = R.pos;
  R.cache = hl < HOT_CACHE ? S.stg[STG_HOT + 4 + hl] : 0u;
  R.early_issue();
  HSTAMP(1);
  T.live = u.num_roads >= 1 && u.num_roads <= 3;
  T.enemies = false;
  T.fail_def = 0;
  T.real_def = (int64_t)6 * x.NCr;
  if (!T.live) {
    // never reset (its road generation failed): nothing to step.  Every output defined
    // (done, no reward, no action taken); the image is cleared so that the pair's writer
    // emits an all-zero observation for this board.
    if (hl == 0) {
      a.hdr[b].flags = u.flags | FLAG_NO_LAYOUT;
      a.reward[b] = 0.0;
      a.done[b] = 1;
      if (a.win) a.win[b] = -1;
      if (a.allow_next) a.allow_next[b] = 0;
      if (a.cooldowns) a.cooldowns[b] = 0;
      if (a.fail_def) a.fail_def[b] = 0;
      if (a.real_def) a.real_def[b] = (int64_t)6 * x.NCr;
      if (a.ep_return) a.ep_return[b] = 0.0;
      if (a.ep_len) a.ep_len[b] = 0;
    }
    for (int i = hl; i < x.NCr; i += 32) S.cell[i] = 0u;
    for (int i = hl; i < 48; i += 32) S.chv[i] = 0.0f;
    if (hl == 0) S.d9[0] = 0.0f;
    wsync();
    return;
  }
  u.atk_cd = u.atk_cd - 1 > 0 ? u.atk_cd - 1 : 0;
  u.def_cd = u.def_cd - 1 > 0 ? u.def_cd - 1 : 0;
  const int64_t empty_def = (int64_t)6 * x.NCr;
  // ---- defender (TDDefense.py:40-77): op = act // L^2, row, column
  {
    int64_t act = act_in;
    if (act < 0 || act > empty_def) { u.flags |= FLAG_BAD_ACTION; act = empty_def; }
    if (u.def_cd == 0 && act != empty_def) {
      const int a32 = (int)act;
      const int op = a32 / (LT * LT);
      T.fail_def = h_defender_op(S, u, x, op, a32 - op * LT * LT);
      if (T.fail_def == FC_OK) { u.def_cd = C.def_interval; T.real_def = act; }
    }
  }
  HSTAMP(11);
  // ---- attacker: the built-in opponent
  h_with_opp_rng(a, b, x, R, [&](auto& G) { h_opponent_enemy(S, u, x, G, a.difficulty); });
  HSTAMP(12);
  // the towers and map[6] are final: cell words back to HBM if they changed, then packed
  h_store_cells(S, u, x, a, b);
  u.cells_dirty = false;
  h_pack_obs_cells(S, x);
  T.enemies = u.n > 0;
  h_early_scalars(S, u, x);
}

// Part B: TDBoard.step, done, auto-reset, the board's state and outputs, the group
// statistics and the final broadcast channels.  Returns whether the board was reset.
template <int NC, int LT>
__device__ __forceinline__ bool h_step_b(HalfBoard<NC>& S, const HCtx& x, const StepArgs& a, int b, HStep& T,
                                         HalfMt& R) {
  const TdDevCfg& C = x.C;
  const int hl = x.hl;
  HU& u = T.u;
  uint32_t* const hot = a.opp_hot + (size_t)b * HOT_WORDS;
  HSTAMP(2);
  double reward = h_board_step(S, u, x, a, b);
  R.early_finish();  // the next step's pre-drawn opponent outputs
  const bool done = (u.base_LP <= 0) || (u.steps >= C.max_episode_steps);  // :384-385
  u.ep_ret = dadd(u.ep_ret, reward);
  const int ep_steps = u.steps;
  const int8_t win = done ? (u.base_LP > 0 ? 1 : 0) : -1;
  const uint8_t allow = (uint8_t)((u.atk_cd <= 1 ? 1 : 0) | (u.def_cd <= 1 ? 2 : 0));
  const int acd = u.atk_cd < 15 ? u.atk_cd : 15, dcd = u.def_cd < 15 ? u.def_cd : 15;
  const uint8_t cool = (uint8_t)(acd | (dcd << 4));
  const double ep_ret = u.ep_ret;
  if (done) u.episodes += 1;
  bool was_reset = false;
  uint32_t lay_head = 0;
  if (done && a.autoreset && !a.opp_np) {  // random_agent=False: td_autoreset_kernel follows
    // the staged layout: relaxed sc1 poll of its tag, then one agent-scope acquire
    lay_head = a.lay_head[b];
    const uint32_t* rec = a.nxt + ((size_t)b * NSLOT + lay_head % NSLOT) * a.slot_words;
    bool ready = ld_relaxed(rec) == slot_tag(lay_head);
    if (!ready) ready = take_dry_ring(a, b, lay_head, &u.flags);
    if (ready) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      h_reset_board(S, u, x, rec);
      was_reset = true;
    } else {
      u.flags |= FLAG_NO_LAYOUT;  // 65 failing draws in a row (the reference raises): the board keeps its episode
    }
  }
  {  // the enemy list back to HBM (a reset board has none)
    const size_t eb = (size_t)b * ECAP;
    for (int i = hl; i < u.n; i += 32) {
      sst(&a.en_lp[eb + i], S.eLP[i]);
      sst(&a.en_mg[eb + i], S.eMg[i]);
      sst(&a.en_inf[eb + i], S.eInf[i]);
    }
  }
  if (hl == 0) {
    if (was_reset) st_relaxed(a.lay_head + b, lay_head + 1u);  // the record is in LDS: its slot may be redrawn
    sst(&hot[0], R.pos);
    sst(&hot[1], R.tw);
    sst(&hot[2], R.cn);
    sst(&hot[3], R.cbase);
  }
  if (hl < HOT_CACHE) sst(&hot[4 + hl], R.cache);
  HSTAMP(5);
  h_enemy_stats(S, u, x);
  HSTAMP(13);
  h_channel_scalars(S, u, x);
  HSTAMP(14);
  if (was_reset) {  // the new episode's layout
    h_store_cells(S, u, x, a, b);
    h_pack_obs_cells(S, x);
  }
  if (hl == 0) a.hdr[b] = h_hdr_of(u);
  {
    const size_t tb = (size_t)b * TCAP;
    if (hl < u.nt) {
      sst(&a.tw_cd[tb + hl], S.tCd[hl]);
      if (u.tw_dirty) sst(&a.tw_inf[tb + hl], S.tInf[hl]);
    }
  }
  if (hl == 0) {
    sst(&a.reward[b], reward);
    sst(&a.done[b], (uint8_t)(done ? 1 : 0));
    if (a.win) sst(&a.win[b], win);
    if (a.allow_next) sst(&a.allow_next[b], allow);
    if (a.cooldowns) sst(&a.cooldowns[b], cool);
    if (a.fail_def) sst(&a.fail_def[b], (int32_t)T.fail_def);
    if (a.real_def) sst(&a.real_def[b], T.real_def);
    if (a.ep_return) sst(&a.ep_return[b], ep_ret);
    if (a.ep_len) sst(&a.ep_len[b], (int32_t)ep_steps);
    if (done && a.last_ep) {  // the board's last finished episode (td_episode_records)
      td_episode_record r;
      r.ret = ep_ret;
      r.length = ep_steps;
      r.win = win;
      a.last_ep[b] = r;
    }
    if (done && a.ep_stats) {  // device-side episode accounting (td_episode_stats)
      atomicAdd(&a.ep_stats[0], 1.0);
      atomicAdd(&a.ep_stats[1], ep_ret);
    }
  }
  T.u.n = u.n;
  return was_reset;
}

// ---------------------------------------------------------------------------
// the pair's observation: one contiguous stretch of 2 x 45 x L x L float32
// ---------------------------------------------------------------------------
// Window classes of the pair's stream (td_step.hip ObsWinTab for a two-board stretch):
// store k covers 16-B units [64k - mis, 64k - mis + 64) of the pair, mis = the units of
// the 128-B line before it; bits 0-1 the class of the channels the window covers in
// either board (0 binary planes only, 1 broadcast only, 2 enemy planes only, 3 mixed),
// bit 2 a line shared with a neighbouring pair.
template <int LT>
struct PairWinTab {
  static constexpr int Q = LT * LT / 4, N4 = NCH * Q, N2 = 2 * N4, K = (N2 + 7 + 63) / 64, W = (K + 7) / 8;
  struct T { uint32_t w[8][W]; };
  static constexpr uint32_t cls(int mis, int k) {
    const int head = mis ? 8 - mis : 0, tail = ((N2 + mis) & ~7) - mis;
    const int ulo = 64 * k - mis, uhi = ulo + 63;
    const int lo = ulo < 0 ? 0 : ulo, hi = uhi > N2 - 1 ? N2 - 1 : uhi;
    uint64_t chm = 0;
    for (int u = lo; u <= hi; ++u) chm |= 1ull << ((u % N4) / Q);
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

// Channels the step itself decides for a board with enemies: base_LP (5) and the enemy_LP
// planes (25-40).  Everything else of the observation is final once the actions are.
__device__ __forceinline__ bool late_channel(int ch) { return ch == 5 || (unsigned)(ch - 25) < 16u; }

// What the pair writer knows of each board: any[] enemies after the step (the group
// statistics are in LDS), en[] enemies after the actions (late channels), rs[] reset.
struct PairFlags {
  bool any0, any1, en0, en1, rs0, rs1;
};

// The pair's (2, 45, L, L) observation in 128-B-aligned 1-KB windows by the whole wave
// (td_step.hip write_obs_lines over two board images): lane unit i of the stretch is
// board i / N4's unit i % N4 (channel, quad of 4 cells).  nunits: N4 when the pair has
// one board (an odd batch's last wave: its units beyond are dropped by the buffer range).
// PASS 0: every unit; 1 (early, before the board steps): every unit but the late channels
// of a board with enemies; 2 (late): those, and every unit of a board that was reset.
// Windows no lane of which stores in this pass are skipped.  wt: every line write-through
// (the batch's observation fits the Infinity Cache); else whole lines non-temporal and the
// two lines shared with neighbouring pairs as plain write-back (edge_wt 2) or
// write-through (1) stores.
template <int NC, int LT, int PASS, int G = 4>
__device__ __forceinline__ void write_obs_pair(const PairSmem<NC>& SP, int lane, float* out, int nunits,
                                               const PairFlags& f, bool wt, int edge_wt) {
  static_assert(LT >= 8, "a 128-B line spans at most two channel planes");
  using Tab = PairWinTab<LT>;
  constexpr int Q = Tab::Q, N4 = Tab::N4, N2 = Tab::N2, K = Tab::K;
  constexpr uint32_t OOB = 0x80000000u;  // beyond the buffer's num_records: store dropped
  constexpr int BSZ = (int)sizeof(HalfBoard<NC>);
  const char* const sb = reinterpret_cast<const char*>(&SP.hb[0]);
  const HalfBoard<NC>& S0 = SP.hb[0];
  const char* const s0 = reinterpret_cast<const char*>(&S0);
  const int o_cell = (int)(reinterpret_cast<const char*>(S0.cell) - s0);
  const int o_grp = (int)(reinterpret_cast<const char*>(&S0.grp[0][0]) - s0);
  const int o_chv = (int)(reinterpret_cast<const char*>(S0.chv) - s0);
  const int o_d9 = (int)(reinterpret_cast<const char*>(S0.d9) - s0);
  const int o_gst = (int)(reinterpret_cast<const char*>(&S0.gst[0][0]) - s0);
  const int mis = (int)((reinterpret_cast<uintptr_t>(out) >> 4) & 7u);
  const int head = mis ? 8 - mis : 0, tail = ((N2 + mis) & ~7) - mis;  // [0, head), [tail, N2): shared lines
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, nunits * 16, 0x00020000);
  const int i0 = lane - mis;
  auto wclass = [&](int k) { return (Tab::tab.w[mis][k >> 3] >> (4 * (k & 7))) & 7u; };
  auto unit = [&](int i, uint32_t wc) { return (wc & 4u) ? (i < 0 ? 0 : (i > N2 - 1 ? N2 - 1 : i)) : i; };
  // this pass's units of a lane (board bd, channel ch)
  auto wanted = [&](int bd, int ch) {
    if constexpr (PASS == 0) return true;
    const bool en = bd ? f.en1 : f.en0;
    if constexpr (PASS == 1) return !(en && late_channel(ch));
    const bool r = bd ? f.rs1 : f.rs0;
    return r || (en && late_channel(ch));
  };
  for (int k0 = 0; k0 < K; k0 += G) {
    uint4 A[G];
    uint32_t W[G];
    uint32_t skip = 0;  // wave-uniform: windows of the group with no unit to store in this pass
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int k = k0 + j;
      if (K % G == 0 || k < K) {
        const uint32_t wc = wclass(k);
        const int i = unit(i0 + 64 * k, wc);
        const int bd = i >= N4 ? 1 : 0, ib = i - bd * N4;
        const int ch = ib / Q, q = ib - ch * Q;
        if (PASS != 0 && !__ballot(wanted(bd, ch))) { skip |= 1u << j; continue; }
        const int base = bd * BSZ;
        A[j] = *reinterpret_cast<const uint4*>(sb + base + o_cell + 16 * q);
        if ((wc & 3u) == 1) {
          W[j] = *reinterpret_cast<const uint32_t*>(sb + base + o_chv + 4 * ch);
        } else if ((wc & 3u) >= 2) {
          const int e = ch - 25;
          const int wa = base + o_grp + (e & 3) * NC + 4 * q, wb = base + o_chv + 4 * ch, m = -(int)((unsigned)e < 16u);
          W[j] = *reinterpret_cast<const uint32_t*>(sb + (wb ^ ((wa ^ wb) & m)));
        } else {
          W[j] = 0u;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int k = k0 + j;
      if (!(K % G == 0 || k < K) || ((skip >> j) & 1u)) continue;
      const uint32_t wc = wclass(k);
      const bool edge = (wc & 4u) != 0;
      const int i = i0 + 64 * k;
      const int iu = unit(i, wc);
      const int bd = iu >= N4 ? 1 : 0, ib = iu - bd * N4, ch = ib / Q;
      const int base = bd * BSZ;
      const bool anyE = bd ? f.any1 : f.any0;
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
      } else if (isbin) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (float)((a4[c] >> (ch & 31)) & 1u);
      } else if (isd9) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const float*>(sb + base + o_d9 + 4 * (int)(a4[c] >> 24));
      } else if (isen && anyE) {  // enemy stats by the cell's group head
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t g = (W[j] >> (8 * c)) & 0xffu;
          const float fv = *reinterpret_cast<const float*>(sb + base + o_gst + 16 * (int)(g & 0x7fu) + 4 * ((e >> 2) & 3));
          v[c] = g != 0xffu ? fv : 0.0f;
        }
      } else {
        const float cv = isen ? 0.0f : __uint_as_float(W[j]);
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = cv;
      }
      const f32x4 val = f32x4{v[0], v[1], v[2], v[3]};
      // i < 0 or i >= nunits: out of range already; a unit of another pass: dropped
      const uint32_t off = wanted(bd, ch) ? (uint32_t)i * 16u : OOB;
      if (wt) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, off, 0, 16 /* sc1 */);
      } else if (!edge) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, off, 0, 2 /* nt */);
      } else {
        const bool shared = i < head || i >= tail;
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
// the kernel: wave w steps boards 2p and 2p + 1 of its XCD-mapped pair p
// ---------------------------------------------------------------------------
// 16 waves per CU (LDS: 8.9 KB per pair), so 4,096 waves = 8,192 boards run as one round;
// up to 128 VGPRs per lane.  Where the batch's observation fits the Infinity Cache
// (write-through stores) the pair writes all it can right after the actions -- the whole
// observation of a board without enemies -- so the store stream drains while the boards
// step (a one-round grid otherwise starts storing only once its first boards finish
// stepping); the channels the step decides follow after it.  Larger batches write each
// pair once, after the step.
template <int LT, int MODE, bool SCAN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void td_step_kernel_half(StepArgs a_) {
  static_assert(LT == 10 && MODE == MODE_DEF && !SCAN, "the half-wave step is built for TD-def discrete at L = 10");
  const StepArgs& a = kargs(a_);
  constexpr int NC = LT * LT;
  __shared__ PairSmem<NC> SP;
  const int npair = (a.B + 1) >> 1;
  if ((int)blockIdx.x >= npair) return;
  const int p = a.xcd_map ? xcd_board((int)blockIdx.x, npair) : (int)blockIdx.x;
  const int lane = (int)threadIdx.x & 63, h = lane >> 5, hl = lane & 31;
  const int b = 2 * p + h;
#ifdef TD_STAMPS
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  static_assert(sizeof(TdDevCfg) % 16 == 0 && sizeof(TdDevCfg) <= 64 * 16, "cfg staging");
  if (lane < (int)(sizeof(TdDevCfg) / 16))
    reinterpret_cast<uint4*>(&SP.cfg)[lane] = reinterpret_cast<const uint4*>(a.cfg)[lane];
  wsync();
  const bool mine = b < a.B;
  const bool two = 2 * p + 1 < a.B;
  constexpr int N4 = NCH * LT * LT / 4;
  float* const out = a.obs + (size_t)2 * p * NCH * NC;
  const int nunits = two ? 2 * N4 : N4;
#ifndef TD_HALF_EARLY  // (temporary A/B macro, round 5: the early observation pass)
#define TD_HALF_EARLY 1
#endif
  const bool early = TD_HALF_EARLY && a.obs_wt != 0;
  const HCtx x{SP.cfg, LT, NC, lane, hl, h, a.cfgs, a.epoch};
  HStep T;
  HalfMt R{nullptr, 0u, 0u, hl, h, lane};
  T.live = false;
  T.enemies = false;
  if (mine) {
    HPrefetch P;
    h_prefetch<NC>(P, a, b, hl);
    h_step_a<NC, LT>(SP.hb[h], x, a, b, P, T, R);
  }
  wsync();
  PairFlags f{false, false, false, false, false, false};
  {
    const uint64_t em = __ballot(T.enemies);
    f.en0 = (em & 1ull) != 0;
    f.en1 = ((em >> 32) & 1ull) != 0;
  }
  if (early) write_obs_pair<NC, LT, 1>(SP, lane, out, nunits, f, true, a.edge_wt);
  bool reset = false;
  if (mine && T.live) reset = h_step_b<NC, LT>(SP.hb[h], x, a, b, T, R);
  wsync();
  {
    const uint64_t am = __ballot(T.live && T.u.n > 0), rm = __ballot(reset);
    f.any0 = (am & 1ull) != 0;
    f.any1 = ((am >> 32) & 1ull) != 0;
    f.rs0 = (rm & 1ull) != 0;
    f.rs1 = ((rm >> 32) & 1ull) != 0;
  }
#ifdef TD_STAMPS
  if (hl == 0 && mine) { HSTAMP_AT(b, 6, __builtin_amdgcn_s_memtime()); HSTAMP_AT(b, 9, rt0); }
#endif
  if (early) write_obs_pair<NC, LT, 2>(SP, lane, out, nunits, f, true, a.edge_wt);
  else write_obs_pair<NC, LT, 0>(SP, lane, out, nunits, f, false, a.edge_wt);
#ifdef TD_STAMPS
  if (hl == 0 && mine) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    HSTAMP_AT(b, 7, t); HSTAMP_AT(b, 8, t); HSTAMP_AT(b, 10, __builtin_amdgcn_s_memrealtime());
  }
#endif
}

bool half_supported(const StepArgs& a) { return a.L == 10 && a.mode == MODE_DEF && !a.multi; }

hipError_t launch_step_half(const StepArgs& a, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  if (!half_supported(a)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((a.B + 1) / 2)), block(64);
  if (ev0) hipExtLaunchKernelGGL((td_step_kernel_half<10, MODE_DEF, false>), grid, block, 0, s, ev0, ev1, 0, a);
  else hipLaunchKernelGGL((td_step_kernel_half<10, MODE_DEF, false>), grid, block, 0, s, a);
  return hipGetLastError();
}

int half_resident_boards(const StepArgs& a, int cus) {
  if (!half_supported(a)) return 0;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, td_step_kernel_half<10, MODE_DEF, false>, 64, 0) != hipSuccess)
    return 0;
  return 2 * n * cus;
}

}  // namespace td
