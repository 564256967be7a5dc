// td_wavegen.h -- create_road_v2 run by a whole wave (WaveRoadGen) over the LDS image
// of one layout draw (LayoutSmem): the device form of td_layout.h RoadGen::draw.
#pragma once
#include "td_layout.h"
#include "td_rng.h"
#include "td_wave.h"

namespace td {

// ---------------------------------------------------------------------------
// episode layouts on the device
// ---------------------------------------------------------------------------
// LDS image of one layout draw: the board's numpy stream, the output record,
// create_road_v2's scratch and the draw's resume state (WaveRoadGen runs on it).
template <int NC>
struct LayoutSmem {
  uint32_t mt[OPP_WORDS];
  uint32_t rec[LAYOUT_HDR + NC];
  uint8_t scratch[14 * NC + 64];
  RoadResume res;
};

// create_road_v2 (TDRoadGen.py:4-199) and TDGymBasic.reset's num_roads draw (:42) run by
// a whole wave: the device form of td_layout.h RoadGen::draw, draw for draw the same
// (both are pinned against the reference's road table).  RoadGen on one lane waited on
// LDS for every stream draw (three dependent words of the lazy twist) and for every
// move (the field byte); here the stream is a window of 64 tempered outputs in a
// register, one per lane, refilled 64 at a time with one LDS round trip, and the field
// / turn maps are bitmaps in registers (lane j holds cells [32j, 32j + 32)), read with
// v_readlane.  Control flow is wave-uniform.  The road lists stay in LDS (the resumable
// state); the main road, its branch points and the stamping of a road onto the record
// run one cell per lane (an accepted road is shorter than 2L <= 64 cells).
// At L <= 11 (at most 128 cells) the hopeless-branch search runs on the field as two
// wave-uniform 64-bit words (SBP): a 128-bit frontier is shifted instead of lane words
// exchanged -- 17.5 k -> 3.7 k cycles per search (r04/s11, probe_draw_parts, 1,024 boards
// at L = 10).  The walks keep the lane-word bitmaps (as scalar words they were slower:
// 6.8 k -> 7.3 k cycles per walk, the refill kernel has no SGPRs to spare).  The refill
// kernel only: the reset kernels have no registers to spare.
constexpr bool kGenSBProof = true;
template <int NC, bool SBP = false>  // SBP: the search on scalar words
struct WaveRoadGen {
  static __device__ __forceinline__ void sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  static constexpr int NW = (NC + 31) / 32;  // bitmap words (at most)
  uint32_t* mt;   // LDS stream words (LazyMt format: [624] position, [625] lazy-twist boundary)
  uint32_t* rec;  // LDS record
  uint32_t* picks;
  uint16_t *r1, *r2, *rb, *mainr;
  uint32_t *fieldw, *rotw;  // the bitmaps' resumable copies in the scratch
  int L, lane;
  uint32_t pos, tw, base, n, win;
  uint32_t field, rot;  // lane j holds cells [32j, 32j + 32)

  // scratch carve for L*L = nc cells: picks u32[nc], r1 / r2 / rb / mainr u16[nc], field / rot
  // u32[(nc + 31) / 32] -- 12 nc + 8 (nc + 31) / 32 <= road_scratch_bytes(L) bytes
  __device__ void carve(uint8_t* sc, int nc) {
    picks = reinterpret_cast<uint32_t*>(sc);
    r1 = reinterpret_cast<uint16_t*>(sc + 4 * nc);
    r2 = r1 + nc; rb = r2 + nc; mainr = rb + nc;
    fieldw = reinterpret_cast<uint32_t*>(sc + 12 * nc);
    rotw = fieldw + (nc + 31) / 32;
  }

  // ---- the numpy-legacy stream (LazyMt semantics, 64 words per refill) ----
  __device__ void refill() {
    if (pos >= (uint32_t)MT_N) { pos = 0; tw = 0; }
    base = pos;
    n = (uint32_t)MT_N - pos < 64u ? (uint32_t)MT_N - pos : 64u;
    const uint32_t q = base + (uint32_t)lane;
    const bool mine = (uint32_t)lane < n, lazy = mine && q >= tw;
    uint32_t y = 0;
    if (mine) {
      y = mt[q];
      if (lazy) {  // new[q] from old[q], old[q + 1] and old[q + 397] / new[q - 227] (< base: done)
        const uint32_t nb = mt[q == MT_N - 1 ? 0u : q + 1u];
        const uint32_t far = mt[q < (uint32_t)(MT_N - MT_M) ? q + MT_M : q - (MT_N - MT_M)];
        const uint32_t yy = (y & 0x80000000u) | (nb & 0x7fffffffu);
        y = far ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
      }
    }
    sync();  // every lane's old words are read before any new word is stored
    if (lazy) mt[q] = y;
    if (base + n > tw) tw = base + n;
    win = mt_temper(y);
  }
  __device__ __forceinline__ uint32_t next() {
    if (pos - base >= n) refill();
    const uint32_t r = rdl(win, (int)(pos - base));
    ++pos;
    return r;
  }
  __device__ int np_randint(int lo, int hi) {  // numpy legacy masked rejection (hi exclusive)
    if (hi <= lo) return lo;
    const uint32_t rng = (uint32_t)(hi - lo - 1);
    if (rng == 0) return lo;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v = next() & mask;
    while (v > rng) v = next() & mask;
    return lo + (int)v;
  }

  // ---- field / turn bitmaps ----
  __device__ __forceinline__ bool bit(uint32_t m, int c) const { return (rdl(m, c >> 5) >> (c & 31)) & 1u; }
  __device__ __forceinline__ uint32_t with(uint32_t m, int c) const {
    return m | (lane == (c >> 5) ? 1u << (c & 31) : 0u);
  }
  __device__ __forceinline__ uint32_t without(uint32_t m, int c) const {
    return m & ~(lane == (c >> 5) ? 1u << (c & 31) : 0u);
  }
  __device__ __forceinline__ bool fbit(int c) const { return bit(field, c); }
  __device__ __forceinline__ bool rbit(int c) const { return bit(rot, c); }
  __device__ __forceinline__ void fset(int c) { field = with(field, c); }
  __device__ __forceinline__ void rset(int c) { rot = with(rot, c); }
  __device__ __forceinline__ void clear_maps() { field = rot = 0u; }
  // The bitmaps from / to their resumable copies (fieldw / rotw: u32 word i = cells [32i, 32i + 32)).
  __device__ __forceinline__ void load_maps(bool resumed) {
    const int nw = (L * L + 31) / 32;
    field = resumed && lane < nw ? fieldw[lane] : 0u;
    rot = resumed && lane < nw ? rotw[lane] : 0u;
  }
  __device__ __forceinline__ void save_maps() {
    const int nw = (L * L + 31) / 32;
    if (lane < nw) {
      fieldw[lane] = field;
      rotw[lane] = rot;
    }
  }
  __device__ __forceinline__ bool inner(int r, int c) const { return r > 0 && r < L - 1 && c > 0 && c < L - 1; }

  // generate_road (TDRoadGen.py:31-119), as RoadGen::walk; *last = the last cell appended
  __device__ int walk(int r0, int c0, int d, uint16_t* out, int* len, int* last) {
    int pr = r0, pc = c0, cnt = 0, pending = 0, loop = 0;
    while (inner(pr, pc) && loop < 100) {
      ++loop;
      const int shape = np_randint(0, 2);
      const int seg = np_randint(L * 3 / 20, L / 4);
      bool cross = false;
      auto run = [&](int k_max, int dd, bool reset_cross) {
        const int dr = dd == 0 ? 1 : dd == 2 ? -1 : 0, dc = dd == 1 ? -1 : dd == 3 ? 1 : 0;  // :15
        for (int k = 0; k < k_max; ++k) {
          pr += dr; pc += dc;
          const int cell = pr * L + pc;
          if (fbit(cell)) { pr -= dr; pc -= dc; cross = true; return; }
          if (reset_cross) cross = false;
          if (lane == 0) out[cnt] = (uint16_t)cell;
          ++cnt;
          fset(cell);
          if (!inner(pr, pc)) return;
        }
      };
      if (shape <= 0) {
        run(seg * 2, d, false);
      } else {
        run(seg, d, false);
        if (!inner(pr, pc)) break;
        int rd;
        if (pending != 0) { rd = pending; pending = 0; }
        else { rd = np_randint(0, 2) * 2 - 1; pending = -rd; }
        rset(pr * L + pc);
        d = (d + 4 + rd) % 4;
        run(seg, d, true);
      }
      if (cross) {  // the free neighbours in direction order, one picked at random
        const uint32_t fm = (fbit((pr + 1) * L + pc) ? 0u : 1u) | (fbit(pr * L + pc - 1) ? 0u : 2u) |
                            (fbit((pr - 1) * L + pc) ? 0u : 4u) | (fbit(pr * L + pc + 1) ? 0u : 8u);
        const int nf = __popc(fm);
        if (nf == 0) { *len = cnt; *last = pr * L + pc; return 0; }
        int pick = np_randint(0, nf);
        uint32_t m = fm;
        while (pick-- > 0) m &= m - 1;
        d = __builtin_ctz(m);
        pending = 0;
        rset(pr * L + pc);
      }
    }
    *len = cnt;
    *last = pr * L + pc;
    return loop >= 100 ? 0 : 1;
  }

  // Bitmap shifts across the lanes' words: cell c -> c + sh (up) / c - sh (down), 0 < sh <= 32.
  // (The shuffles run in every lane: a lane reading a lane that is switched off by a
  // branch around the shuffle would read garbage.)
  __device__ __forceinline__ uint32_t up(uint32_t x, int sh) const {
    const uint32_t t = (uint32_t)__shfl((int)x, lane > 0 ? lane - 1 : 0);
    const uint32_t b = lane > 0 ? t : 0u;
    return sh == 32 ? b : (x << sh) | (b >> (32 - sh));
  }
  __device__ __forceinline__ uint32_t down(uint32_t x, int sh) const {
    const uint32_t t = (uint32_t)__shfl((int)x, lane < 63 ? lane + 1 : 63);
    const uint32_t a = lane < 63 ? t : 0u;
    return sh == 32 ? a : (x >> sh) | (a << (32 - sh));
  }

  // td_layout.h RoadGen::branch_hopeless on the register bitmaps: a breadth-first search
  // from each candidate branch point picks[klo, khi) over the free cells, one frontier
  // bitmap step per walk length; true when no candidate reaches a border cell at
  // Manhattan distance >= 3L/4 from endc in fewer than 2L - (nm - index) cells.
  // 128-bit shifts of a scalar-word bitmap (0 < sh < 64)
  static __device__ __forceinline__ void shl128(uint64_t& lo, uint64_t& hi, int sh) {
    hi = (hi << sh) | (lo >> (64 - sh)); lo <<= sh;
  }
  static __device__ __forceinline__ void shr128(uint64_t& lo, uint64_t& hi, int sh) {
    lo = (lo >> sh) | (hi << (64 - sh)); hi >>= sh;
  }
  // (fs0, fs1: the field as scalar words, converted from the lane words)
  __device__ bool hopeless_sb(int klo, int khi, int nm, int endc, uint64_t fs0, uint64_t fs1) {
    const int ncells = L * L, dmin = L * 3 / 4;
    // masks by ballot: lane l tests cells l and 64 + l
    uint64_t valid[2], first[2], last[2], inn[2], qual[2];
    for (int h = 0; h < 2; ++h) {
      const int c = 64 * h + lane, r = c / L, cc = c - r * L;
      const bool v = c < ncells;
      valid[h] = ballot(v);
      first[h] = ballot(v && cc == 0);
      last[h] = ballot(v && cc == L - 1);
      inn[h] = ballot(v && inner(r, cc));
      qual[h] = ballot(v && !inner(r, cc) && iabs(r - endc / L) + iabs(cc - endc % L) >= dmin);
    }
    sync();
    for (int k = klo; k < khi; ++k) {
      const uint32_t pk = picks[k];
      const int bc = (int)(pk & 0xffffu), lim = 2 * L - (nm - (int)(pk >> 16));
      if (lim <= 0) continue;                      // every walk from here is too long
      if (!inner(bc / L, bc % L)) return false;    // an empty branch: IndexError (:189), not a hang
      uint64_t F0 = bc < 64 ? 1ull << bc : 0ull, F1 = bc < 64 ? 0ull : 1ull << (bc - 64);
      uint64_t V0 = F0 | fs0, V1 = F1 | fs1;
      for (int d = 1; d < lim; ++d) {
        uint64_t a0 = F0 & ~last[0], a1 = F1 & ~last[1];
        shl128(a0, a1, 1);
        uint64_t b0 = F0 & ~first[0], b1 = F1 & ~first[1];
        shr128(b0, b1, 1);
        uint64_t c0 = F0, c1 = F1;
        shl128(c0, c1, L);
        uint64_t e0 = F0, e1 = F1;
        shr128(e0, e1, L);
        const uint64_t N0 = (a0 | b0 | c0 | e0) & valid[0] & ~V0, N1 = (a1 | b1 | c1 | e1) & valid[1] & ~V1;
        if ((N0 & qual[0]) | (N1 & qual[1])) return false;  // a walk could end here
        V0 |= N0; V1 |= N1;
        F0 = N0 & inn[0]; F1 = N1 & inn[1];
        if (!(F0 | F1)) break;
      }
    }
    return true;
  }
  __device__ bool hopeless(int klo, int khi, int nm, int endc) {
    if constexpr (NC <= 128 && SBP) {
      // the lane-word field as two scalar words (lane l: cells l and 64 + l), then the
      // scalar search: 4.7x faster than the lane-word search (r04/s11 probe_draw_parts)
      const uint32_t w0 = (uint32_t)__shfl((int)field, lane >> 5), w1 = (uint32_t)__shfl((int)field, 2 + (lane >> 5));
      return hopeless_sb(klo, khi, nm, endc, ballot(((w0 >> (lane & 31)) & 1u) != 0u),
                         ballot(((w1 >> (lane & 31)) & 1u) != 0u));
    }
    const int ncells = L * L, dmin = L * 3 / 4;
    uint32_t valid = 0, first = 0, last = 0, inn = 0, qual = 0;
    for (int i = 0; i < 32; ++i) {
      const int c = 32 * lane + i, r = c / L, cc = c - r * L;
      if (c >= ncells) break;
      const uint32_t m = 1u << i;
      valid |= m;
      if (cc == 0) first |= m;
      if (cc == L - 1) last |= m;
      if (inner(r, cc)) inn |= m;
      else if (iabs(r - endc / L) + iabs(cc - endc % L) >= dmin) qual |= m;
    }
    sync();
    for (int k = klo; k < khi; ++k) {
      const uint32_t pk = picks[k];
      const int bc = (int)(pk & 0xffffu), lim = 2 * L - (nm - (int)(pk >> 16));
      if (lim <= 0) continue;                      // every walk from here is too long
      if (!inner(bc / L, bc % L)) return false;    // an empty branch: IndexError (:189), not a hang
      uint32_t F = lane == (bc >> 5) ? 1u << (bc & 31) : 0u;
      uint32_t V = F | field;
      for (int d = 1; d < lim; ++d) {
        const uint32_t N = (up(F & ~last, 1) | down(F & ~first, 1) | up(F, L) | down(F, L)) & valid & ~V;
        if (ballot((N & qual) != 0u)) return false;  // a walk could end here
        V |= N;
        F = N & inn;
        if (!ballot(F != 0u)) break;
      }
    }
    return true;
  }

  // clean_up (TDRoadGen.py:121-124): field and turn marks of the road's cells cleared
  __device__ void erase(const uint16_t* road, int cnt) {
    sync();
    for (int i0 = 0; i0 < cnt; i0 += 64) {
      const uint32_t cv = i0 + lane < cnt ? road[i0 + lane] : 0u;
      const int m = cnt - i0 < 64 ? cnt - i0 : 64;
      for (int i = 0; i < m; ++i) {
        const int c = (int)rdl(cv, i);
        field = without(field, c);
        rot = without(rot, c);
      }
    }
  }

  // One road onto the record (TDBoard.py:38-59): lane k < tot holds cell k (`cv`).
  __device__ void stamp(uint32_t cv, int tot, int ri, uint32_t* maxdist) {
    uint32_t* cw = rec + LAYOUT_HDR;
    const int p = (int)cv;
    const int pn = __shfl((int)cv, lane + 1 < 64 ? lane + 1 : 63);
    sync();
    if (lane < tot) {
      uint32_t w = cw[p] | 1u | (1u << (1 + ri));
      w = (w & 0x00ffffffu) | (1u << 24);
      w = (w & ~(0xffu << 16)) | ((uint32_t)(tot - 1 - lane) << 16);
      if (lane < tot - 1) {
        const int dr = pn / L - p / L, dc = pn % L - p % L;
        const uint32_t dir = dr == 0 ? (dc == 1 ? 0u : 1u) : (dr == 1 ? 2u : 3u);
        w = (w & ~(3u << 8)) | (dir << 8);
      }
      cw[p] = w;
    }
    // (readfirstlane: written as a plain if, the update was merged into the join of the
    // lane < tot branch above and read as divergent; every value the draw's loop carries
    // then followed -- the stream position and the draw's state in VGPRs behind exec-masked
    // branches, 6.7 k cycles per walk in r04/s12)
    *maxdist = __builtin_amdgcn_readfirstlane((uint32_t)(tot - 1) > *maxdist ? (uint32_t)(tot - 1) : *maxdist);
    sync();
  }

  __device__ int fail(RoadResume& st, int status) {
    sync();
    if (lane == 0) { rec[0] = 0; rec[1] = st.nr; rec[7] = (uint32_t)status; }
    st.phase = RP_NEW;
    return status;
  }

  static __device__ __forceinline__ int iabs(int x) { return x < 0 ? -x : x; }

  // RoadGen::draw: the same state machine over the same RoadResume (st lives in
  // registers, wave-uniform; the caller moves it from / to LDS; pad holds road 1's last
  // cell), written as ONE loop of attempts with one walk, one erase and one stamp for
  // all three retry loops (road 1, road 2, the branches): three inlined walks in nested
  // loops cost the compiler ~135 VGPRs, one ~50.  A failing draw is skipped (restart
  // at RP_NEW with the full budget) up to `retries` times, as the auto-reset loops do;
  // the last status is returned.
  __device__ int draw(RoadResume& st, int budget0, int max_attempts, int retries = 0) {
    int budget = budget0, status = ROAD_OK;
    for (;;) {
      if (st.phase == RP_NEW) {
        st.nr = (uint32_t)np_randint(1, 4);  // TDGymBasic.reset :42
        const int nr = (int)st.nr;
        if (L < 4 || L > MAX_L || nr < 1 || nr > 3) { status = ROAD_ERR_ARGS; goto failed; }
        if (L / 4 <= L * 3 / 20) { status = ROAD_ERR_RANDINT; goto failed; }  // segment randint raises (:41)
        clear_maps();
        const int lo = L / 3, hi = (L * 2 + 2) / 3;
        st.cr = (uint32_t)np_randint(lo, hi);
        st.cc = (uint32_t)np_randint(lo, hi);
        fset((int)(st.cr * L + st.cc));
        st.d0 = (uint32_t)np_randint(0, 4);
        st.phase = RP_ROAD1; st.att = 0;
      }
      if (st.phase == RP_BRANCH && (int)st.ri >= (int)st.nr) break;  // every road drawn
      {
        // one attempt of the phase's retry loop: center -> end (:128-137), center ->
        // start (:141-155) or a branch (:174-197)
        if ((int)st.att >= max_attempts) { status = ROAD_ERR_BOUND; goto failed; }
        if (budget-- <= 0) return ROAD_PENDING;
        ++st.att;
        const int phase = (int)st.phase, cr = (int)st.cr, cc = (int)st.cc, d0 = (int)st.d0;
        int r0 = cr, c0 = cc, d = d0, k = 0;
        uint16_t* out = r1;
        if (phase == RP_ROAD2) {
          d = (d0 + 2) % 4; out = r2;
        } else if (phase == RP_BRANCH) {
          const int np = (int)st.np, nm = (int)st.nm;
          const int klo = np * 2 / 5, khi = np * 4 / 5;
          if (khi <= klo) { status = ROAD_ERR_RANDINT; goto failed; }
          bool hp = false;
          if (st.att == 1) {
            hp = hopeless(klo, khi, nm, (int)st.endc);
          }
          if (hp) { status = ROAD_ERR_BOUND; goto failed; }  // RoadGen::branch_hopeless
          k = np_randint(klo, khi);
          d = np_randint(0, 4);
          sync();
          const uint32_t pkv = __builtin_amdgcn_readfirstlane(picks[k]);
          r0 = (int)(pkv & 0xffffu) / L; c0 = (int)(pkv & 0xffffu) % L;
          k = (int)(pkv >> 16);
          out = rb;
        }
        int n = 0, e = 0;
        int ok;
        {
          ok = walk(r0, c0, d, out, &n, &e);
        }
        bool accept = ok != 0;
        if (phase == RP_ROAD1) {
          accept = accept && n < L;
        } else if (phase == RP_ROAD2) {
          const int e1 = (int)st.pad;
          accept = accept && (int)st.n1 + n + 1 < L * 2 && iabs(e / L - e1 / L) + iabs(e % L - e1 % L) >= L * 3 / 4;
        } else if (accept) {
          const int nm = (int)st.nm, endc = (int)st.endc;
          accept = n + nm - k < L * 2;
          if (accept && n == 0) { status = ROAD_ERR_EMPTY; goto failed; }
          accept = accept && iabs(e / L - endc / L) + iabs(e % L - endc % L) >= L * 3 / 4;
        }
        if (!accept) {
          erase(out, n);
          continue;
        }
        if (phase == RP_ROAD1) {
          st.n1 = (uint32_t)n; st.pad = (uint32_t)e; st.phase = RP_ROAD2; st.att = 0;
          continue;
        }
        // the road onto the record, one cell per lane (< 2L): main = reversed(road2) +
        // [center] + road1 (:157-158), or road = reversed(branch) + main[k:]
        sync();
        uint32_t cv = 0;
        int tot;
        const int n1 = (int)st.n1;
        if (phase == RP_ROAD2) {
          tot = n1 + n + 1;
          if (lane < n) cv = r2[n - 1 - lane];
          else if (lane == n) cv = (uint32_t)(cr * L + cc);
          else if (lane < tot) cv = r1[lane - n - 1];
          if (lane < tot) mainr[lane] = (uint16_t)cv;
          // branch points (:162-170): cells i with no turn at i and i + 1; a turn at i skips i + 1
          int np = 0;
          uint32_t pk = 0;
          for (int i = 0; i < tot;) {
            const int ci = (int)rdl(cv, i);
            if (!rbit(ci)) {
              if (i < tot - 1 && !rbit((int)rdl(cv, i + 1))) {
                if (lane == np) pk = ((uint32_t)i << 16) | (uint32_t)ci;
                ++np;
              }
              i += 1;
            } else {
              i += 2;
            }
          }
          if (lane < np) picks[lane] = pk;
          for (int i = lane; i < L * L; i += 64) rec[LAYOUT_HDR + i] = 0u;  // map planes from the main road first
          st.nm = (uint32_t)tot; st.np = (uint32_t)np; st.maxdist = 0;
          st.start[0] = rdl(cv, 0); st.start[1] = st.start[2] = 0;
          st.endc = rdl(cv, tot - 1);
        } else {
          tot = n + (int)st.nm - k;
          if (lane < n) cv = rb[n - 1 - lane];
          else if (lane < tot) cv = mainr[k + lane - n];
          sync();
          if (lane < n) rb[lane] = (uint16_t)cv;  // kept reversed, as RoadGen leaves it
          if (st.ri == 1) st.start[1] = rdl(cv, 0);  // (no dynamic index: keeps st in registers)
          else st.start[2] = rdl(cv, 0);
        }
        uint32_t maxdist = st.maxdist;
        {
          stamp(cv, tot, phase == RP_ROAD2 ? 0 : (int)st.ri, &maxdist);
        }
        st.maxdist = maxdist;
        if (phase == RP_ROAD2) { st.phase = RP_BRANCH; st.ri = 1; }
        else ++st.ri;
        st.att = 0;
        continue;
      }
    failed:
      fail(st, status);
      if (retries-- <= 0) return status;
      budget = budget0;  // the next draw of the stream, as a new call would
    }
    const int nr = (int)st.nr;
    uint32_t* cw = rec + LAYOUT_HDR;
    sync();
    if (lane == 0) {
      cw[st.start[0]] |= 1u << 5;
      if (nr > 1) cw[st.start[1]] |= 1u << 6;
      if (nr > 2) cw[st.start[2]] |= 1u << 7;
      cw[st.endc] |= 1u << 4;
      rec[0] = TD_LAYOUT_MAGIC;
      rec[1] = (uint32_t)nr;
      rec[2] = st.endc;
      rec[3] = st.maxdist;
      rec[4] = st.start[0];
      rec[5] = nr > 1 ? st.start[1] : 0u;
      rec[6] = nr > 2 ? st.start[2] : 0u;
      rec[7] = ROAD_OK;
    }
    st.phase = RP_NEW;
    return ROAD_OK;
  }
};

}  // namespace td
