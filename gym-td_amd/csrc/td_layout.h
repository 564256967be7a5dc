// td_layout.h -- per-episode board layout: road generation and the packed
// layout record shared by host and device.
//
// Road generation restates create_road_v2 (TDRoadGen.py:4-199) draw for draw on a
// numpy-legacy MT19937 stream (td_rng.h), so a board seeded with RandomState(s)
// gets the reference's exact roads.  The reference's three ``while not succ``
// loops are unbounded (TDRoadGen.py:129,142,177) and can raise (ValueError at
// :178, IndexError at :189); here every loop is bounded and each failure mode is
// a status code.
//
// Hopeless branch loops.  About 1 % of L = 10 draws reach a branch loop (:177) that no
// attempt can ever finish: the reference spins there forever, and a bounded loop
// burns its whole bound (1,000 walks -- 69 % of all generator walks at L = 10).  The
// loop's field is static (a failed walk is erased), so on its first attempt a
// breadth-first search from every candidate branch point over the free cells decides
// whether ANY walk could end on a border cell at Manhattan distance >= 3L/4 from the
// main road's end within the length bound (a walk moves one cell per appended cell and
// stops on the first border cell, so the search's distance is a lower bound on every
// walk's length).  If none can, the draw fails at once with ROAD_ERR_BOUND, before the
// attempt draws anything (branch_hopeless).  Draws the reference finishes are never
// affected: a search can only prove a failure every attempt would have had.  The
// stream position after such a failed draw is the loop's entry (the bounded loop's
// was 1,000 attempts later); both are restatements of a reference that never returns.
//
// Layout record (uint32 words), the unit the device resets a board from:
//   [0] TD_LAYOUT_MAGIC   [1] num_roads   [2] end cell   [3] max dist
//   [4..6] start cell of road 0..2 (row*L+col)  [7] status
//   [8 + cell] cell word:
//      bits 0-3  road planes (map[0], map[1..3])       TDBoard.py:41-42
//      bit  4    end point                              TDBoard.py:114
//      bits 5-7  start point of road 0..2               TDBoard.py:119-120
//      bits 8-9  next direction map[5] (0:+c 1:-c 2:+r 3:-r)  TDBoard.py:44-54
//      bits 16-23 distance to end map[4]                TDBoard.py:56-59
//      bits 24-31 build-block counter map[6] (=1 on road at reset)  TDBoard.py:43
#pragma once
#include <stdint.h>
#include "td_rng.h"

namespace td {

constexpr uint32_t TD_LAYOUT_MAGIC = 0x7D1A0001u;
constexpr int LAYOUT_HDR = 8;
constexpr int MAX_L = 64;

enum RoadStatus : int {
  ROAD_OK = 0,
  ROAD_ERR_RANDINT = 1,   // ValueError at TDRoadGen.py:178 (empty pick range)
  ROAD_ERR_EMPTY = 2,     // IndexError at TDRoadGen.py:189 (branch road of length 0)
  ROAD_ERR_BOUND = 3,     // retry bound exceeded (the reference loops forever)
  ROAD_ERR_ARGS = 4,
  ROAD_PENDING = 5,       // resumable draw: budget exhausted, state kept (RoadGen::draw)
};

// State of a layout draw between RoadGen::draw calls (with the scratch arrays and
// the partial record).  16 words.
enum RoadPhase : uint32_t { RP_NEW = 0, RP_ROAD1 = 1, RP_ROAD2 = 2, RP_BRANCH = 3 };
struct RoadResume {
  uint32_t phase, att, nr, ri, n1, cr, cc, d0, nm, np, maxdist, endc;
  uint32_t start[3], pad;
};

TD_HD inline int layout_words(int L) { return LAYOUT_HDR + L * L; }

// Scratch for one road generation: 14 * L * L bytes.
struct RoadScratch {
  uint8_t* field;   // [NC]
  uint8_t* rot;     // [NC]
  uint16_t* r1;     // [NC] center -> end
  uint16_t* r2;     // [NC] center -> start
  uint16_t* rb;     // [NC] branch
  uint16_t* mainr;  // [NC]
  uint32_t* picks;  // [NC] (index << 16) | cell
};

TD_HD inline size_t road_scratch_bytes(int L) { return (size_t)L * L * 14 + 64; }

TD_HD inline RoadScratch road_scratch_carve(void* base, int L) {
  int nc = L * L;
  RoadScratch s;
  uint8_t* p = (uint8_t*)base;
  s.picks = (uint32_t*)p; p += 4 * nc;
  s.r1 = (uint16_t*)p; p += 2 * nc;
  s.r2 = (uint16_t*)p; p += 2 * nc;
  s.rb = (uint16_t*)p; p += 2 * nc;
  s.mainr = (uint16_t*)p; p += 2 * nc;
  s.field = p; p += nc;
  s.rot = p;
  return s;
}

template <class RNG>
struct RoadGen {
  RNG& rng;
  int L;
  RoadScratch s;
  int max_attempts;

  TD_HD bool inner(int r, int c) const { return r > 0 && r < L - 1 && c > 0 && c < L - 1; }

  // generate_road (TDRoadGen.py:31-119): walk from (r0,c0) in direction d.
  // Returns 1 on success, 0 on failure; *len = cells appended to out.
  TD_HD int walk(int r0, int c0, int d, uint16_t* out, int* len) {
    const int DR[4] = {1, 0, -1, 0}, DC[4] = {0, -1, 0, 1};  // :15 up,left,down,right
    int pr = r0, pc = c0, n = 0, pending = 0, loop = 0;  // pending: 0 = None, else +-1
    while (inner(pr, pc) && loop < 100) {
      ++loop;
      int shape = (int)rng.np_randint(0, 2);
      int seg = (int)rng.np_randint(L * 3 / 20, L / 4);
      bool cross = false;
      // one run of moves; reset_cross mirrors the `cross = False` at :98
      auto run = [&](int cnt, int dd, bool reset_cross) {
        for (int k = 0; k < cnt; ++k) {
          pr += DR[dd]; pc += DC[dd];
          if (s.field[pr * L + pc] != 0) { pr -= DR[dd]; pc -= DC[dd]; cross = true; return; }
          if (reset_cross) cross = false;
          out[n++] = (uint16_t)(pr * L + pc);
          s.field[pr * L + pc] = 1;
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
        else { rd = (int)rng.np_randint(0, 2) * 2 - 1; pending = -rd; }
        s.rot[pr * L + pc] = 1;
        d = (d + 4 + rd) % 4;
        run(seg, d, true);
      }
      if (cross) {
        int freed[4], nf = 0;
        for (int i = 0; i < 4; ++i)
          if (s.field[(pr + DR[i]) * L + pc + DC[i]] == 0) freed[nf++] = i;
        if (nf == 0) { *len = n; return 0; }
        d = freed[rng.np_randint(0, nf)];
        pending = 0;
        s.rot[pr * L + pc] = 1;
      }
    }
    *len = n;
    return loop >= 100 ? 0 : 1;
  }

  TD_HD void erase(const uint16_t* road, int n) {
    for (int i = 0; i < n; ++i) { s.field[road[i]] = 0; s.rot[road[i]] = 0; }
  }

  // The branch loop's first attempt (see the file comment): 1 when no candidate branch
  // point picks[klo, khi) can start a walk that ends on a border cell at Manhattan
  // distance >= 3L/4 from endc with fewer than 2L - (nm - index) cells.  BFS over the
  // free cells: s.r1 (free in the branch phase) is the queue, s.r2 the distances.
  TD_HD int branch_hopeless(int klo, int khi, int nm, int endc) {
    const int NC = L * L, dmin = L * 3 / 4;
    const int DR[4] = {1, 0, -1, 0}, DC[4] = {0, -1, 0, 1};
    for (int k = klo; k < khi; ++k) {
      const int bc = (int)(s.picks[k] & 0xffffu), lim = 2 * L - (nm - (int)(s.picks[k] >> 16));
      if (lim <= 0) continue;                              // every walk from here is too long
      if (!inner(bc / L, bc % L)) return 0;                // an empty branch: IndexError (:189), not a hang
      for (int i = 0; i < NC; ++i) s.r2[i] = 0xffffu;
      int qh = 0, qt = 0;
      s.r1[qt++] = (uint16_t)bc;
      s.r2[bc] = 0;
      while (qh < qt) {
        const int u = s.r1[qh++], du = s.r2[u];
        if (du + 1 >= lim) break;                          // BFS order: every later cell is as far
        for (int d = 0; d < 4; ++d) {
          const int r = u / L + DR[d], c = u % L + DC[d], v = r * L + c;
          if (s.field[v] || s.r2[v] != 0xffffu) continue;  // u is inner: v is on the board
          s.r2[v] = (uint16_t)(du + 1);
          if (inner(r, c)) s.r1[qt++] = (uint16_t)v;
          else if (iabs(r - endc / L) + iabs(c - endc % L) >= dmin) return 0;  // a walk could end here
        }
      }
    }
    return 1;
  }

  static TD_HD int iabs(int x) { return x < 0 ? -x : x; }

  // TDGymBasic.reset's draws (num_roads, :42) + create_road_v2 (TDRoadGen.py:4-199)
  // + the TDBoard map planes, as a resumable state machine: ``budget`` bounds the
  // walks (retry-loop attempts) run in this call.  Returns ROAD_OK (record complete),
  // a ROAD_ERR_* status (the reference raises, or the retry bound hit), or
  // ROAD_PENDING with the draw's state kept in ``st``, the scratch arrays and the
  // partial record -- a later call continues it draw for draw, so splitting a draw
  // over calls gives exactly the draws of one uninterrupted run.
  TD_HD int draw(RoadResume& st, int budget, uint32_t* rec) {
    const int NC = L * L;
    uint32_t* cw = rec + LAYOUT_HDR;
    if (st.phase == RP_NEW) {
      st.nr = (uint32_t)rng.np_randint(1, 4);  // TDGymBasic.reset :42
      const int nr = (int)st.nr;
      if (L < 4 || L > MAX_L || nr < 1 || nr > 3) return fail(st, ROAD_ERR_ARGS, rec);
      if (L / 4 <= L * 3 / 20) return fail(st, ROAD_ERR_RANDINT, rec);  // segment randint raises (:41)
      for (int i = 0; i < NC; ++i) { s.field[i] = 0; s.rot[i] = 0; }
      const int lo = L / 3, hi = (L * 2 + 2) / 3;
      st.cr = (uint32_t)rng.np_randint(lo, hi);
      st.cc = (uint32_t)rng.np_randint(lo, hi);
      s.field[st.cr * L + st.cc] = 1;
      st.d0 = (uint32_t)rng.np_randint(0, 4);
      st.phase = RP_ROAD1; st.att = 0;
    }
    const int cr = (int)st.cr, cc = (int)st.cc, d0 = (int)st.d0;
    while (st.phase == RP_ROAD1) {  // center -> end, :128-137
      if ((int)st.att >= max_attempts) return fail(st, ROAD_ERR_BOUND, rec);
      if (budget-- <= 0) return ROAD_PENDING;
      ++st.att;
      int n1 = 0;
      const int ok = walk(cr, cc, d0, s.r1, &n1);
      if (!ok || n1 >= L) { erase(s.r1, n1); continue; }
      st.n1 = (uint32_t)n1; st.phase = RP_ROAD2; st.att = 0;
    }
    while (st.phase == RP_ROAD2) {  // center -> start, :141-155
      if ((int)st.att >= max_attempts) return fail(st, ROAD_ERR_BOUND, rec);
      if (budget-- <= 0) return ROAD_PENDING;
      ++st.att;
      const int n1 = (int)st.n1;
      int n2 = 0;
      const int ok = walk(cr, cc, (d0 + 2) % 4, s.r2, &n2);
      if (!ok || n1 + n2 + 1 >= L * 2) { erase(s.r2, n2); continue; }
      const int e2 = s.r2[n2 - 1], e1 = s.r1[n1 - 1];
      if (iabs(e2 / L - e1 / L) + iabs(e2 % L - e1 % L) < L * 3 / 4) { erase(s.r2, n2); continue; }
      // main = reversed(road2) + [center] + road1 (:157-158), branch points (:162-170)
      int nm = 0;
      for (int i = n2 - 1; i >= 0; --i) s.mainr[nm++] = s.r2[i];
      s.mainr[nm++] = (uint16_t)(cr * L + cc);
      for (int i = 0; i < n1; ++i) s.mainr[nm++] = s.r1[i];
      int np = 0;
      for (int i = 0; i < nm;) {
        if (!s.rot[s.mainr[i]]) {
          if (i < nm - 1 && !s.rot[s.mainr[i + 1]]) s.picks[np++] = ((uint32_t)i << 16) | s.mainr[i];
          i += 1;
        } else {
          i += 2;
        }
      }
      // map planes from the main road first (roads[0])
      for (int i = 0; i < NC; ++i) cw[i] = 0;
      int maxdist = 0;
      stamp_road(cw, s.mainr, nm, 0, nullptr, 0, &maxdist);
      st.nm = (uint32_t)nm; st.np = (uint32_t)np; st.maxdist = (uint32_t)maxdist;
      st.start[0] = s.mainr[0]; st.start[1] = st.start[2] = 0;
      st.endc = s.mainr[nm - 1];
      st.phase = RP_BRANCH; st.ri = 1; st.att = 0;
    }
    while (st.phase == RP_BRANCH && (int)st.ri < (int)st.nr) {  // :174-197
      if ((int)st.att >= max_attempts) return fail(st, ROAD_ERR_BOUND, rec);
      if (budget-- <= 0) return ROAD_PENDING;
      ++st.att;
      const int np = (int)st.np, nm = (int)st.nm, endc = (int)st.endc;
      const int klo = np * 2 / 5, khi = np * 4 / 5;
      if (khi <= klo) return fail(st, ROAD_ERR_RANDINT, rec);
      if (st.att == 1 && branch_hopeless(klo, khi, nm, endc)) return fail(st, ROAD_ERR_BOUND, rec);
      int k = (int)rng.np_randint(klo, khi);
      const int nd = (int)rng.np_randint(0, 4);
      const int bcell = s.picks[k] & 0xffffu;
      k = (int)(s.picks[k] >> 16);
      int nb = 0;
      const int ok = walk(bcell / L, bcell % L, nd, s.rb, &nb);
      if (!ok) { erase(s.rb, nb); continue; }
      if (nb + nm - k >= L * 2) { erase(s.rb, nb); continue; }
      if (nb == 0) return fail(st, ROAD_ERR_EMPTY, rec);
      const int eb = s.rb[nb - 1];
      if (iabs(eb / L - endc / L) + iabs(eb % L - endc % L) < L * 3 / 4) { erase(s.rb, nb); continue; }
      // road = reversed(branch) + main[k:]
      for (int i = 0; i < nb / 2; ++i) { uint16_t t = s.rb[i]; s.rb[i] = s.rb[nb - 1 - i]; s.rb[nb - 1 - i] = t; }
      int maxdist = (int)st.maxdist;
      stamp_road(cw, s.rb, nb, (int)st.ri, s.mainr + k, nm - k, &maxdist);
      st.maxdist = (uint32_t)maxdist;
      st.start[st.ri] = (uint32_t)s.rb[0];
      ++st.ri; st.att = 0;
    }
    const int nr = (int)st.nr;
    for (int ri = 0; ri < nr; ++ri) cw[st.start[ri]] |= 1u << (5 + ri);
    cw[st.endc] |= 1u << 4;
    rec[0] = TD_LAYOUT_MAGIC;
    rec[1] = (uint32_t)nr;
    rec[2] = st.endc;
    rec[3] = st.maxdist;
    rec[4] = st.start[0];
    rec[5] = nr > 1 ? st.start[1] : 0u;
    rec[6] = nr > 2 ? st.start[2] : 0u;
    rec[7] = ROAD_OK;
    st.phase = RP_NEW;
    return ROAD_OK;
  }

  TD_HD static int fail(RoadResume& st, int status, uint32_t* rec) {
    rec[0] = 0; rec[1] = st.nr; rec[7] = (uint32_t)status;
    st.phase = RP_NEW;
    return status;
  }

  // One road's cells: rd[0..n) then tail[0..nt).  TDBoard.py:38-59.
  TD_HD void stamp_road(uint32_t* cw, const uint16_t* rd, int n, int ri, const uint16_t* tail, int nt, int* maxdist) {
    int tot = n + nt, prev = -1;
    for (int k = 0; k < tot; ++k) {
      int p = k < n ? rd[k] : tail[k - n];
      uint32_t w = cw[p] | 1u | (1u << (1 + ri));
      w = (w & 0x00ffffffu) | (1u << 24);
      int dist = tot - 1 - k;
      w = (w & ~(0xffu << 16)) | ((uint32_t)dist << 16);
      cw[p] = w;
      if (prev >= 0) {
        int dr = p / L - prev / L, dc = p % L - prev % L;
        uint32_t dir = dr == 0 ? (dc == 1 ? 0u : 1u) : (dr == 1 ? 2u : 3u);
        cw[prev] = (cw[prev] & ~(3u << 8)) | (dir << 8);
      }
      if (dist > *maxdist) *maxdist = dist;
      prev = p;
    }
  }
};

// Build a layout record from explicit road cell lists (road i = cells[off[i] .. off[i+1])),
// exactly as TDBoard.__init__ fills its map planes (TDBoard.py:31-59).
TD_HD inline int layout_from_roads(int L, int num_roads, const int32_t* cells, const int32_t* off, uint32_t* rec) {
  if (L < 2 || L > MAX_L || num_roads < 1 || num_roads > 3) return ROAD_ERR_ARGS;
  for (int i = 0; i < L * L; ++i) rec[LAYOUT_HDR + i] = 0;
  uint32_t* cw = rec + LAYOUT_HDR;
  int maxdist = 0;
  for (int ri = 0; ri < num_roads; ++ri) {
    int a = off[ri], b = off[ri + 1], prev = -1;
    if (b <= a) return ROAD_ERR_ARGS;
    for (int k = a; k < b; ++k) {
      int p = cells[k];
      if (p < 0 || p >= L * L) return ROAD_ERR_ARGS;
      uint32_t w = cw[p] | 1u | (1u << (1 + ri));
      w = (w & 0x00ffffffu) | (1u << 24);
      int dist = b - 1 - k;
      w = (w & ~(0xffu << 16)) | ((uint32_t)dist << 16);
      cw[p] = w;
      if (prev >= 0) {
        int dr = p / L - prev / L, dc = p % L - prev % L;
        uint32_t dir = dr == 0 ? (dc == 1 ? 0u : 1u) : (dr == 1 ? 2u : 3u);
        cw[prev] = (cw[prev] & ~(3u << 8)) | (dir << 8);
      }
      if (dist > maxdist) maxdist = dist;
      prev = p;
    }
  }
  for (int ri = 0; ri < num_roads; ++ri) cw[cells[off[ri]]] |= 1u << (5 + ri);
  int endc = cells[off[1] - 1];
  cw[endc] |= 1u << 4;
  rec[0] = TD_LAYOUT_MAGIC;
  rec[1] = (uint32_t)num_roads;
  rec[2] = (uint32_t)endc;
  rec[3] = (uint32_t)maxdist;
  for (int ri = 0; ri < 3; ++ri) rec[4 + ri] = ri < num_roads ? (uint32_t)cells[off[ri]] : 0u;
  rec[7] = ROAD_OK;
  return ROAD_OK;
}

// TDGymBasic.reset (:42-51): num_roads = randint(1, 4) then create_road_v2, on one
// stream, in one uninterrupted call.
template <class RNG>
TD_HD inline int episode_layout_rng(RNG& rng, int L, void* scratch, int max_attempts, uint32_t* rec) {
  RoadGen<RNG> g{rng, L, road_scratch_carve(scratch, L), max_attempts};
  RoadResume st{};
  return g.draw(st, 0x7fffffff, rec);
}

// Host form on a 625-word numpy state (RandomState.get_state() words + position).
TD_HD inline int episode_layout(uint32_t* np_state, int L, void* scratch, int max_attempts, uint32_t* rec) {
  MtRef rng{np_state};
  return episode_layout_rng(rng, L, scratch, max_attempts, rec);
}

}  // namespace td
