// Probe (host only): how many layout draws hit the retry bound (the reference never
// finishes them, TDRoadGen.py:129-189), how many walks they burn, and how many a static
// reachability proof (BFS over the free cells at the loop's entry) shows hopeless up
// front.  g++ -O2 -std=c++17 -I gym-td_amd/csrc scripts/roadgen_hopeless.cpp
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "td_layout.h"
using namespace td;

static int manh(int a, int b, int L) { return std::abs(a / L - b / L) + std::abs(a % L - b % L); }

// shortest number of appended cells from `from` to any border cell e with manh(e, far) >= dmin,
// moving through free inner cells (a walk stops at its first border cell); -1 if none
static int bfs(const uint8_t* field, int L, int from, int far, int dmin) {
  std::vector<int> dist(L * L, -1), q;
  dist[from] = 0; q.push_back(from);
  const int DR[4] = {1, 0, -1, 0}, DC[4] = {0, -1, 0, 1};
  int best = -1;
  for (size_t h = 0; h < q.size(); ++h) {
    int u = q[h], r = u / L, c = u % L;
    for (int d = 0; d < 4; ++d) {
      int rr = r + DR[d], cc = c + DC[d];
      if (rr < 0 || rr >= L || cc < 0 || cc >= L) continue;
      int v = rr * L + cc;
      if (field[v] || dist[v] >= 0) continue;
      dist[v] = dist[u] + 1;
      bool inner = rr > 0 && rr < L - 1 && cc > 0 && cc < L - 1;
      if (!inner) { if (manh(v, far, L) >= dmin && (best < 0 || dist[v] < best)) best = dist[v]; continue; }
      q.push_back(v);
    }
  }
  return best;
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 10;
  const int nseeds = argc > 2 ? atoi(argv[2]) : 2000;
  const int per = argc > 3 ? atoi(argv[3]) : 20;  // draws per seed (an auto-reset sequence)
  std::vector<uint8_t> scratch(road_scratch_bytes(L));
  std::vector<uint32_t> rec(layout_words(L));
  long draws = 0, ok = 0, bound = 0, other = 0, walks_all = 0, walks_bound = 0, proved = 0, proved_wrong = 0;
  long bound_phase[4] = {0, 0, 0, 0};
  for (int s = 0; s < nseeds; ++s) {
    uint32_t w[625];
    np_seed(w, (uint32_t)s);
    MtRef rng{w};
    for (int d = 0; d < per; ++d) {
      RoadGen<MtRef> g{rng, L, road_scratch_carve(scratch.data(), L), 1000};
      RoadResume st{};
      int walks = 0, status, last_phase = 0;
      bool hopeless = false;
      while (true) {
        status = g.draw(st, 1, rec.data());
        if (status != ROAD_PENDING) break;
        ++walks;
        last_phase = (int)st.phase;
        if (st.att == 0 && !hopeless) {  // a loop's entry: the field is the loop's static field
          if (st.phase == RP_ROAD2) {
            int lim = 2 * L - 1 - (int)st.n1;
            int e1 = g.s.r1[st.n1 - 1];
            int b = bfs(g.s.field, L, (int)(st.cr * L + st.cc), e1, L * 3 / 4);
            if (b < 0 || b >= lim) hopeless = true;
          } else if (st.phase == RP_BRANCH && st.ri < st.nr) {
            int np = (int)st.np, nm = (int)st.nm, klo = np * 2 / 5, khi = np * 4 / 5;
            if (khi > klo) {
              bool any = false;
              for (int k = klo; k < khi && !any; ++k) {
                int bc = (int)(g.s.picks[k] & 0xffffu), idx = (int)(g.s.picks[k] >> 16);
                int lim = 2 * L - (nm - idx);
                if (lim <= 0) continue;
                int r = bc / L, c = bc % L;
                if (!(r > 0 && r < L - 1 && c > 0 && c < L - 1)) { any = true; break; }
                int b = bfs(g.s.field, L, bc, (int)st.endc, L * 3 / 4);
                if (b >= 0 && b < lim) any = true;
              }
              if (!any) hopeless = true;
            }
          }
          if (hopeless) ++proved;
        }
      }
      ++walks;
      ++draws; walks_all += walks;
      if (status == ROAD_OK) ++ok;
      else if (status == ROAD_ERR_BOUND) { ++bound; walks_bound += walks; bound_phase[last_phase] += 1; }
      else ++other;
      if (hopeless && status != ROAD_ERR_BOUND) ++proved_wrong;
    }
  }
  printf("L=%d draws=%ld ok=%ld bound=%ld (road1 %ld road2 %ld branch %ld) other_err=%ld\n", L, draws, ok, bound,
         bound_phase[1], bound_phase[2], bound_phase[3], other);
  printf("walks: all=%ld in bound draws=%ld (%.1f%%), mean per ok draw=%.1f\n", walks_all, walks_bound,
         100.0 * walks_bound / walks_all, (double)(walks_all - walks_bound) / (draws - bound));
  printf("proved hopeless up front: %ld of %ld bound draws; proofs on draws that did not hit the bound: %ld\n", proved,
         bound, proved_wrong);
}
