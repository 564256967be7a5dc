/* td_cpu.c -- plain-C restatement of the gym-TD env step (CPU oracle / CPU baseline).
 *
 * TEST AND BENCH INFRASTRUCTURE ONLY (oracle/__init__.py): the native CPU path
 * that bench.py's cpu_baseline times (SURVEY.md 8(d) ii) and a second checker the
 * parity tests replay against the golden vectors.  The product never links it.
 * It restates the same reference code as oracle/td_oracle.py, written
 * independently of the HIP kernels (no shared source):
 *
 *   RNG      CPython random (Modules/_randommodule.c: init_by_array, getrandbits,
 *            _randbelow, random(), shuffle) and numpy's legacy RandomState
 *            (init_genrand, masked-rejection randint)            -- SURVEY 8(c)
 *   roads    create_road_v2                                      TDRoadGen.py:4-199
 *   board    TDBoard.__init__ / get_states / summon_cluster /
 *            tower_build / tower_lvup / tower_destruct / step / done
 *                                                                TDBoard.py:14-385
 *   elements Enemy.damage, Tower*.attack, create/upgrade_tower   TDElements.py:4-170
 *   envs     TDGymBasic.reset + built-in opponents               TDGymBasic.py:37-292
 *            TDDefense.step / TDAttack.step / TDMulti.step        TDDefense.py:34-87,
 *                                                                TDAttack.py:27-56, TDMulti.py:46-138
 *
 * Floating point: Python floats are IEEE binary64 and numpy-2 float32 rules apply
 * to the observation; build with -ffp-contract=off (no FMA), no -ffast-math.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MT_N 624
#define MT_M 397
#define ECAP 512
#define TCAP 128
#define NCH 45
#define MAXL 32

/* ------------------------------------------------------------------ MT19937 */
typedef struct { uint32_t mt[MT_N]; int pos; } Mt;

static void mt_init_genrand(Mt* m, uint32_t s) {
  m->mt[0] = s;
  for (int i = 1; i < MT_N; ++i) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
  m->pos = MT_N;
}

static void mt_init_by_array(Mt* m, const uint32_t* key, int klen) {  /* CPython random.seed(int) */
  mt_init_genrand(m, 19650218u);
  int i = 1, j = 0;
  for (int k = MT_N > klen ? MT_N : klen; k; --k) {
    m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= MT_N) { m->mt[0] = m->mt[MT_N - 1]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = MT_N - 1; k; --k) {
    m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= MT_N) { m->mt[0] = m->mt[MT_N - 1]; i = 1; }
  }
  m->mt[0] = 0x80000000u;
  m->pos = MT_N;
}

static uint32_t mt_next(Mt* m) {
  if (m->pos >= MT_N) {
    for (int k = 0; k < MT_N; ++k) {
      uint32_t y = (m->mt[k] & 0x80000000u) | (m->mt[(k + 1) % MT_N] & 0x7fffffffu);
      m->mt[k] = m->mt[(k + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->pos = 0;
  }
  uint32_t y = m->mt[m->pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* CPython random */
static int bit_length(uint64_t n) { int k = 0; while (n) { ++k; n >>= 1; } return k; }
static uint32_t py_randbelow(Mt* m, uint32_t n) {  /* n >= 1, n < 2^32 */
  const int k = bit_length(n);
  uint32_t r = mt_next(m) >> (32 - k);
  while (r >= n) r = mt_next(m) >> (32 - k);
  return r;
}
static int py_randint(Mt* m, int a, int b) { return a + (int)py_randbelow(m, (uint32_t)(b - a + 1)); }
static double py_random(Mt* m) {
  const uint32_t a = mt_next(m) >> 5, b = mt_next(m) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* numpy legacy RandomState.randint(lo, hi) (hi exclusive), masked rejection */
static int np_randint(Mt* m, int lo, int hi, int* err) {
  if (hi <= lo) { *err = 1; return lo; }  /* ValueError: high <= low */
  const uint32_t rng = (uint32_t)(hi - lo - 1);
  if (rng == 0) return lo;
  uint32_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next(m) & mask)) > rng) {}
  return lo + (int)v;
}

/* ------------------------------------------------------------------ config */
/* Value order of tdc_cfg_names() (oracle/td_cpu.py mirrors it). */
typedef struct {
  double enemy_LP[4][2], enemy_speed[4][2], enemy_defense[4][2], enemy_cost[4][2];
  double tower_attack[4][2], tower_range[4][2], tower_splash_range[4][2], tower_cost[4][2],
      tower_attack_interval[4][2];
  double tower_destruct_return, frozen_time, frozen_ratio, attacker_init_cost, defender_init_cost, base_LP,
      max_cost, reward_kill, penalty_leak, reward_time, attacker_cost_init_rate, attacker_cost_final_rate,
      defender_cost_rate, tower_distance, enemy_upgrade_at, attacker_action_interval, defender_action_interval,
      max_tower_lv;
} Cfg;
#define CFG_DOUBLES ((int)(sizeof(Cfg) / sizeof(double)))

static const int MAX_EPISODE_STEPS = 1200, MAX_CLUSTER = 8, MAX_ROADS = 3;  /* TDParam.py:107-111 */
enum { FC_OK = 0, FC_COST = 1, FC_POS = 2, FC_LVMAX = 3, FC_TARGET = 4 };     /* utils/fail_code.py */
enum { MODE_DEF = 0, MODE_ATK = 1, MODE_2P = 2 };

/* ------------------------------------------------------------------ board */
typedef struct { int type, lv, r, c, dist, slowdown; double LP, maxLP, speed, defense, cost, margin; } Enemy;
typedef struct { int type, lv, r, c; double atk, rge, dmgrge, intv, cost, cd; } Tower;

typedef struct {
  int L, mode, difficulty, multi, road_attempts;
  Cfg cfg;
  Mt np_rng, py_rng;
  /* TDBoard */
  int map[7][MAXL][MAXL];
  int num_roads, start[3][2], end[2];
  Enemy en[ECAP];
  int n_en;
  Tower tw[TCAP];
  int n_tw;
  double cost_def, cost_atk, progress;
  int base_LP, steps, fail_code;
  float elp[4 * 4 * MAXL * MAXL];  /* [4][4][L][L], dense at the board's L (ELP) */
  int attacker_cd, defender_cd;
  int overflow;
} Env;

/* ---- create_road_v2 (TDRoadGen.py:4-199) on the numpy stream ---- */
typedef struct { int n; int16_t p[MAXL * MAXL][2]; } Road;
typedef struct {
  Env* e;
  int L, err;
  uint8_t field[MAXL][MAXL], rot[MAXL][MAXL];
} Gen;

#define ELP(e, k, t, r, c) ((e)->elp[((((k) * 4 + (t)) * (e)->L + (r)) * (e)->L) + (c)])
#define ELP_BYTES(e) ((size_t)16 * (e)->L * (e)->L * sizeof(float))

static int g_inner(const Gen* g, int r, int c) { return r > 0 && r < g->L - 1 && c > 0 && c < g->L - 1; }
static const int STEP[4][2] = {{1, 0}, {0, -1}, {-1, 0}, {0, 1}};  /* :15 */

/* one run of moves of generate_road (:43-104); returns 1 when it stopped on a crossing */
static void g_run(Gen* g, Road* rd, int* pos, int n, int d, int reset_cross, int* cross) {
  for (int k = 0; k < n; ++k) {
    pos[0] += STEP[d][0]; pos[1] += STEP[d][1];
    if (g->field[pos[0]][pos[1]]) { pos[0] -= STEP[d][0]; pos[1] -= STEP[d][1]; *cross = 1; return; }
    if (reset_cross) *cross = 0;
    rd->p[rd->n][0] = (int16_t)pos[0]; rd->p[rd->n][1] = (int16_t)pos[1]; rd->n++;
    g->field[pos[0]][pos[1]] = 1;
    if (!g_inner(g, pos[0], pos[1])) return;
  }
}

/* generate_road (:31-119): 1 = success */
static int g_walk(Gen* g, int r0, int c0, int d, Road* rd) {
  Mt* m = &g->e->np_rng;
  const int L = g->L;
  int pos[2] = {r0, c0}, pending = 0, loop = 0;
  rd->n = 0;
  while (g_inner(g, pos[0], pos[1]) && loop < 100) {
    ++loop;
    const int shape = np_randint(m, 0, 2, &g->err);
    const int seg = np_randint(m, L * 3 / 20, L / 4, &g->err);
    int cross = 0;
    if (shape <= 0) {
      g_run(g, rd, pos, seg * 2, d, 0, &cross);
    } else {
      g_run(g, rd, pos, seg, d, 0, &cross);
      if (!g_inner(g, pos[0], pos[1])) break;
      int rdir;
      if (pending) { rdir = pending; pending = 0; }
      else { rdir = np_randint(m, 0, 2, &g->err) * 2 - 1; pending = -rdir; }
      g->rot[pos[0]][pos[1]] = 1;
      d = (d + 4 + rdir) % 4;
      g_run(g, rd, pos, seg, d, 1, &cross);
    }
    if (cross) {
      int fr[4], nf = 0;
      for (int i = 0; i < 4; ++i)
        if (!g->field[pos[0] + STEP[i][0]][pos[1] + STEP[i][1]]) fr[nf++] = i;
      if (!nf) return 0;
      d = fr[np_randint(m, 0, nf, &g->err)];
      pending = 0;
      g->rot[pos[0]][pos[1]] = 1;
    }
  }
  return loop >= 100 ? 0 : 1;
}

static void g_erase(Gen* g, const Road* rd) {
  for (int i = 0; i < rd->n; ++i) { g->field[rd->p[i][0]][rd->p[i][1]] = 0; g->rot[rd->p[i][0]][rd->p[i][1]] = 0; }
}

static int iabs(int x) { return x < 0 ? -x : x; }

/* The branch loop's first attempt: 1 when no candidate branch point main[pick_i[k]],
 * k in [klo, khi), can start a walk ending on a border cell at Manhattan distance
 * >= 3L/4 from the main road's end within the length bound -- the loop would never
 * finish (TDRoadGen.py:177; the rule of td_layout.h branch_hopeless, restated).  BFS
 * over the free cells; a walk stops on its first border cell. */
static int branch_hopeless(const Gen* g, const Road* mainr, const int* pick_i, int klo, int khi) {
  const int L = g->L, dmin = L * 3 / 4;
  const int er = mainr->p[mainr->n - 1][0], ec = mainr->p[mainr->n - 1][1];
  static __thread int16_t dist[MAXL][MAXL];
  static __thread int16_t q[MAXL * MAXL][2];
  for (int k = klo; k < khi; ++k) {
    const int idx = pick_i[k], lim = 2 * L - (mainr->n - idx);
    const int br = mainr->p[idx][0], bcc = mainr->p[idx][1];
    if (lim <= 0) continue;
    if (!g_inner(g, br, bcc)) return 0;  /* an empty branch raises IndexError (:189) */
    for (int r = 0; r < L; ++r)
      for (int c = 0; c < L; ++c) dist[r][c] = -1;
    int qh = 0, qt = 0;
    q[qt][0] = (int16_t)br; q[qt][1] = (int16_t)bcc; ++qt;
    dist[br][bcc] = 0;
    while (qh < qt) {
      const int ur = q[qh][0], uc = q[qh][1];
      ++qh;
      const int du = dist[ur][uc];
      if (du + 1 >= lim) break;
      for (int d = 0; d < 4; ++d) {
        const int r = ur + STEP[d][0], c = uc + STEP[d][1];
        if (g->field[r][c] || dist[r][c] >= 0) continue;
        dist[r][c] = (int16_t)(du + 1);
        if (g_inner(g, r, c)) { q[qt][0] = (int16_t)r; q[qt][1] = (int16_t)c; ++qt; }
        else if (iabs(r - er) + iabs(c - ec) >= dmin) return 0;
      }
    }
  }
  return 1;
}

/* roads[i] as cell lists; returns 0 or an error (1 randint ValueError, 2 IndexError, 3 bound) */
static int create_road(Env* e, int num_roads, Road* roads) {
  Gen g;
  memset(&g, 0, sizeof g);
  g.e = e; g.L = e->L;
  const int L = e->L, lo = L / 3, hi = (L * 2 + 2) / 3;
  Mt* m = &e->np_rng;
  const int cr = np_randint(m, lo, hi, &g.err), cc = np_randint(m, lo, hi, &g.err);
  g.field[cr][cc] = 1;
  const int d0 = np_randint(m, 0, 4, &g.err);
  static __thread Road r1, r2, rb;
  int att;
  for (att = 0;; ++att) {  /* :128-137 */
    if (att >= e->road_attempts) return 3;
    const int ok = g_walk(&g, cr, cc, d0, &r1);
    if (g.err) return 1;
    if (!ok || r1.n >= L) { g_erase(&g, &r1); continue; }
    break;
  }
  for (att = 0;; ++att) {  /* :141-155 */
    if (att >= e->road_attempts) return 3;
    const int ok = g_walk(&g, cr, cc, (d0 + 2) % 4, &r2);
    if (g.err) return 1;
    if (!ok || r1.n + r2.n + 1 >= L * 2) { g_erase(&g, &r2); continue; }
    if (iabs(r2.p[r2.n - 1][0] - r1.p[r1.n - 1][0]) + iabs(r2.p[r2.n - 1][1] - r1.p[r1.n - 1][1]) < L * 3 / 4) {
      g_erase(&g, &r2);
      continue;
    }
    break;
  }
  Road* mainr = &roads[0];  /* reversed(road2) + [center] + road1, :157-158 */
  mainr->n = 0;
  for (int i = r2.n - 1; i >= 0; --i) { mainr->p[mainr->n][0] = r2.p[i][0]; mainr->p[mainr->n][1] = r2.p[i][1]; mainr->n++; }
  mainr->p[mainr->n][0] = (int16_t)cr; mainr->p[mainr->n][1] = (int16_t)cc; mainr->n++;
  for (int i = 0; i < r1.n; ++i) { mainr->p[mainr->n][0] = r1.p[i][0]; mainr->p[mainr->n][1] = r1.p[i][1]; mainr->n++; }
  static __thread int pick_i[MAXL * MAXL];
  int np = 0;  /* selectable branch points, :162-170 */
  for (int i = 0; i < mainr->n;) {
    if (!g.rot[mainr->p[i][0]][mainr->p[i][1]]) {
      if (i < mainr->n - 1 && !g.rot[mainr->p[i + 1][0]][mainr->p[i + 1][1]]) pick_i[np++] = i;
      i += 1;
    } else {
      i += 2;
    }
  }
  for (int ri = 1; ri < num_roads; ++ri) {  /* :174-197 */
    int k = 0;
    for (att = 0;; ++att) {
      if (att >= e->road_attempts) return 3;
      if (np * 4 / 5 <= np * 2 / 5) return 1;  /* randint's ValueError (:178) */
      if (att == 0 && branch_hopeless(&g, mainr, pick_i, np * 2 / 5, np * 4 / 5)) return 3;
      k = np_randint(m, np * 2 / 5, np * 4 / 5, &g.err);
      if (g.err) return 1;
      const int nd = np_randint(m, 0, 4, &g.err);
      k = pick_i[k];
      const int ok = g_walk(&g, mainr->p[k][0], mainr->p[k][1], nd, &rb);
      if (g.err) return 1;
      if (!ok) { g_erase(&g, &rb); continue; }
      if (rb.n + mainr->n - k >= L * 2) { g_erase(&g, &rb); continue; }
      if (rb.n == 0) return 2;
      if (iabs(rb.p[rb.n - 1][0] - mainr->p[mainr->n - 1][0]) + iabs(rb.p[rb.n - 1][1] - mainr->p[mainr->n - 1][1]) <
          L * 3 / 4) {
        g_erase(&g, &rb);
        continue;
      }
      break;
    }
    Road* out = &roads[ri];  /* reversed(branch) + main[k:] */
    out->n = 0;
    for (int i = rb.n - 1; i >= 0; --i) { out->p[out->n][0] = rb.p[i][0]; out->p[out->n][1] = rb.p[i][1]; out->n++; }
    for (int i = k; i < mainr->n; ++i) { out->p[out->n][0] = mainr->p[i][0]; out->p[out->n][1] = mainr->p[i][1]; out->n++; }
  }
  return 0;
}

/* TDBoard.__init__ map planes (TDBoard.py:31-59) */
static void board_init(Env* e, const Road* roads, int nr) {
  const Cfg* c = &e->cfg;
  memset(e->map, 0, sizeof e->map);
  for (int i = 0; i < nr; ++i) {
    const Road* rd = &roads[i];
    for (int k = 0; k < rd->n; ++k) {
      const int r = rd->p[k][0], cc = rd->p[k][1];
      e->map[0][r][cc] = 1; e->map[i + 1][r][cc] = 1; e->map[6][r][cc] = 1;
      if (k > 0) {
        const int pr = rd->p[k - 1][0], pc = rd->p[k - 1][1], dr = r - pr, dc = cc - pc;
        e->map[5][pr][pc] = dr == 0 ? (dc == 1 ? 0 : 1) : (dr == 1 ? 2 : 3);
      }
    }
    for (int k = 0; k < rd->n; ++k) e->map[4][rd->p[rd->n - 1 - k][0]][rd->p[rd->n - 1 - k][1]] = k;
    e->start[i][0] = rd->p[0][0]; e->start[i][1] = rd->p[0][1];
  }
  e->end[0] = roads[0].p[roads[0].n - 1][0]; e->end[1] = roads[0].p[roads[0].n - 1][1];
  e->num_roads = nr;
  e->n_en = e->n_tw = 0;
  e->cost_def = c->defender_init_cost;
  e->cost_atk = c->attacker_init_cost;
  e->base_LP = (int)c->base_LP;
  e->steps = 0;
  e->progress = 0.0;
  e->fail_code = FC_OK;
  memset(e->elp, 0, ELP_BYTES(e));
}

/* TDGymBasic.reset (:37-55): 0 or the road error (the board is left unchanged) */
static int env_reset(Env* e) {
  int err = 0;
  const int nr = np_randint(&e->np_rng, 1, MAX_ROADS + 1, &err);
  static __thread Road roads[3];
  const int st = create_road(e, nr, roads);
  if (st) return st;
  board_init(e, roads, nr);
  e->attacker_cd = e->defender_cd = 0;
  return 0;
}

/* ---- TDBoard.get_states (TDBoard.py:85-144), numpy-2 float32 ---- */
static void get_states(const Env* e, float* s) {
  const Cfg* c = &e->cfg;
  const int L = e->L, P = L * L;
  memset(s, 0, sizeof(float) * NCH * P);
#define S(ch, r, cc) s[(ch) * P + (r) * L + (cc)]
  int maxd = 0;
  for (int r = 0; r < L; ++r)
    for (int cc = 0; cc < L; ++cc) if (e->map[4][r][cc] > maxd) maxd = e->map[4][r][cc];
  const float v5 = (float)((double)e->base_LP / c->base_LP), v11 = (float)(e->cost_def / c->max_cost),
              v12 = (float)(e->cost_atk / c->max_cost), v13 = (float)e->progress;
  float v21[4], v41[4];
  for (int t = 0; t < 4; ++t) {
    v21[t] = e->cost_def >= c->tower_cost[t][0] ? 1.0f : 0.0f;
    v41[t] = (float)(e->cost_def / c->enemy_cost[t][0] / MAX_CLUSTER);
  }
  for (int r = 0; r < L; ++r)
    for (int cc = 0; cc < L; ++cc) {
      for (int k = 0; k < 4; ++k) S(k, r, cc) = (float)e->map[k][r][cc];
      S(5, r, cc) = v5;
      S(9, r, cc) = (float)((double)e->map[4][r][cc] / (double)(maxd + 1));
      S(11, r, cc) = v11; S(12, r, cc) = v12; S(13, r, cc) = v13;
      S(14, r, cc) = e->map[6][r][cc] == 0 ? 1.0f : 0.0f;
      for (int t = 0; t < 4; ++t) {
        S(21 + t, r, cc) = v21[t];
        for (int k = 0; k < 4; ++k) S(25 + 4 * k + t, r, cc) = ELP(e, k, t, r, cc);
        S(41 + t, r, cc) = v41[t];
      }
    }
  S(4, e->end[0], e->end[1]) = 1.0f;
  for (int i = 0; i < e->num_roads; ++i) S(6 + i, e->start[i][0], e->start[i][1]) = 1.0f;
  const int lv0 = 15, ty0 = lv0 + (int)c->max_tower_lv + 1;
  for (int i = 0; i < e->n_tw; ++i) {
    const Tower* w = &e->tw[i];
    S(lv0 + w->lv, w->r, w->c) = 1.0f;
    S(ty0 + w->type, w->r, w->c) = 1.0f;
  }
#undef S
}

/* ---- summon_cluster (TDBoard.py:199-224): returns ok (the tuple is truthy to callers) ---- */
static int summon_cluster(Env* e, const int* types, int road, int* real) {
  const Cfg* c = &e->cfg;
  const int lv = e->progress >= c->enemy_upgrade_at ? 1 : 0;
  int tried = 0, summoned = 0;
  for (int k = 0; k < MAX_CLUSTER; ++k) {
    const int t = types[k];
    if (real) real[k] = t;
    if (t == 4) continue;
    tried = 1;
    if (e->cost_atk < c->enemy_cost[t][lv]) { if (real) real[k] = 4; continue; }
    if (e->n_en >= ECAP) { e->overflow = 1; if (real) real[k] = 4; continue; }
    e->cost_atk -= c->enemy_cost[t][lv];
    Enemy* en = &e->en[e->n_en++];
    en->type = t; en->lv = lv; en->r = e->start[road][0]; en->c = e->start[road][1];
    en->dist = e->map[4][en->r][en->c];
    en->LP = en->maxLP = c->enemy_LP[t][lv];
    en->speed = c->enemy_speed[t][lv]; en->defense = c->enemy_defense[t][lv]; en->cost = c->enemy_cost[t][lv];
    en->margin = 0.0; en->slowdown = 0;
    summoned = 1;
  }
  if (tried && !summoned) { e->fail_code = FC_COST; return 0; }
  e->fail_code = FC_OK;
  return 1;
}

/* ---- defender operations (TDBoard.py:226-293) ---- */
static void diamond(Env* e, int r0, int c0, int delta) {
  const int k = (int)e->cfg.tower_distance;
  for (int i = -k; i <= k; ++i)
    for (int j = -k; j <= k; ++j)
      if (iabs(i) + iabs(j) <= k) {
        const int r = r0 + i, c = c0 + j;
        if (r >= 0 && r < e->L && c >= 0 && c < e->L) e->map[6][r][c] += delta;
      }
}

static int tower_build(Env* e, int t, int r, int c) {
  const Cfg* cf = &e->cfg;
  if (e->cost_def < cf->tower_cost[t][0]) { e->fail_code = FC_COST; return 0; }
  if (e->map[6][r][c] > 0) { e->fail_code = FC_POS; return 0; }
  if (e->n_tw >= TCAP) { e->overflow = 1; e->fail_code = FC_POS; return 0; }
  Tower* w = &e->tw[e->n_tw++];
  w->type = t; w->lv = 0; w->r = r; w->c = c;
  w->atk = cf->tower_attack[t][0]; w->rge = cf->tower_range[t][0]; w->dmgrge = cf->tower_splash_range[t][0];
  w->intv = cf->tower_attack_interval[t][0]; w->cost = cf->tower_cost[t][0]; w->cd = 0.0;
  e->cost_def -= w->cost;
  diamond(e, r, c, 1);
  e->fail_code = FC_OK;
  return 1;
}

static int tower_at(const Env* e, int r, int c) {
  for (int i = 0; i < e->n_tw; ++i) if (e->tw[i].r == r && e->tw[i].c == c) return i;
  return -1;
}

static int tower_lvup(Env* e, int r, int c) {
  const Cfg* cf = &e->cfg;
  const int i = tower_at(e, r, c);
  if (i < 0) { e->fail_code = FC_TARGET; return 0; }
  Tower* w = &e->tw[i];
  if (w->lv >= (int)cf->max_tower_lv) { e->fail_code = FC_LVMAX; return 0; }
  const double cost = cf->tower_cost[w->type][w->lv + 1];
  if (e->cost_def < cost) { e->fail_code = FC_COST; return 0; }
  /* upgrade_tower -> lvup with interval and cost swapped (TDElements.py:152-170) */
  const int t = w->type, l = w->lv + 1;
  w->lv = l;
  w->atk = cf->tower_attack[t][l]; w->rge = cf->tower_range[t][l]; w->dmgrge = cf->tower_splash_range[t][l];
  w->intv = cf->tower_cost[t][l];
  w->cost += cf->tower_attack_interval[t][l];
  e->cost_def -= cost;
  e->fail_code = FC_OK;
  return 1;
}

static int tower_destruct(Env* e, int r, int c) {
  const int i = tower_at(e, r, c);
  if (i < 0) { e->fail_code = FC_TARGET; return 0; }
  e->cost_def += e->tw[i].cost * e->cfg.tower_destruct_return;
  e->cost_def = e->cfg.max_cost < e->cost_def ? e->cfg.max_cost : e->cost_def;  /* min(cost, max_cost) */
  memmove(&e->tw[i], &e->tw[i + 1], sizeof(Tower) * (size_t)(e->n_tw - i - 1));
  e->n_tw--;
  diamond(e, r, c, -1);
  e->fail_code = FC_OK;
  return 1;
}

/* ---- Enemy.damage / Tower*.attack (TDElements.py:19-28, 71-132) ---- */
static void hit(Enemy* en, double atk, int magic) {
  double dmg = magic ? atk : (atk - en->defense > 0 ? atk - en->defense : 0);
  if (dmg < atk * .05) dmg = atk * .05;
  en->LP -= dmg;
  if (en->LP <= 0) en->LP = 0;
}
static int cheb(int r0, int c0, int r1, int c1) {
  const int a = iabs(r0 - r1), b = iabs(c0 - c1);
  return a > b ? a : b;
}

/* appends newly killed enemy indices to dead[] (unique) */
static void fire(Env* e, Tower* w, int* dead, int* nd) {
  int tg = -1;
  for (int i = 0; i < e->n_en; ++i)
    if (cheb(e->en[i].r, e->en[i].c, w->r, w->c) <= w->rge) { tg = i; break; }
  if (tg < 0) return;
  w->cd += w->intv;
#define KILLED(i) do { if (!(e->en[i].LP > 0)) { int seen = 0; for (int q = 0; q < *nd; ++q) if (dead[q] == (i)) seen = 1; if (!seen) dead[(*nd)++] = (i); } } while (0)
  if (w->type == 0 || w->type == 1) {
    hit(&e->en[tg], w->atk, w->type == 1);
    KILLED(tg);
  } else if (w->type == 2) {
    const int tr = e->en[tg].r, tc = e->en[tg].c;
    for (int i = 0; i < e->n_en; ++i)
      if (cheb(tr, tc, e->en[i].r, e->en[i].c) <= w->dmgrge) { hit(&e->en[i], w->atk, 0); KILLED(i); }
  } else {
    const int tr = e->en[tg].r, tc = e->en[tg].c;
    for (int i = 0; i < e->n_en; ++i)
      if (cheb(tr, tc, e->en[i].r, e->en[i].c) <= w->dmgrge) {
        hit(&e->en[i], w->atk, 1);
        e->en[i].slowdown = (int)e->cfg.frozen_time;
        KILLED(i);
        break;
      }
  }
#undef KILLED
}

/* ---- TDBoard.step (TDBoard.py:295-368) ---- */
static double board_step(Env* e) {
  const Cfg* c = &e->cfg;
  double reward = 0.0;
  reward += c->reward_time;
  e->steps += 1;
  e->progress = (double)e->steps / MAX_EPISODE_STEPS;
  /* stable sort by dist - margin (f64 key): insertion sort */
  for (int i = 1; i < e->n_en; ++i) {
    Enemy t = e->en[i];
    const double k = (double)t.dist - t.margin;
    int j = i - 1;
    while (j >= 0 && (double)e->en[j].dist - e->en[j].margin > k) { e->en[j + 1] = e->en[j]; --j; }
    e->en[j + 1] = t;
  }
  static __thread int dead[ECAP];
  int nd = 0;
  for (int i = 0; i < e->n_tw; ++i) {
    Tower* w = &e->tw[i];
    w->cd -= 1;
    if (w->cd > 0) continue;
    fire(e, w, dead, &nd);
    if (w->cd < 0) w->cd = 0;
  }
  reward += c->reward_kill * nd;
  if (nd) {
    static __thread uint8_t gone[ECAP];
    memset(gone, 0, (size_t)e->n_en);
    for (int q = 0; q < nd; ++q) gone[dead[q]] = 1;
    int k = 0;
    for (int i = 0; i < e->n_en; ++i) if (!gone[i]) e->en[k++] = e->en[i];
    e->n_en = k;
  }
  static const int MOVE[4][2] = {{0, 1}, {0, -1}, {1, 0}, {-1, 0}};  /* :319 */
  int k = 0;
  for (int i = 0; i < e->n_en; ++i) {
    Enemy* en = &e->en[i];
    if (en->slowdown > 0) { en->margin += en->speed * c->frozen_ratio; en->slowdown -= 1; }
    else en->margin += en->speed;
    int leaked = 0;
    while (en->margin >= 1.0) {
      en->margin -= 1.0;
      const int d = e->map[5][en->r][en->c];
      en->r += MOVE[d][0]; en->c += MOVE[d][1];
      en->dist = e->map[4][en->r][en->c];
      if (en->r == e->end[0] && en->c == e->end[1]) {
        if (e->base_LP > 0) reward -= c->penalty_leak;
        e->base_LP = e->base_LP - 1 > 0 ? e->base_LP - 1 : 0;
        leaked = 1;
        break;
      }
    }
    if (!leaked) e->en[k++] = *en;
  }
  e->n_en = k;
  const double rate = e->progress >= 0.5 ? c->attacker_cost_final_rate
      : c->attacker_cost_init_rate * (1. - e->progress) + c->attacker_cost_final_rate * e->progress;
  e->cost_atk = e->cost_atk + rate < c->max_cost ? e->cost_atk + rate : c->max_cost;
  e->cost_def = e->cost_def + c->defender_cost_rate < c->max_cost ? e->cost_def + c->defender_cost_rate : c->max_cost;
  /* enemy_LP planes (:355-365), numpy-2 float32: min / max / sequential sum / count */
  memset(e->elp, 0, ELP_BYTES(e));
  const int L = e->L;
  for (int t = 0; t < 4; ++t)
    for (int r = 0; r < L; ++r)
      for (int cc = 0; cc < L; ++cc) ELP(e, 0, t, r, cc) = 1.0f;
  for (int i = 0; i < e->n_en; ++i) {
    const Enemy* en = &e->en[i];
    const float r = (float)(en->LP / en->maxLP);
    float* mn = &ELP(e, 0, en->type, en->r, en->c);
    float* mx = &ELP(e, 1, en->type, en->r, en->c);
    if (r < *mn) *mn = r;
    if (r > *mx) *mx = r;
    ELP(e, 2, en->type, en->r, en->c) += r;
    ELP(e, 3, en->type, en->r, en->c) += 1.0f;
  }
  for (int t = 0; t < 4; ++t)
    for (int r = 0; r < L; ++r)
      for (int cc = 0; cc < L; ++cc) {
        const float n = ELP(e, 3, t, r, cc);
        if (!(n > 0)) { ELP(e, 0, t, r, cc) = 0.0f; ELP(e, 2, t, r, cc) = 0.0f; }
        else ELP(e, 2, t, r, cc) = ELP(e, 2, t, r, cc) / n;
        ELP(e, 3, t, r, cc) = n / (float)MAX_CLUSTER;
      }
  return reward;
}

static int board_done(const Env* e) { return e->base_LP <= 0 || e->steps >= MAX_EPISODE_STEPS; }

/* ---- built-in opponents (TDGymBasic.py:81-292), random_agent=True ---- */
static void random_enemy(Env* e) {
  if (e->attacker_cd != 0) return;
  int types[MAX_CLUSTER], road;
  if (e->difficulty == 0) {
    for (int k = 0; k < MAX_CLUSTER; ++k) types[k] = py_randint(&e->py_rng, 0, 4);
    road = py_randint(&e->py_rng, 0, e->num_roads - 1);
  } else {
    const int t = py_randint(&e->py_rng, 0, 3);
    road = py_randint(&e->py_rng, 0, e->num_roads - 1);
    for (int k = 0; k < MAX_CLUSTER; ++k) types[k] = t;
  }
  summon_cluster(e, types, road, NULL);
  e->attacker_cd = (int)e->cfg.attacker_action_interval;
}

static void build_near_road(Env* e, int t, int draw_type) {
  static __thread int cells[MAXL * MAXL][2];
  int n = 0;
  for (int r = 0; r < e->L; ++r)
    for (int c = 0; c < e->L; ++c)
      if (e->map[0][r][c] == 1) { cells[n][0] = r; cells[n][1] = c; ++n; }
  for (int i = n - 1; i >= 1; --i) {  /* random.shuffle */
    const int j = (int)py_randbelow(&e->py_rng, (uint32_t)(i + 1));
    int a0 = cells[i][0], a1 = cells[i][1];
    cells[i][0] = cells[j][0]; cells[i][1] = cells[j][1]; cells[j][0] = a0; cells[j][1] = a1;
  }
  if (draw_type) t = py_randint(&e->py_rng, 0, 3);
  for (int i = 0; i < n; ++i) {
    const int k = py_randint(&e->py_rng, 0, 24);
    const int r = cells[i][0] + k / 5 - 2, c = cells[i][1] + k % 5 - 2;
    if (r < 0 || r >= e->L || c < 0 || c >= e->L) continue;
    if (tower_build(e, t, r, c)) { e->defender_cd = (int)e->cfg.defender_action_interval; return; }
    if (e->fail_code == FC_COST) return;
  }
}

static void upgrade_or_destruct(Env* e, int act) {
  if (!e->n_tw) return;
  if (act == 1) {
    const int i = py_randint(&e->py_rng, 0, e->n_tw - 1);
    if (tower_lvup(e, e->tw[i].r, e->tw[i].c)) e->defender_cd = (int)e->cfg.defender_action_interval;
  } else {
    if (py_random(&e->py_rng) > .01) return;
    const int i = py_randint(&e->py_rng, 0, e->n_tw - 1);
    if (tower_destruct(e, e->tw[i].r, e->tw[i].c)) e->defender_cd = (int)e->cfg.defender_action_interval;
  }
}

static void random_tower(Env* e) {
  if (e->defender_cd != 0) return;
  if (e->difficulty == 0) {
    const int r = py_randint(&e->py_rng, 0, e->L - 1), c = py_randint(&e->py_rng, 0, e->L - 1);
    const int t = py_randint(&e->py_rng, 0, 3);
    if (tower_build(e, t, r, c)) e->defender_cd = (int)e->cfg.defender_action_interval;
    return;
  }
  const int act = py_randint(&e->py_rng, 0, 2);
  if (act != 0) { upgrade_or_destruct(e, act); return; }
  if (e->difficulty == 1) { build_near_road(e, 0, 1); return; }
  /* lv2: tower type against the enemy mix (np.unique counts, f64 ratios) */
  if (!e->n_en) return;
  int cnt[4] = {0, 0, 0, 0};
  for (int i = 0; i < e->n_en; ++i) cnt[e->en[i].type]++;
  double p = py_random(&e->py_rng);
  int chosen = -1;
  for (int t = 0, i = 0; t < 4; ++t) {
    if (!cnt[t]) continue;
    const double ratio = (double)cnt[t] / (double)e->n_en;
    if (p < ratio) { chosen = t; break; }
    p -= ratio;
    ++i;
  }
  if (chosen < 0) return;  /* the reference would raise IndexError here (rounding) */
  static const int REMAP[4] = {2, 0, 1, 0};
  int t = REMAP[chosen];
  if (py_random(&e->py_rng) < 0.2) t = 3;
  build_near_road(e, t, 0);
}

/* ---- env steps ---- */
static int def_discrete(Env* e, int64_t a) {  /* TDDefense.py:62-77 / TDMulti.py:243-258: fail code or -1 (acted) */
  const int L = e->L;
  if (e->defender_cd == 0 && a != (int64_t)L * L * 6) {
    const int op = (int)(a / (L * L)), r = (int)((a / L) % L), c = (int)(a % L);
    int res;
    if (op < 4) res = tower_build(e, op, r, c);
    else if (op == 4) res = tower_lvup(e, r, c);
    else res = tower_destruct(e, r, c);
    if (res) { e->defender_cd = (int)e->cfg.defender_action_interval; return -1; }
    return e->fail_code;
  }
  return 0;
}

static void def_scan(Env* e, const int64_t* a) {  /* TDDefense.py:41-60 / TDMulti.py:208-227 */
  const int L = e->L, P = L * L;
  if (e->defender_cd != 0) return;
  for (int r = 0; r < L; ++r)
    for (int c = 0; c < L; ++c) {
      for (int t = 0; t < 4; ++t)
        if (a[t * P + r * L + c] == 1 && tower_build(e, t, r, c)) e->defender_cd = (int)e->cfg.defender_action_interval;
      if (a[4 * P + r * L + c] == 1 && tower_lvup(e, r, c)) e->defender_cd = (int)e->cfg.defender_action_interval;
      if (a[5 * P + r * L + c] == 1 && tower_destruct(e, r, c)) e->defender_cd = (int)e->cfg.defender_action_interval;
    }
}

static void atk_clusters(Env* e, const int64_t* a) {
  if (e->attacker_cd != 0) return;
  for (int i = 0; i < e->num_roads; ++i) {
    int cl[MAX_CLUSTER], all4 = 1;
    for (int k = 0; k < MAX_CLUSTER; ++k) { cl[k] = (int)a[i * MAX_CLUSTER + k]; all4 &= cl[k] == 4; }
    if (e->mode == MODE_2P && e->multi) {  /* TDMulti.py:199-206: every road, truthy */
      summon_cluster(e, cl, i, NULL);
      e->attacker_cd = (int)e->cfg.attacker_action_interval;
      continue;
    }
    if (all4) continue;
    const int ok = summon_cluster(e, cl, i, NULL);
    if (e->mode == MODE_ATK) { if (ok) e->attacker_cd = (int)e->cfg.attacker_action_interval; }  /* TDAttack.py:43-44 */
    else e->attacker_cd = (int)e->cfg.attacker_action_interval;                                  /* TDMulti.py:237-238 */
  }
}

static double env_step(Env* e, const int64_t* da, const int64_t* aa, int* done) {
  e->attacker_cd = e->attacker_cd - 1 > 0 ? e->attacker_cd - 1 : 0;
  e->defender_cd = e->defender_cd - 1 > 0 ? e->defender_cd - 1 : 0;
  if (e->mode == MODE_DEF) {
    if (e->multi) def_scan(e, da); else def_discrete(e, da[0]);
    random_enemy(e);
  } else if (e->mode == MODE_ATK) {
    atk_clusters(e, aa);
    random_tower(e);
  } else {
    atk_clusters(e, aa);
    if (e->multi) def_scan(e, da); else def_discrete(e, da[0]);
  }
  double reward = board_step(e);
  if (e->mode == MODE_ATK) reward = -reward;
  *done = board_done(e);
  return reward;
}

/* ------------------------------------------------------------------ C API (ctypes, oracle/td_cpu.py) */
int tdc_cfg_doubles(void) { return CFG_DOUBLES; }

void* tdc_new(int L, int mode, int difficulty, int multi, uint32_t np_seed, uint32_t py_seed, const double* cfg,
              int road_attempts, int* status) {
  Env* e = (Env*)calloc(1, sizeof(Env));
  if (!e || L < 4 || L > MAXL) { free(e); if (status) *status = 4; return NULL; }
  e->L = L; e->mode = mode; e->difficulty = difficulty; e->multi = multi;
  e->road_attempts = road_attempts > 0 ? road_attempts : 1000;
  memcpy(&e->cfg, cfg, sizeof(Cfg));
  mt_init_genrand(&e->np_rng, np_seed);
  mt_init_by_array(&e->py_rng, &py_seed, 1);
  const int st = env_reset(e);
  if (status) *status = st;
  return e;
}

void tdc_free(void* p) { free(p); }
int tdc_reset(void* p) { return env_reset((Env*)p); }

double tdc_step(void* p, const int64_t* def_act, const int64_t* atk_act, float* obs, int* done) {
  Env* e = (Env*)p;
  const double r = env_step(e, def_act, atk_act, done);
  if (obs) get_states(e, obs);
  return r;
}

void tdc_obs(void* p, float* obs) { get_states((Env*)p, obs); }

/* canon.state_bytes layout (oracle/canon.py): returns the byte count */
int tdc_state_bytes(void* p, uint8_t* out, int cap) {
  const Env* e = (const Env*)p;
  const int need = 64 + e->n_en * 56 + e->n_tw * 40 + e->L * e->L * 8;
  if (!out || cap < need) return need;
  uint8_t* q = out;
#define PUT_I(v) do { int64_t t_ = (int64_t)(v); memcpy(q, &t_, 8); q += 8; } while (0)
#define PUT_D(v) do { double t_ = (double)(v); memcpy(q, &t_, 8); q += 8; } while (0)
  PUT_I(e->steps); PUT_I(e->base_LP); PUT_D(e->cost_def); PUT_D(e->cost_atk);
  PUT_I(e->attacker_cd); PUT_I(e->defender_cd); PUT_I(e->n_en); PUT_I(e->n_tw);
  for (int i = 0; i < e->n_en; ++i) {
    const Enemy* en = &e->en[i];
    PUT_I(en->type); PUT_I(en->lv); PUT_I(en->r); PUT_I(en->c); PUT_I(en->slowdown); PUT_D(en->LP); PUT_D(en->margin);
  }
  for (int i = 0; i < e->n_tw; ++i) {
    const Tower* w = &e->tw[i];
    PUT_I(w->type); PUT_I(w->lv); PUT_I(w->r); PUT_I(w->c); PUT_D(w->cd);
  }
  for (int r = 0; r < e->L; ++r)
    for (int c = 0; c < e->L; ++c) PUT_I(e->map[6][r][c]);
#undef PUT_I
#undef PUT_D
  return need;
}

/* map planes 0-6 (int64 [7][L][L]), start cells [3][2], end [2]; returns num_roads */
int tdc_layout(void* p, int64_t* map7, int64_t* start, int64_t* end) {
  const Env* e = (const Env*)p;
  const int L = e->L;
  for (int k = 0; k < 7; ++k)
    for (int r = 0; r < L; ++r)
      for (int c = 0; c < L; ++c) map7[(k * L + r) * L + c] = e->map[k][r][c];
  for (int i = 0; i < e->num_roads; ++i) { start[2 * i] = e->start[i][0]; start[2 * i + 1] = e->start[i][1]; }
  end[0] = e->end[0]; end[1] = e->end[1];
  return e->num_roads;
}

int tdc_overflow(void* p) { return ((Env*)p)->overflow; }

/* CPU baseline: n_envs independent TD-def envs (discrete defender actions uniform
 * over [0, 6 L^2], built-in opponent lv `difficulty`, auto-reset skipping failing
 * layout draws), stepped for `seconds` on `threads` OpenMP threads, each env's
 * observation written every step.  Returns env-steps; *wall = seconds taken. */
long long tdc_bench(int L, int mode, int multi, int n_envs, double seconds, int threads, uint32_t seed,
                    const double* cfg, double* wall) {
  long long total = 0;
  double t_max = 0.0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(+ : total) reduction(max : t_max)
#endif
  {
#ifdef _OPENMP
    const int tid = omp_get_thread_num(), nth = omp_get_num_threads();
#else
    const int tid = 0, nth = 1;
#endif
    const int lo = (int)((long long)n_envs * tid / nth), hi = (int)((long long)n_envs * (tid + 1) / nth);
    const int n = hi - lo;
    Env** envs = (Env**)calloc((size_t)(n > 0 ? n : 1), sizeof(Env*));
    float* obs = (float*)malloc(sizeof(float) * NCH * L * L);
    int64_t* da = (int64_t*)calloc((size_t)6 * L * L, sizeof(int64_t));
    int64_t aa[24];
    Mt act;
    mt_init_genrand(&act, seed + 7919u * (uint32_t)tid);
    for (int i = 0; i < n; ++i) {
      int st = 1;
      uint32_t s = seed + (uint32_t)(lo + i);
      while (st) {  /* the reference raises for a few L=10 draws: take the next seed */
        free(envs[i]);
        envs[i] = (Env*)tdc_new(L, mode, 1, multi, s, s, cfg, 1000, &st);
        s += 1000003u;
      }
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    double el = 0.0;
    long long steps = 0;
    while (el < seconds && n > 0) {
      for (int i = 0; i < n; ++i) {
        Env* e = envs[i];
        if (mode != MODE_ATK) {
          if (multi) for (int k = 0; k < 6 * L * L; ++k) da[k] = (int64_t)(mt_next(&act) % 3u);
          else da[0] = (int64_t)(mt_next(&act) % (uint32_t)(6 * L * L + 1));
        }
        if (mode != MODE_DEF) for (int k = 0; k < 24; ++k) aa[k] = (int64_t)(mt_next(&act) % 5u);
        int done = 0;
        tdc_step(e, da, aa, obs, &done);
        ++steps;
        if (done) while (env_reset(e)) {}
      }
      clock_gettime(CLOCK_MONOTONIC, &t1);
      el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    }
    for (int i = 0; i < n; ++i) free(envs[i]);
    free(envs); free(obs); free(da);
    total += steps;
    t_max = el;
  }
  if (wall) *wall = t_max;
  return total;
}

/* ------------------------------------------------------------------ batched checker
 * n independent envs stepped together on OpenMP threads, as the device steps a batch: the
 * every-board steady-state parity test (tests/test_gpu_steady.py) runs bench.py's burn-in
 * recipe on the device and here side by side.  Resets follow the device's auto-reset
 * semantics: the next layout draw that succeeds (TDGymBasic.reset, TDGymBasic.py:37-55;
 * failing draws -- where the reference raises, TDRoadGen.py:177-189 -- skipped, at most
 * LAYOUT_RETRIES + 1 draws; a board with none keeps its state and is flagged). */
#define LAYOUT_RETRIES 64
typedef struct {
  int n, L, mode, multi, threads;
  Env** envs;
  int* no_layout;
} Batch;

static int reset_skipping(Env* e) {
  for (int k = 0; k <= LAYOUT_RETRIES; ++k)
    if (env_reset(e) == 0) return 0;
  return 1;
}

static void set_threads(int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
}

/* status[b]: 0, or 1 when no initial draw of board b succeeded.  Returns NULL on a bad
 * argument or an allocation failure. */
void* tdc_batch_new(int n, int L, int mode, int difficulty, int multi, const uint32_t* np_seeds,
                    const uint32_t* py_seeds, const double* cfg, int road_attempts, int threads, int* status) {
  if (n < 1 || L < 4 || L > MAXL) return NULL;
  Batch* bt = (Batch*)calloc(1, sizeof(Batch));
  if (!bt) return NULL;
  bt->n = n; bt->L = L; bt->mode = mode; bt->multi = multi; bt->threads = threads;
  bt->envs = (Env**)calloc((size_t)n, sizeof(Env*));
  bt->no_layout = (int*)calloc((size_t)n, sizeof(int));
  if (!bt->envs || !bt->no_layout) { free(bt->envs); free(bt->no_layout); free(bt); return NULL; }
  int oom = 0;
  set_threads(threads);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) reduction(| : oom)
#endif
  for (int b = 0; b < n; ++b) {
    int st = 0;
    Env* e = (Env*)tdc_new(L, mode, difficulty, multi, np_seeds[b], py_seeds[b], cfg, road_attempts, &st);
    if (!e) { oom = 1; continue; }
    if (st) st = reset_skipping(e);  /* the first draw failed: the next ones from the same stream */
    bt->envs[b] = e;
    bt->no_layout[b] = st != 0;
    if (status) status[b] = st != 0;
  }
  if (oom) {
    for (int b = 0; b < n; ++b) free(bt->envs[b]);
    free(bt->envs); free(bt->no_layout); free(bt);
    return NULL;
  }
  return bt;
}

void tdc_batch_free(void* p) {
  Batch* bt = (Batch*)p;
  if (!bt) return;
  for (int b = 0; b < bt->n; ++b) free(bt->envs[b]);
  free(bt->envs); free(bt->no_layout); free(bt);
}

/* Explicit reset of the boards with mask[b] != 0 (next succeeding draw).  Returns the
 * number of masked boards that found no layout (they keep their state). */
int tdc_batch_reset(void* p, const uint8_t* mask) {
  Batch* bt = (Batch*)p;
  int missed = 0;
  set_threads(bt->threads);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : missed)
#endif
  for (int b = 0; b < bt->n; ++b) {
    if (mask && !mask[b]) continue;
    if (reset_skipping(bt->envs[b])) { bt->no_layout[b] = 1; ++missed; }
  }
  return missed;
}

/* One step of every board that has a layout.  def_act int64 [n] (discrete) or [n][6][L][L]
 * (multi-action), atk_act int64 [n][3][8] (NULL in TD-def), reward f64 [n], done u8 [n],
 * obs f32 [n][45][L][L] or NULL (not built: faster burn-in).  autoreset != 0: a board that
 * finishes starts its next episode and obs holds that episode's first observation.
 * Boards without a layout are not stepped (reward 0, done 0, obs zeros).  Returns the
 * number of boards that finished. */
int tdc_batch_step(void* p, const int64_t* def_act, const int64_t* atk_act, double* reward, uint8_t* done,
                   float* obs, int autoreset) {
  Batch* bt = (Batch*)p;
  const int L = bt->L;
  const size_t nd = bt->multi ? (size_t)6 * L * L : 1, no = (size_t)NCH * L * L;
  int finished = 0;
  set_threads(bt->threads);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : finished)
#endif
  for (int b = 0; b < bt->n; ++b) {
    Env* e = bt->envs[b];
    float* ob = obs ? obs + no * (size_t)b : NULL;
    if (bt->no_layout[b]) {
      reward[b] = 0.0;
      done[b] = 0;
      if (ob) memset(ob, 0, no * sizeof(float));
      continue;
    }
    static const int64_t empty_atk[24] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4};
    const int64_t* da = def_act ? def_act + nd * (size_t)b : NULL;
    const int64_t* aa = atk_act ? atk_act + (size_t)24 * b : empty_atk;
    int64_t idle = 6 * L * L;
    int d = 0;
    reward[b] = env_step(e, da ? da : &idle, aa, &d);
    done[b] = (uint8_t)d;
    if (d) {
      ++finished;
      if (autoreset && reset_skipping(e)) bt->no_layout[b] = 1;
    }
    if (ob) get_states(e, ob);
  }
  return finished;
}

/* Every board's observation (f32 [n][45][L][L]). */
void tdc_batch_obs(void* p, float* obs) {
  Batch* bt = (Batch*)p;
  const size_t no = (size_t)NCH * bt->L * bt->L;
  set_threads(bt->threads);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int b = 0; b < bt->n; ++b) get_states(bt->envs[b], obs + no * (size_t)b);
}

/* no_layout flags (int32 [n]): 1 where a reset found no layout. */
void tdc_batch_flags(void* p, int32_t* out) {
  Batch* bt = (Batch*)p;
  for (int b = 0; b < bt->n; ++b) out[b] = bt->no_layout[b];
}

/* canon.state_bytes of board b (tdc_state_bytes). */
int tdc_batch_state_bytes(void* p, int b, uint8_t* out, int cap) {
  Batch* bt = (Batch*)p;
  return tdc_state_bytes(bt->envs[b], out, cap);
}
