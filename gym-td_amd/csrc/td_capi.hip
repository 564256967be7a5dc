// td_capi.hip -- the C-ABI (include/tdstep.h): handle, HBM buffers, launches.
//
// Everything per board lives on the device: board records, both RNG streams
// (layouts: numpy-legacy MT19937; built-in opponent: CPython MT19937) and the
// staged next-episode layout.  Layouts are generated on the device
// (td_refill_kernel / td_reset_kernel), so the step loop has no host work.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/tdstep.h"
#include "../../include/td_diag.h"
#include "td_kernels.h"
#include "td_layout.h"
#include "td_rng.h"

using namespace td;

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}

#define HIP_OK(expr)                                                                                         \
  do {                                                                                                       \
    hipError_t e_ = (expr);                                                                                  \
    if (e_ != hipSuccess) return fail("%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

// Steps between refill launches (td_set_refill_interval).  Every 16th step instead of
// every 4th: 23.7 / 36.3 / 208.3 vs 24.9 / 37.1 / 209.2 us per step at 4,096 / 8,192 /
// 65,536 boards, no ring dry over 5,000 steps, the GPU suite green (profiles/r02/s44).
// Every launch is ordered behind the step stream (start_refill):
// refills left unordered between steps ran 4-8 % faster at 4,096 / 8,192 boards, but a
// step that finds a ring empty then has no refill beside it to wait for: under load a
// board missed its layout (test_autoreset_under_load, profiles/r02/s43_unordered).
// With rings of 16 and the ring guard, every 64th step: 34.3 / 21.5 us per step at
// 8,192 / 4,096 boards vs 34.8 / 22.2-22.75 at every 16th, +-0 at 65,536; no refill and
// no guard at all (rings draining, not a product setting): 33.1-33.8 / 20.0
// (profiles/r03/s23).
constexpr int kRefillEvery = 64;
constexpr int kRefillWaves = 1024;
// A pending draw advances 3 walks per step of refill interval (48 per launch at 16): the
// fewer walks a refill wave runs per launch, the less it holds a wave slot the next
// step's waves need (8,192 boards, a refill every 4th step: 37.9 us per step at 48 walks, 36.5 at 12, 36.6 at 4,
// 36.9 at 1; 34.3 without refills, profiles/r02/s21_session.log).
constexpr int kWalksPerStep = 3;
// The ring guard (td_step.hip td_refill_kernel, guard = G) runs on the step stream before
// every G-th step and fills every ring below G layouts to G: a board consumes at most one
// layout per step, so none of the next G steps finds a ring empty, whatever the refill
// cadence.  G = NSLOT - 1: a ring the side refills keep full only falls below it when a
// board finishes two episodes between two refills, so the guard rarely draws (G = NSLOT
// made it draw for every board that finished one: 8,192 boards 78 vs 35 us per step,
// profiles/r03/s12); a launch is then a scan of the rings, paid every G steps.
constexpr int kGuardEvery = NSLOT - 1;
constexpr int kSideStreams = 2;  // refill streams: one stuck on a long draw does not stall the next (the HIP
                                 // runtime has 4 hardware queues per process; the step stream needs one)

}  // namespace

struct td_handle {
  int L = 0, NC = 0, B = 0, mode = 0, multi = 0, difficulty = 1, device = 0, autoreset = 1;
  int opp_np = 0;  // random_agent=False
  int small = 0, obs_wt = 0;  // the step kernel (0 large, 1 small, 2 small2), write-through observation stores
  int small_auto = 0;         // td_create's choice (TD_KERNEL_AUTO)
  std::string kernel_name;    // td_step_kernel_name
  int lw = 0;  // layout record words
  size_t scratch_stride = 0;
  TdDevCfg dcfg;
  TdDevCfg* d_cfg = nullptr;  // [NCFG]: one constant block per paramConfig epoch
  int epoch = 0;              // the current block
  int cfg_fresh = 1;          // blocks [cfg_fresh, NCFG) never used yet
  TdHdr* d_hdr = nullptr;
  double *d_en_lp = nullptr, *d_en_mg = nullptr, *d_tw_cd = nullptr;
  uint32_t *d_en_inf = nullptr, *d_tw_inf = nullptr, *d_cells = nullptr, *d_opp = nullptr, *d_np = nullptr;
  uint32_t* d_hot = nullptr;  // opponent hot record [B][HOT_WORDS]
  uint32_t *d_nxt = nullptr, *d_stage = nullptr;  // staged-layout rings [B][NSLOT][slot_words]; caller records
  uint32_t *d_lay_head = nullptr, *d_lay_tail = nullptr, *d_lay_claim = nullptr;  // rings (td_kernels.h)
  int32_t* d_ovr_idx = nullptr;                           // td_reset_layouts: [B] index into d_stage or -1
  uint8_t *d_scratch = nullptr, *d_mask = nullptr, *d_fail = nullptr;
  int stage_cap = 0;
  double* d_epstats = nullptr;   // [2] finished episodes, sum of their returns
  td_episode_record* d_lastep = nullptr;  // [B] each board's last finished episode
  // Layout refills run on kSideStreams side streams in turn; the step stream never
  // waits for them (the rings give every board NSLOT episodes of slack, and
  // per-board claims keep concurrent refills apart).
  hipStream_t side[kSideStreams] = {};
  hipEvent_t ev_main = nullptr;  // orders a refill after a reset kernel (system-scope fence)
  hipEvent_t ev_step = nullptr;  // orders a refill after the previous step (no system-scope fence)
  int next_side = 0;
  int refill_every = kRefillEvery;  // 0: no refill launches (td_set_refill_interval)
  int refill_waves = kRefillWaves;  // waves per refill launch
  int guard_every = kGuardEvery;  // ring guard cadence
  int since_guard = kGuardEvery;  // steps launched since the last ring guard (>= guard_every: guard first)
  // td_kernel_timing: event pairs bound to the next `tev_cap` step-kernel dispatches
  std::vector<hipEvent_t> tev;
  int tev_cap = 0, tev_n = 0, tev_every = 1;
  long long tev_from = 0;  // h->steps when td_kernel_timing was called
  long long steps = 0;
  std::vector<int32_t> last_reset_failed;
  uint32_t* d_guard_to = nullptr;  // [1] ring-guard claim waits that gave up (td_guard_timeouts)
  int xcd_map = 1;  // XCD-contiguous board map (td_kernels.h xcd_board; td_set_store_policy)
  int edge_wt = 2;  // observation lines shared with a neighbour: plain write-back stores, merged in the XCD's L2
                    // (1.088x vs 1.093x the algorithmic bytes at 65,536 boards, step time +-0, profiles/r04/s20);
                    // 1: write-through (sc1), the reference form of tests/test_gpu_store_policy.py
};

namespace {

void build_dev_cfg(const td_config& c, TdDevCfg& d) {
  std::memset(&d, 0, sizeof d);
  for (int t = 0; t < 4; ++t)
    for (int l = 0; l < 2; ++l) {
      d.e_lp[t][l] = c.enemy_LP[t][l];
      d.e_speed[t][l] = c.enemy_speed[t][l];
      d.e_def[t][l] = c.enemy_defense[t][l];
      d.e_cost[t][l] = c.enemy_cost[t][l];
      d.t_atk[t][l] = c.tower_attack[t][l];
      d.t_rge[t][l] = c.tower_range[t][l];
      d.t_dmg[t][l] = c.tower_splash_range[t][l];
      d.t_price[t][l] = c.tower_cost[t][l];
    }
  // Tower attributes after create_tower / upgrade_tower (TDElements.py:134-170):
  // lvup(atk, rge, dmgrge, intv=tower_cost[t][l], cost += tower_attack_interval[t][l]).
  for (int t = 0; t < 4; ++t) {
    d.t_intv[t][0] = c.tower_attack_interval[t][0];
    d.t_intv[t][1] = c.tower_cost[t][1];
    d.t_addcost[t][0] = 0.0;
    d.t_addcost[t][1] = c.tower_attack_interval[t][1];
  }
  d.destruct_return = c.tower_destruct_return;
  d.frozen_ratio = c.frozen_ratio;
  d.max_cost = c.max_cost;
  d.reward_kill = c.reward_kill;
  d.penalty_leak = c.penalty_leak;
  d.reward_time = c.reward_time;
  d.atk_init_rate = c.attacker_cost_init_rate;
  d.atk_final_rate = c.attacker_cost_final_rate;
  d.def_rate = c.defender_cost_rate;
  d.enemy_upgrade_at = c.enemy_upgrade_at;
  d.def_init_cost = c.defender_init_cost;
  d.atk_init_cost = c.attacker_init_cost;
  d.frozen_time = (int32_t)c.frozen_time;
  d.base_LP = (int32_t)c.base_LP;
  d.tower_distance = (int32_t)c.tower_distance;
  d.atk_interval = (int32_t)c.attacker_action_interval;
  d.def_interval = (int32_t)c.defender_action_interval;
  d.max_episode_steps = c.max_episode_steps;
  d.max_cluster_length = c.max_cluster_length;
  d.max_tower_lv = c.max_tower_lv;
}

int check_cfg(const td_config& c) {
  if (c.enemy_types != 4 || c.tower_types != 4) return fail("enemy_types / tower_types must be 4 (obs has 45 channels)");
  if (c.max_enemy_lv != 1 || c.max_tower_lv < 0 || c.max_tower_lv > 1) return fail("max_enemy_lv must be 1, max_tower_lv 0 or 1");
  if (c.max_cluster_length != 8 || c.max_num_of_roads != 3) return fail("max_cluster_length must be 8, max_num_of_roads 3");
  if (c.max_episode_steps <= 0) return fail("max_episode_steps must be > 0");
  if (c.tower_distance < 0 || c.tower_distance > 15) return fail("tower_distance out of range");
  if (c.frozen_time < 0 || c.frozen_time > 255) return fail("frozen_time must be in [0, 255] (8-bit slowdown)");
  if (c.base_LP < 1) return fail("base_LP must be a positive int (None is not supported)");
  for (int t = 0; t < 4; ++t)
    for (int l = 0; l < 2; ++l)
      if (c.enemy_LP[t][l] <= 0) return fail("enemy_LP must be > 0");
  return 0;
}

// Device allocations.  The library's own arrays are plain hipMalloc: every state array
// physically contiguous as well measured slower at most sizes (8,192 boards 35.1 vs 32.5
// us, 65,536 215.0 vs 210.4, profiles/r04/s25).  Callers' output buffers: td_alloc_device.
// *granted: whether the block is physically contiguous (a refused request falls back).
static hipError_t dev_malloc(void** p, size_t bytes, bool contiguous, bool* granted) {
  *granted = false;
  if (contiguous && hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) {
    *granted = true;
    return hipSuccess;
  }
  (void)hipGetLastError();  // (a refused contiguous request is not the caller's error)
  return hipMalloc(p, bytes);
}

// Live td_alloc_device blocks and how each was placed (td_alloc_is_contiguous).
std::mutex g_blocks_mu;
std::unordered_map<const void*, bool> g_blocks;

template <class T>
int dalloc(T** p, size_t n) {
  HIP_OK(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
  HIP_OK(hipMemset(*p, 0, std::max<size_t>(n, 1) * sizeof(T)));
  return 0;
}

StepArgs base_args(td_handle* h) {
  StepArgs a;
  std::memset(&a, 0, sizeof a);
  a.B = h->B; a.L = h->L; a.mode = h->mode; a.multi = h->multi; a.difficulty = h->difficulty;
  a.autoreset = h->autoreset;
  a.xcd_map = h->xcd_map;
  a.edge_wt = h->edge_wt;
  a.opp_np = h->opp_np;
  a.small = h->small;
  a.obs_wt = h->obs_wt;
  a.hdr = h->d_hdr; a.en_lp = h->d_en_lp; a.en_mg = h->d_en_mg; a.en_inf = h->d_en_inf;
  a.tw_cd = h->d_tw_cd; a.tw_inf = h->d_tw_inf; a.cells = h->d_cells; a.opp_mt = h->d_opp; a.opp_hot = h->d_hot;
  a.np_mt = h->d_np; a.nxt = h->d_nxt; a.scratch = h->d_scratch; a.scratch_stride = h->scratch_stride;
  a.lay_head = h->d_lay_head; a.lay_tail = h->d_lay_tail; a.lay_claim = h->d_lay_claim;
  a.slot_words = slot_words(h->L);
  a.refill_grp = refill_group(h->B, h->refill_waves);
  a.refill_waves = h->refill_waves;
  a.refill_walks = kWalksPerStep * (h->refill_every > 0 ? h->refill_every : kRefillEvery);
  a.guard_to = h->d_guard_to;
  a.reset_fail = h->d_fail; a.cfg = h->d_cfg + h->epoch; a.cfgs = h->d_cfg; a.epoch = h->epoch;
  return a;
}

// fn(i) for i in [0, n) on a few host threads (seeding only).
template <class F>
void parallel_for(int n, F fn) {
  unsigned hw = std::thread::hardware_concurrency();
  int nt = std::max(1, std::min<int>((int)std::min(8u, hw ? hw : 1u), (n + 1023) / 1024));
  std::vector<std::thread> pool;
  for (int w = 0; w < nt; ++w)
    pool.emplace_back([&, w]() {
      for (int i = w; i < n; i += nt) fn(i);
    });
  for (auto& t : pool) t.join();
}

// The step kernel (td_set_step_kernel): small = 0 large, 1 small, 2 small2.  Write-through
// observation stores go with the small kernels where the batch's observation fits the
// 256-MiB Infinity Cache (scripts/storepol.hip: 21.8 vs 30.0 us at 8,192 boards).
int apply_kernel(td_handle* h, int small) {
  h->small = small;
  const double obs_bytes = (double)h->B * NCH * h->NC * 4.0;
  // (Write-through beyond the Infinity Cache -- any kernel, TD_OBS_WT=1 -- measured 1.5-1.7x
  // slower steps at 16,384-65,536 boards, profiles/r03/s21.)
  h->obs_wt = h->small && obs_bytes <= 192.0 * 1024 * 1024 ? 1 : 0;
  const bool has_small = h->L == 10 || h->L == 20 || h->L == 30;
  const char* k = !has_small || small == 0 ? "td_step_kernel" : small == 1 ? "td_step_kernel_small" : "td_step_kernel_small2";
  char buf[96];
  std::snprintf(buf, sizeof buf, "%s<%d, %d, %s>", k, has_small ? h->L : 0, h->mode, h->multi ? "true" : "false");
  h->kernel_name = buf;
  return 0;
}

// Drop staged layouts: they were drawn from a stream that has been replaced.
int drop_staged(td_handle* h, int b) {
  HIP_OK(hipDeviceSynchronize());
  h->since_guard = kGuardEvery;
  const size_t ring = (size_t)NSLOT * slot_words(h->L);
  HIP_OK(hipMemset(h->d_nxt + (size_t)b * ring, 0, ring * 4));
  HIP_OK(hipMemset(h->d_lay_head + b, 0, 4));
  HIP_OK(hipMemset(h->d_lay_tail + b, 0, 4));
  HIP_OK(hipMemset(h->d_lay_claim + b, 0, 4));
  HIP_OK(hipMemset(h->d_scratch + (size_t)b * h->scratch_stride, 0, sizeof(RoadResume)));  // no pending draw
  return 0;
}

int drop_all_staged(td_handle* h) {
  HIP_OK(hipDeviceSynchronize());
  h->since_guard = kGuardEvery;
  HIP_OK(hipMemset(h->d_nxt, 0, (size_t)h->B * NSLOT * slot_words(h->L) * 4));
  HIP_OK(hipMemset(h->d_lay_head, 0, (size_t)h->B * 4));
  HIP_OK(hipMemset(h->d_lay_tail, 0, (size_t)h->B * 4));
  HIP_OK(hipMemset(h->d_lay_claim, 0, (size_t)h->B * 4));
  HIP_OK(hipMemset(h->d_scratch, 0, (size_t)h->B * h->scratch_stride));  // no pending draws
  return 0;
}

// Launch a ring refill behind the work queued on `s` so far, on the side streams in
// turn.  Refills are anchored to the step stream (each waits for the step before it,
// then runs beside the next one), never to host time: the host may run thousands of
// steps ahead of the GPU, and a refill launched "when a stream looks free" from there
// would leave the GPU without refills for as long.  A refill stuck on a draw the
// reference never finishes (milliseconds) delays only its own stream's queue.
// The refill is ordered after the work on s so far: after a reset kernel, whose
// draws-now use the boards' numpy streams and ring slots without a claim, and after the
// previous step (see kRefillEvery).
int start_refill(td_handle* h, hipStream_t s, bool after_step = false) {
  const int q = h->next_side;
  StepArgs a = base_args(h);
  hipEvent_t ev = after_step ? h->ev_step : h->ev_main;
  HIP_OK(hipEventRecord(ev, s));
  HIP_OK(hipStreamWaitEvent(h->side[q], ev, 0));
  HIP_OK(launch_refill(a, h->side[q]));
  h->next_side = (q + 1) % kSideStreams;
  return 0;
}

int run_reset(td_handle* h, const std::vector<uint8_t>& mask, float* obs, hipStream_t s) {
  HIP_OK(hipMemcpy(h->d_mask, mask.data(), (size_t)h->B, hipMemcpyHostToDevice));
  HIP_OK(hipMemset(h->d_fail, 0, (size_t)h->B));
  StepArgs a = base_args(h);
  a.obs = obs;
  a.reset_mask = h->d_mask;
  HIP_OK(launch_step(a, s, true));
  h->since_guard = kGuardEvery;  // a reset consumed layouts: guard before the next step
  if (h->autoreset && !h->opp_np && start_refill(h, s)) return -1;
  HIP_OK(hipDeviceSynchronize());
  return 0;
}

}  // namespace

extern "C" {

int td_abi_version(void) { return TD_ABI_VERSION; }

int td_step_io_size(void) { return (int)sizeof(td_step_io); }

int td_alloc_device(size_t bytes, int device, int contiguous, void** out) {
  if (!out || bytes == 0) return fail("td_alloc_device: bad arguments");
  *out = nullptr;
  int prev = 0;
  HIP_OK(hipGetDevice(&prev));
  HIP_OK(hipSetDevice(device));
  bool granted = false;
  hipError_t e = dev_malloc(out, bytes, contiguous != 0, &granted);
  if (e == hipSuccess) e = hipMemset(*out, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();  // zeroed before any stream uses it
  (void)hipSetDevice(prev);  // (the caller's current device is left as it was)
  if (e != hipSuccess) {
    if (*out) (void)hipFree(*out);
    *out = nullptr;
    return fail("td_alloc_device: %s", hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> g(g_blocks_mu);
  g_blocks[*out] = granted;
  return 0;
}

int td_free_device(void* p) {
  if (!p) return 0;
  {
    std::lock_guard<std::mutex> g(g_blocks_mu);
    g_blocks.erase(p);
  }
  HIP_OK(hipFree(p));
  return 0;
}

int td_alloc_is_contiguous(const void* p) {
  std::lock_guard<std::mutex> g(g_blocks_mu);
  auto it = g_blocks.find(p);
  return it == g_blocks.end() ? -1 : it->second ? 1 : 0;
}

void td_step_io_init(td_step_io* io) {
  if (!io) return;
  std::memset(io, 0, sizeof *io);
  io->size = (uint32_t)sizeof(td_step_io);
  io->abi = TD_ABI_VERSION;
}

const char* td_last_error(void) { return g_err.c_str(); }

void td_config_default(td_config* c) {
  // gym_TD/envs/TDParam.py:2-64, :105-111
  std::memset(c, 0, sizeof *c);
  const double lp[4][2] = {{820, 1700}, {2050, 3000}, {6000, 8000}, {8000, 12000}};
  const double sp[4][2] = {{.25, .25}, {.13, .13}, {.1, .1}, {.1, .1}};
  const double df[4][2] = {{0, 0}, {200, 250}, {600, 800}, {80, 100}};
  const double ec[4][2] = {{8, 8}, {15, 15}, {40, 40}, {30, 30}};
  const double ta[4][2] = {{454, 540}, {651, 771}, {566, 691}, {358, 424}};
  const double tr[4][2] = {{3, 3}, {2, 2}, {4, 4}, {3, 3}};
  const double ts[4][2] = {{0, 0}, {0, 0}, {1, 1}, {0, 0}};
  const double tc[4][2] = {{10, 10}, {17, 17}, {23, 23}, {12, 12}};
  const double ti[4][2] = {{2, 2}, {4, 4}, {7, 7}, {4.75, 4.75}};
  std::memcpy(c->enemy_LP, lp, sizeof lp);
  std::memcpy(c->enemy_speed, sp, sizeof sp);
  std::memcpy(c->enemy_defense, df, sizeof df);
  std::memcpy(c->enemy_cost, ec, sizeof ec);
  std::memcpy(c->tower_attack, ta, sizeof ta);
  std::memcpy(c->tower_range, tr, sizeof tr);
  std::memcpy(c->tower_splash_range, ts, sizeof ts);
  std::memcpy(c->tower_cost, tc, sizeof tc);
  std::memcpy(c->tower_attack_interval, ti, sizeof ti);
  c->tower_destruct_return = .5;
  c->frozen_time = 2;
  c->frozen_ratio = .2;
  c->attacker_init_cost = 0;
  c->defender_init_cost = 10;
  c->base_LP = 5;
  c->max_cost = 100;
  c->reward_kill = 0.1;
  c->penalty_leak = 10.;
  c->reward_time = 0.001;
  c->attacker_cost_init_rate = .5;
  c->attacker_cost_final_rate = 1;
  c->defender_cost_rate = .2;
  c->tower_distance = 2;
  c->enemy_upgrade_at = 0.75;
  c->attacker_action_interval = 1;
  c->defender_action_interval = 1;
  c->max_enemy_lv = 1;
  c->max_tower_lv = 1;
  c->enemy_types = 4;
  c->tower_types = 4;
  c->max_episode_steps = 1200;
  c->max_cluster_length = 8;
  c->max_num_of_roads = 3;
}

td_handle* td_create(const td_config* cfg, int map_size, int n_boards, int mode, int multi_action, int difficulty,
                     int device) {
  if (!cfg) { fail("td_create: cfg is NULL"); return nullptr; }
  if (check_cfg(*cfg)) return nullptr;
  if (map_size < 4 || map_size > 32) { fail("map_size must be in [4, 32], got %d", map_size); return nullptr; }
  if (n_boards < 1) { fail("n_boards must be >= 1"); return nullptr; }
  if (mode < 0 || mode > 2) { fail("mode must be 0 (def), 1 (atk) or 2 (2p)"); return nullptr; }
  if (mode == TD_MODE_DEF && (difficulty < 0 || difficulty > 1)) { fail("TD-def difficulty must be 0 or 1 (random_enemy_lv0/lv1)"); return nullptr; }
  if (mode == TD_MODE_ATK && (difficulty < 0 || difficulty > 2)) { fail("TD-atk difficulty must be 0, 1 or 2 (random_tower_lv0/1/2)"); return nullptr; }
  if (mode == TD_MODE_ATK && multi_action) { fail("TD-atk has no multi-action defender"); return nullptr; }
  if (hipSetDevice(device) != hipSuccess) {
    fail("hipSetDevice(%d) failed: %s", device, hipGetErrorString(hipGetLastError()));
    return nullptr;
  }
  td_handle* h = new td_handle();
  h->L = map_size; h->NC = map_size * map_size; h->B = n_boards; h->mode = mode; h->multi = multi_action ? 1 : 0;
  h->difficulty = difficulty; h->device = device; h->lw = layout_words(map_size);
  h->scratch_stride = (sizeof(RoadResume) + road_scratch_bytes(map_size) + 15) & ~(size_t)15;
  h->stage_cap = std::min(n_boards, 4096);
  build_dev_cfg(*cfg, h->dcfg);
  const size_t B = (size_t)n_boards;
  int rc = 0;
  rc |= dalloc(&h->d_cfg, NCFG);
  rc |= dalloc(&h->d_hdr, B);
  rc |= dalloc(&h->d_en_lp, B * ECAP);
  rc |= dalloc(&h->d_en_mg, B * ECAP);
  rc |= dalloc(&h->d_en_inf, B * ECAP);
  rc |= dalloc(&h->d_tw_cd, B * TCAP);
  rc |= dalloc(&h->d_tw_inf, B * TCAP);
  rc |= dalloc(&h->d_cells, B * h->NC);
  rc |= dalloc(&h->d_opp, B * OPP_WORDS);
  rc |= dalloc(&h->d_hot, B * HOT_WORDS);
  rc |= dalloc(&h->d_np, B * OPP_WORDS);
  rc |= dalloc(&h->d_nxt, (size_t)B * NSLOT * slot_words(map_size));
  rc |= dalloc(&h->d_lay_head, B);
  rc |= dalloc(&h->d_lay_tail, B);
  rc |= dalloc(&h->d_lay_claim, B);
  rc |= dalloc(&h->d_ovr_idx, B);
  rc |= dalloc(&h->d_scratch, B * h->scratch_stride);
  rc |= dalloc(&h->d_mask, B);
  rc |= dalloc(&h->d_fail, B);
  rc |= dalloc(&h->d_stage, (size_t)h->stage_cap * h->lw);
  rc |= dalloc(&h->d_epstats, 2);
  rc |= dalloc(&h->d_lastep, B);
  rc |= dalloc(&h->d_guard_to, 1);
  if (rc) {  // name the footprint (the staged-layout rings are most of it at large L)
    const double ring = (double)B * NSLOT * slot_words(map_size) * 4.0;
    const double total = (double)B * (sizeof(TdHdr) + ECAP * 20 + TCAP * 12 + (size_t)h->NC * 4 + 2 * OPP_WORDS * 4 +
                                      HOT_WORDS * 4 + 12 + h->scratch_stride + 2 + sizeof(td_episode_record)) + ring;
    std::string e = g_err;
    fail("td_create: %d boards at L = %d need %.1f MB of device memory (%.1f MB of it the staged-layout rings, "
         "%d x %d words per board): %s", n_boards, map_size, total / 1e6, ring / 1e6, NSLOT, slot_words(map_size),
         e.c_str());
  }
  if (!rc) {  // win = -1: no finished episode yet
    std::vector<td_episode_record> init((size_t)B, td_episode_record{0.0, 0, -1});
    if (hipMemcpy(h->d_lastep, init.data(), B * sizeof(td_episode_record), hipMemcpyHostToDevice) != hipSuccess)
      rc = fail("episode records init");
  }
  if (!rc && hipMemcpy(h->d_cfg, &h->dcfg, sizeof(TdDevCfg), hipMemcpyHostToDevice) != hipSuccess) rc = fail("cfg upload");
  for (int q = 0; q < kSideStreams && !rc; ++q) {  // side streams (layout refills)
    const hipError_t e = hipStreamCreateWithFlags(&h->side[q], hipStreamNonBlocking);
    if (e != hipSuccess) rc = fail("side stream: %s", hipGetErrorString(e));
  }
  if (!rc && hipEventCreateWithFlags(&h->ev_main, hipEventDisableTiming) != hipSuccess) rc = fail("event");
  {
    // The step-cadence refill needs the previous step finished, not its memory fenced:
    // everything a refill reads of a step (lay_head) and publishes (slots, tags, claims,
    // the stream) goes through write-through / atomic accesses.  Without the event's
    // system-scope fence (a cache writeback): -0.6 % / -0.8 % per step at 8,192 / 4,096
    // boards (profiles/r03/s17).
    const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
    if (!rc && hipEventCreateWithFlags(&h->ev_step, fl) != hipSuccess) rc = fail("event");
  }
  if (rc) { std::string e = g_err; td_destroy(h); g_err = e; return nullptr; }
  {  // TD_KERNEL_AUTO: the small-batch kernel where the whole batch is one round of waves,
     // two waves per board up to half a round -- and again over a few rounds, where the
     // second wave's half of the observation shortens every board's step more than the
     // halved residency costs (single-action boards, profiles/r03/s7, same box: 10x10
     // 12,288 / 16,384 boards 237.8 / 255.4 vs 224.0 / 238.5 M env-steps/s with the large
     // kernel, 32,768 a tie; 30x30 16,384 / 32,768 boards 30.8 / 31.9 vs 29.8 / 31.2 M, 65,536
     // 30.0 vs 30.2 M; TD-2p 20x20 multi-action at 16,384: 48.0 vs 51.5 M in round 3, 54.0 vs
     // 52.1 M on the round-4 build, r04/s10).
     // td_set_step_kernel overrides.
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const int resident = step_resident_boards(base_args(h), cus, 1);
    const int resident2 = step_resident_boards(base_args(h), cus, 2);
    // two-wave kernel up to this many rounds (TD-2p 20x20 multi-action at 16,384 boards:
    // 303.3-303.6 vs 314-315 us per step with the large kernel, profiles/r04/s10; TD-def
    // 10x10 at every batch above one round since round 5: 32,768 / 49,152 / 65,536 boards
    // 107.5-107.9 / 156.5-156.8 / 203.4-204.1 vs 111.7-111.9 / 160.6-160.9 / 208.2-208.4 us,
    // profiles/r05/s33, s34)
    const int rounds2 = h->multi ? (h->L == 20 && h->mode == TD_MODE_2P ? 8 : 0)
                                 : h->L == 10 ? (h->mode == TD_MODE_DEF ? (1 << 20) : 3) : h->L == 30 ? 10 : 0;
    h->small_auto = n_boards <= resident2                            ? 2
                    : n_boards <= resident                           ? 1
                    : (int64_t)n_boards <= (int64_t)rounds2 * resident ? 2
                                                                     : 0;
    if (apply_kernel(h, h->small_auto)) { std::string e = g_err; td_destroy(h); g_err = e; return nullptr; }
  }
  std::vector<uint32_t> seeds(B);
  for (size_t b = 0; b < B; ++b) seeds[b] = (uint32_t)b;
  if (td_seed(h, seeds.data(), seeds.data()) != 0) { std::string e = g_err; td_destroy(h); g_err = e; return nullptr; }
  return h;
}

void td_destroy(td_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  void* dptrs[] = {h->d_cfg, h->d_hdr, h->d_en_lp, h->d_en_mg, h->d_en_inf, h->d_tw_cd, h->d_tw_inf,
                   h->d_cells, h->d_opp, h->d_hot, h->d_np, h->d_nxt, h->d_scratch, h->d_lay_head, h->d_lay_tail,
                   h->d_lay_claim, h->d_ovr_idx, h->d_mask, h->d_fail, h->d_stage, h->d_epstats, h->d_lastep,
                   h->d_guard_to};
  for (void* p : dptrs)
    if (p) (void)hipFree(p);
  if (h->ev_main) (void)hipEventDestroy(h->ev_main);
  if (h->ev_step) (void)hipEventDestroy(h->ev_step);
  for (hipEvent_t e : h->tev) (void)hipEventDestroy(e);
  for (int q = 0; q < kSideStreams; ++q)
    if (h->side[q]) (void)hipStreamDestroy(h->side[q]);
  delete h;
}

// paramConfig on a live engine (TDParam.py:98-100).  The reference reads most values
// live from `config`, but an Enemy / Tower keeps the stats it was created (or upgraded)
// with and a TDBoard the max_cost / base_LP of its reset.  So a new block becomes the
// current epoch; entities keep referring to the block of their own epoch.  Blocks are
// recycled only when no live enemy or tower refers to them (td_cfg_usage_kernel).
int td_set_config(td_handle* h, const td_config* cfg) {
  if (!h || !cfg) return fail("td_set_config: NULL argument");
  if (check_cfg(*cfg)) return -1;
  TdDevCfg d;
  build_dev_cfg(*cfg, d);
  HIP_OK(hipDeviceSynchronize());
  if (std::memcmp(&d, &h->dcfg, sizeof d) == 0) return 0;  // nothing changed
  int slot = -1;
  if (h->cfg_fresh < NCFG) {
    slot = h->cfg_fresh++;
  } else {
    uint32_t* d_used = nullptr;
    HIP_OK(hipMalloc((void**)&d_used, NCFG / 8));
    HIP_OK(hipMemset(d_used, 0, NCFG / 8));
    StepArgs a = base_args(h);
    const hipError_t e = launch_cfg_usage(a, d_used, nullptr);
    uint32_t used[NCFG / 32];
    const hipError_t e2 = e == hipSuccess ? hipMemcpy(used, d_used, sizeof used, hipMemcpyDeviceToHost) : e;
    (void)hipFree(d_used);
    HIP_OK(e2);
    for (int k = 0; k < NCFG && slot < 0; ++k)
      if (k != h->epoch && !((used[k / 32] >> (k % 32)) & 1u)) slot = k;
    if (slot < 0) return fail("td_set_config: %d configs are still referenced by live enemies/towers", NCFG);
  }
  HIP_OK(hipMemcpy(h->d_cfg + slot, &d, sizeof d, hipMemcpyHostToDevice));
  h->dcfg = d;
  h->epoch = slot;
  return 0;
}

// Both mode setters first wait for the device: a refill may still be drawing on a side
// stream.  Layouts staged so far stay valid for random_agent=True (they are the stream's
// next layouts, in order), so turning auto-reset off keeps them for explicit resets.
int td_config_epoch(td_handle* h) { return h ? h->epoch : fail("NULL handle"); }

int td_set_autoreset(td_handle* h, int on) {
  if (!h) return fail("NULL handle");
  HIP_OK(hipDeviceSynchronize());
  h->autoreset = on ? 1 : 0;
  h->since_guard = kGuardEvery;
  return 0;
}

// random_agent=False interleaves the opponent's draws with the layout draws on one
// stream, so no layout may have been drawn ahead of play: refused while any board has a
// staged layout or a pending draw (td_seed with new numpy seeds, or running the staged
// layouts out with explicit resets, clears them).
int td_set_random_agent(td_handle* h, int random_agent) {
  if (!h) return fail("NULL handle");
  HIP_OK(hipDeviceSynchronize());
  h->since_guard = kGuardEvery;
  if (!random_agent && !h->opp_np) {
    std::vector<uint32_t> head((size_t)h->B), tail((size_t)h->B);
    HIP_OK(hipMemcpy(head.data(), h->d_lay_head, (size_t)h->B * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(tail.data(), h->d_lay_tail, (size_t)h->B * 4, hipMemcpyDeviceToHost));
    std::vector<RoadResume> res((size_t)h->B);
    HIP_OK(hipMemcpy2D(res.data(), sizeof(RoadResume), h->d_scratch, h->scratch_stride, sizeof(RoadResume),
                       (size_t)h->B, hipMemcpyDeviceToHost));
    for (int b = 0; b < h->B; ++b)
      if (head[(size_t)b] != tail[(size_t)b] || res[(size_t)b].phase != RP_NEW)
        return fail("random_agent=False: board %d has layouts drawn ahead of play (auto-reset refills); "
                    "set it before the first reset, or re-seed the layout streams first", b);
  }
  h->opp_np = random_agent ? 0 : 1;
  return 0;
}

int td_seed(td_handle* h, const uint32_t* np_seeds, const uint32_t* py_seeds) {
  if (!h) return fail("NULL handle");
  const size_t B = (size_t)h->B;
  if (np_seeds) {
    std::vector<uint32_t> nw(B * OPP_WORDS);
    parallel_for((int)B, [&](int b) {
      uint32_t* w = &nw[(size_t)b * OPP_WORDS];
      np_seed(w, np_seeds[b]);
      w[MT_N + 1] = MT_N;  // no lazy words
    });
    if (drop_all_staged(h)) return -1;
    HIP_OK(hipMemcpy(h->d_np, nw.data(), B * OPP_WORDS * 4, hipMemcpyHostToDevice));
  }
  if (py_seeds) {
    std::vector<uint32_t> op(B * OPP_WORDS);
    parallel_for((int)B, [&](int b) {
      uint32_t* w = &op[(size_t)b * OPP_WORDS];
      py_seed(w, py_seeds[b]);
      w[MT_N + 1] = MT_N;  // no lazy words
    });
    std::vector<uint32_t> hot(B * HOT_WORDS, 0u);
    for (size_t b = 0; b < B; ++b) { hot[b * HOT_WORDS] = MT_N; hot[b * HOT_WORDS + 1] = MT_N; }
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(h->d_opp, op.data(), B * OPP_WORDS * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(h->d_hot, hot.data(), B * HOT_WORDS * 4, hipMemcpyHostToDevice));
  }
  return 0;
}

int td_set_py_state(td_handle* h, int b, const uint32_t* mt) {
  if (!h || b < 0 || b >= h->B || !mt) return fail("bad board or NULL state");
  uint32_t w[OPP_WORDS];
  std::memcpy(w, mt, (MT_N + 1) * 4);
  w[MT_N + 1] = MT_N;
  uint32_t hot[HOT_WORDS] = {w[MT_N], MT_N, 0u};
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(h->d_opp + (size_t)b * OPP_WORDS, w, sizeof w, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(h->d_hot + (size_t)b * HOT_WORDS, hot, sizeof hot, hipMemcpyHostToDevice));
  return 0;
}
// The device keeps the opponent's position in the hot record and may have
// pre-drawn (and lazily twisted) ahead of it; the exported state is CPython's
// getstate() form of the same stream (equal future draws).
int td_get_py_state(td_handle* h, int b, uint32_t* mt) {
  if (!h || b < 0 || b >= h->B || !mt) return fail("bad board or NULL state");
  uint32_t w[OPP_WORDS], hot[HOT_WORDS];
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(w, h->d_opp + (size_t)b * OPP_WORDS, sizeof w, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(hot, h->d_hot + (size_t)b * HOT_WORDS, sizeof hot, hipMemcpyDeviceToHost));
  w[MT_N] = hot[0];
  w[MT_N + 1] = hot[1];
  mt_finish_lazy(w);
  std::memcpy(mt, w, (MT_N + 1) * 4);
  return 0;
}
int td_get_np_state(td_handle* h, int b, uint32_t* mt) {
  if (!h || b < 0 || b >= h->B || !mt) return fail("bad board or NULL state");
  uint32_t w[OPP_WORDS];
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(w, h->d_np + (size_t)b * OPP_WORDS, sizeof w, hipMemcpyDeviceToHost));
  mt_finish_lazy(w);
  std::memcpy(mt, w, (MT_N + 1) * 4);
  return 0;
}
int td_set_np_state(td_handle* h, int b, const uint32_t* mt) {
  if (!h || b < 0 || b >= h->B || !mt) return fail("bad board or NULL state");
  uint32_t w[OPP_WORDS];
  std::memcpy(w, mt, (MT_N + 1) * 4);
  w[MT_N + 1] = MT_N;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(h->d_np + (size_t)b * OPP_WORDS, w, sizeof w, hipMemcpyHostToDevice));
  return drop_staged(h, b);
}

int td_reset(td_handle* h, const uint8_t* host_mask, float* obs, void* stream) {
  if (!h) return fail("NULL handle");
  hipStream_t s = (hipStream_t)stream;
  std::vector<uint8_t> mask((size_t)h->B, 1);
  if (host_mask) std::memcpy(mask.data(), host_mask, (size_t)h->B);
  HIP_OK(hipDeviceSynchronize());
  if (run_reset(h, mask, obs, s)) return -1;
  std::vector<uint8_t> fl((size_t)h->B);
  HIP_OK(hipMemcpy(fl.data(), h->d_fail, (size_t)h->B, hipMemcpyDeviceToHost));
  h->last_reset_failed.clear();
  for (int b = 0; b < h->B; ++b)
    if (mask[(size_t)b] && fl[(size_t)b]) h->last_reset_failed.push_back(b);
  return (int)h->last_reset_failed.size();
}

int td_last_reset_failures(td_handle* h, int32_t* boards, int cap) {
  if (!h) return fail("NULL handle");
  int n = (int)h->last_reset_failed.size();
  for (int i = 0; i < n && i < cap && boards; ++i) boards[i] = h->last_reset_failed[(size_t)i];
  return n;
}

int td_reset_layouts(td_handle* h, const uint32_t* recs, const int32_t* boards, int n, float* obs, void* stream) {
  if (!h || (n > 0 && (!recs || !boards))) return fail("td_reset_layouts: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < n; ++i)
    if (boards[i] < 0 || boards[i] >= h->B || recs[(size_t)i * h->lw] != TD_LAYOUT_MAGIC)
      return fail("td_reset_layouts: bad board id or layout record %d", i);
  HIP_OK(hipDeviceSynchronize());
  std::vector<int32_t> idx((size_t)h->B, -1);
  for (int i0 = 0; i0 < n; i0 += h->stage_cap) {
    const int m = std::min(h->stage_cap, n - i0);
    std::vector<uint8_t> mask((size_t)h->B, 0);
    std::fill(idx.begin(), idx.end(), -1);
    for (int i = 0; i < m; ++i) { idx[(size_t)boards[i0 + i]] = i; mask[(size_t)boards[i0 + i]] = 1; }
    HIP_OK(hipMemcpy(h->d_stage, recs + (size_t)i0 * h->lw, (size_t)m * h->lw * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(h->d_ovr_idx, idx.data(), (size_t)h->B * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(h->d_mask, mask.data(), (size_t)h->B, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(h->d_fail, 0, (size_t)h->B));
    StepArgs a = base_args(h);
    a.obs = obs;
    a.reset_mask = h->d_mask;
    a.ovr_idx = h->d_ovr_idx;
    a.ovr_rec = h->d_stage;
    HIP_OK(launch_step(a, s, true));
    h->since_guard = kGuardEvery;
    HIP_OK(hipStreamSynchronize(s));
  }
  return 0;
}

int td_step(td_handle* h, const td_step_io* io, void* stream) {
  if (!io) return fail("td_step: NULL io");
  // The two header words first (every td_step_io of any ABI has >= 8 bytes): a caller
  // built against another layout is refused before any pointer of its struct is read.
  if (io->size != (uint32_t)sizeof(td_step_io) || io->abi != (uint32_t)TD_ABI_VERSION)
    return fail("td_step: td_step_io has size %u / abi %u, this library expects size %u / abi %d "
                "(set io.size = sizeof(td_step_io) and io.abi = TD_ABI_VERSION, or call td_step_io_init; "
                "an ABI-2 struct has no header)",
                io->size, io->abi, (unsigned)sizeof(td_step_io), TD_ABI_VERSION);
  if (!h) return fail("td_step: NULL handle");
  if (!io->obs || !io->reward || !io->done) return fail("td_step: obs, reward and done are required");
  if (h->mode != TD_MODE_ATK && !io->def_act) return fail("td_step: def_act required in this mode");
  if (h->mode != TD_MODE_DEF && !io->atk_act) return fail("td_step: atk_act required in this mode");
  hipStream_t s = (hipStream_t)stream;
  StepArgs a = base_args(h);
  a.def_act = io->def_act; a.atk_act = io->atk_act; a.obs = io->obs; a.reward = io->reward; a.done = io->done;
  a.real_def = io->real_def; a.real_atk = io->real_atk; a.fail_def = io->fail_def; a.fail_atk = io->fail_atk;
  a.win = io->win; a.allow_next = io->allow_next; a.ep_return = io->ep_return; a.ep_len = io->ep_len;
  a.cooldowns = io->cooldowns;
  a.ep_stats = h->d_epstats;
  a.last_ep = h->d_lastep;
  // the refill goes first: it waits for the previous step only, so a board whose ring
  // is dry in this step can wait for it (td_step.hip step_board) without a cycle
  // random_agent=True: layouts are staged ahead by refills on the side streams.
  // random_agent=False: they are drawn in stream order right after the step (below).
  if (h->autoreset && !h->opp_np && h->refill_every > 0 && (h->steps % h->refill_every) == 0 &&
      start_refill(h, s, true))
    return -1;
  // the ring guard (kGuardEvery): behind the previous step, beside the refill just launched
  if (h->autoreset && !h->opp_np && h->guard_every > 0 && h->since_guard >= h->guard_every) {
    HIP_OK(launch_refill(a, s, h->guard_every));
    h->since_guard = 0;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->tev_n < h->tev_cap && (h->steps - h->tev_from) % h->tev_every == 0) {
    e0 = h->tev[2 * (size_t)h->tev_n];
    e1 = h->tev[2 * (size_t)h->tev_n + 1];
    h->tev_n += 1;
  }
  HIP_OK(launch_step(a, s, false, e0, e1));
  if (h->autoreset && h->opp_np) HIP_OK(launch_autoreset(a, s));
  h->steps += 1;
  h->since_guard += 1;
  return 0;
}

int td_set_step_kernel(td_handle* h, int kind) {
  if (!h) return fail("NULL handle");
  if (kind < TD_KERNEL_AUTO || kind > TD_KERNEL_SMALL2) return fail("td_set_step_kernel: unknown kernel kind %d", kind);
  if (kind >= TD_KERNEL_SMALL && h->L != 10 && h->L != 20 && h->L != 30)
    return fail("td_set_step_kernel: L = %d has no small-batch step kernel (only L = 10 / 20 / 30)", h->L);
  HIP_OK(hipDeviceSynchronize());  // launches already queued keep the kernel they were enqueued with
  return apply_kernel(h, kind == TD_KERNEL_AUTO ? h->small_auto : kind - 1);
}

int td_step_kernel(td_handle* h) { return h ? h->small + 1 : fail("NULL handle"); }

const char* td_step_kernel_name(td_handle* h) { return h ? h->kernel_name.c_str() : ""; }

int td_set_refill_interval(td_handle* h, int steps) {
  if (!h || steps < 0) return fail("td_set_refill_interval: bad arguments");
  h->refill_every = steps;
  return 0;
}

int td_kernel_timing(td_handle* h, int max_launches, int every) {
  if (!h || max_launches < 0 || every < 1) return fail("td_kernel_timing: bad arguments");
  HIP_OK(hipDeviceSynchronize());
  // Timing events without the system-scope release at the timed kernel's end: the cache
  // write-back it implies lengthens the very kernel being timed (4,096 boards: sampled
  // kernels 21.9 us = the 21.9-us step with it, 20.6 us in a 21.3-us step without;
  // profiles/r04/s2).
  const unsigned flags = hipEventDisableSystemFence;
  while ((int)h->tev.size() < 2 * max_launches) {
    hipEvent_t e = nullptr;
    HIP_OK(hipEventCreateWithFlags(&e, flags));
    h->tev.push_back(e);
  }
  h->tev_cap = max_launches;
  h->tev_n = 0;
  h->tev_every = every;
  h->tev_from = h->steps;
  return 0;
}

int td_kernel_times(td_handle* h, float* us, int cap) {
  if (!h || (cap > 0 && !us)) return fail("td_kernel_times: bad arguments");
  const int n = h->tev_n;
  for (int i = 0; i < n && i < cap; ++i) {
    HIP_OK(hipEventSynchronize(h->tev[2 * (size_t)i + 1]));
    float ms = 0.0f;
    HIP_OK(hipEventElapsedTime(&ms, h->tev[2 * (size_t)i], h->tev[2 * (size_t)i + 1]));
    us[i] = ms * 1000.0f;
  }
  return n;
}

int td_episode_stats(td_handle* h, double* dev_out, int clear, void* stream) {
  if (!h || !dev_out) return fail("td_episode_stats: NULL argument");
  hipStream_t s = (hipStream_t)stream;
  HIP_OK(hipMemcpyAsync(dev_out, h->d_epstats, 2 * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (clear) HIP_OK(hipMemsetAsync(h->d_epstats, 0, 2 * sizeof(double), s));
  return 0;
}

int td_opponent(td_handle* h, int side, int level, const uint8_t* host_mask, void* stream) {
  if (!h) return fail("NULL handle");
  if (side == 0 && (level < 0 || level > 1)) return fail("td_opponent: random_enemy_lv%d does not exist", level);
  if (side == 1 && (level < 0 || level > 2)) return fail("td_opponent: random_tower_lv%d does not exist", level);
  if (side != 0 && side != 1) return fail("td_opponent: side must be 0 (enemy) or 1 (tower)");
  hipStream_t s = (hipStream_t)stream;
  std::vector<uint8_t> mask((size_t)h->B, 1);
  if (host_mask) std::memcpy(mask.data(), host_mask, (size_t)h->B);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(h->d_mask, mask.data(), (size_t)h->B, hipMemcpyHostToDevice));
  StepArgs a = base_args(h);
  a.reset_mask = h->d_mask;
  HIP_OK(launch_opponent(a, side, level, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

int td_episode_records(td_handle* h, td_episode_record* dev_out, void* stream) {
  if (!h || !dev_out) return fail("td_episode_records: NULL argument");
  HIP_OK(hipMemcpyAsync(dev_out, h->d_lastep, (size_t)h->B * sizeof(td_episode_record), hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return 0;
}

int td_layout_words(int map_size) { return layout_words(map_size); }

int td_layout_from_roads(int map_size, int num_roads, const int32_t* cells, const int32_t* offsets, uint32_t* rec) {
  int st = layout_from_roads(map_size, num_roads, cells, offsets, rec);
  return st == ROAD_OK ? 0 : fail("td_layout_from_roads: invalid roads (status %d)", st);
}

int td_layout_generate(uint32_t* np_state625, int map_size, int max_attempts, uint32_t* rec) {
  if (map_size < 4 || map_size > MAX_L) return fail("map_size out of range");
  std::vector<uint8_t> scratch(road_scratch_bytes(map_size));
  return episode_layout(np_state625, map_size, scratch.data(), max_attempts > 0 ? max_attempts : kRoadAttempts, rec);
}

size_t td_state_bytes(td_handle* h, int count) {
  if (!h || count < 0) return 0;
  return (size_t)count * (sizeof(TdHdr) + ECAP * (8 + 8 + 4) + TCAP * (8 + 4) + (size_t)h->NC * 4 + OPP_WORDS * 4);
}

static int state_copy(td_handle* h, int b0, int count, void* host, bool to_host) {
  if (!h || b0 < 0 || count < 0 || b0 + count > h->B) return fail("state copy: bad board range");
  HIP_OK(hipDeviceSynchronize());
  uint8_t* p = (uint8_t*)host;
  auto cp = [&](void* dev, size_t elem) -> int {
    size_t bytes = (size_t)count * elem;
    uint8_t* d = (uint8_t*)dev + (size_t)b0 * elem;
    HIP_OK(hipMemcpy(to_host ? (void*)p : (void*)d, to_host ? (void*)d : (void*)p, bytes,
                     to_host ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice));
    p += bytes;
    return 0;
  };
  uint32_t* opp = (uint32_t*)(p + (size_t)count * (sizeof(TdHdr) + ECAP * 20 + TCAP * 12 + (size_t)h->NC * 4));
  std::vector<uint8_t> retagged;
  if (!to_host) {
    // imported enemies and towers take the current config epoch: epoch tags of another
    // engine (or of blocks since recycled) mean nothing here
    retagged.assign(p, p + td_state_bytes(h, count));
    uint8_t* q = retagged.data();
    uint32_t* einf = (uint32_t*)(q + (size_t)count * (sizeof(TdHdr) + ECAP * 16));
    uint32_t* tinf = (uint32_t*)(q + (size_t)count * (sizeof(TdHdr) + ECAP * 20 + TCAP * 8));
    for (size_t i = 0; i < (size_t)count * ECAP; ++i) einf[i] = (einf[i] & 0x00ffffffu) | ((uint32_t)h->epoch << 24);
    for (size_t i = 0; i < (size_t)count * TCAP; ++i)
      tinf[i] = (tinf[i] & 0x0000ffffu) | ((uint32_t)h->epoch << 16) | ((uint32_t)h->epoch << 24);
    // cell words: bits 10-15 are not part of the layout format (the step keeps the tower of a
    // cell there in LDS only)
    uint32_t* cw = (uint32_t*)(q + (size_t)count * (sizeof(TdHdr) + ECAP * 20 + TCAP * 12));
    for (size_t i = 0; i < (size_t)count * h->NC; ++i) cw[i] &= ~(0x3Fu << 10);
    p = q;
    opp = (uint32_t*)(p + (size_t)count * (sizeof(TdHdr) + ECAP * 20 + TCAP * 12 + (size_t)h->NC * 4));
  }
  std::vector<uint32_t> hot((size_t)count * HOT_WORDS);
  if (!to_host) {  // the hot record follows the imported words (no pre-drawn outputs)
    for (int i = 0; i < count; ++i) {
      hot[(size_t)i * HOT_WORDS] = opp[(size_t)i * OPP_WORDS + MT_N];
      hot[(size_t)i * HOT_WORDS + 1] = opp[(size_t)i * OPP_WORDS + MT_N + 1];
    }
    HIP_OK(hipMemcpy(h->d_hot + (size_t)b0 * HOT_WORDS, hot.data(), hot.size() * 4, hipMemcpyHostToDevice));
  }
  if (cp(h->d_hdr, sizeof(TdHdr)) || cp(h->d_en_lp, ECAP * 8) || cp(h->d_en_mg, ECAP * 8) ||
      cp(h->d_en_inf, ECAP * 4) || cp(h->d_tw_cd, TCAP * 8) || cp(h->d_tw_inf, TCAP * 4) ||
      cp(h->d_cells, (size_t)h->NC * 4) || cp(h->d_opp, OPP_WORDS * 4))
    return -1;
  if (to_host) {  // position and lazy boundary live in the hot record
    HIP_OK(hipMemcpy(hot.data(), h->d_hot + (size_t)b0 * HOT_WORDS, hot.size() * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < count; ++i) {
      opp[(size_t)i * OPP_WORDS + MT_N] = hot[(size_t)i * HOT_WORDS];
      opp[(size_t)i * OPP_WORDS + MT_N + 1] = hot[(size_t)i * HOT_WORDS + 1];
    }
  }
  return 0;
}

int td_export_state(td_handle* h, int b0, int count, void* host_dst) { return state_copy(h, b0, count, host_dst, true); }

// A record whose board has a layout must carry the captured max_cost / max_base_LP the
// step divides by (TdHdr.format: header format 2); a record of another format, or a
// hand-built one with zeros there, would silently clamp every cost to 0 and divide the
// observation's scalar channels by zero.
int td_import_state(td_handle* h, int b0, int count, const void* host_src) {
  if (!h || !host_src || b0 < 0 || count < 0 || b0 + count > h->B) return fail("td_import_state: bad arguments");
  const TdHdr* hdr = static_cast<const TdHdr*>(host_src);
  for (int i = 0; i < count; ++i) {
    const TdHdr& x = hdr[i];
    if (x.num_roads < 1 || x.num_roads > 3) continue;  // a board never reset: nothing is stepped
    if (x.format != kHdrFormat)
      return fail("td_import_state: board %d: header format 0x%x, expected 0x%x (a record of another build?)",
                  b0 + i, (unsigned)x.format, (unsigned)kHdrFormat);
    if (!(x.max_cost > 0.0) || x.max_base_LP < 1)
      return fail("td_import_state: board %d: max_cost %g / max_base_LP %d (must be > 0 / >= 1)", b0 + i, x.max_cost,
                  x.max_base_LP);
    if (x.n_en < 0 || x.n_en > ECAP || x.n_tw < 0 || x.n_tw > TCAP)
      return fail("td_import_state: board %d: %d enemies / %d towers exceed the capacity", b0 + i, x.n_en, x.n_tw);
  }
  return state_copy(h, b0, count, const_cast<void*>(host_src), false);
}

int td_get_flags(td_handle* h, int32_t* host_flags) {
  if (!h || !host_flags) return fail("td_get_flags: NULL argument");
  std::vector<TdHdr> hdr((size_t)h->B);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(hdr.data(), h->d_hdr, hdr.size() * sizeof(TdHdr), hipMemcpyDeviceToHost));
  for (int b = 0; b < h->B; ++b) host_flags[b] = hdr[(size_t)b].flags;
  return 0;
}



// Diagnostic: hold (1) or give back (0) board b's refill claim, as a refill wave drawing
// its layouts would (tests: a claim held past the ring guard's 1-s wait).
int td_debug_set_claim(td_handle* h, int b, int held) {
  if (!h || b < 0 || b >= h->B) return fail("td_debug_set_claim: bad board");
  HIP_OK(hipDeviceSynchronize());
  const uint32_t v = held ? 1u : 0u;
  HIP_OK(hipMemcpy(h->d_lay_claim + b, &v, 4, hipMemcpyHostToDevice));
  return 0;
}

int td_guard_timeouts(td_handle* h, int clear) {
  if (!h) return fail("NULL handle");
  uint32_t n = 0;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(&n, h->d_guard_to, 4, hipMemcpyDeviceToHost));
  if (clear) HIP_OK(hipMemset(h->d_guard_to, 0, 4));
  return (int)std::min<uint32_t>(n, 0x7fffffffu);
}

int td_set_store_policy(td_handle* h, int xcd_map, int edge_wt) {
  if (!h || (xcd_map != 0 && xcd_map != 1) || (edge_wt != 1 && edge_wt != 2))
    return fail("td_set_store_policy: xcd_map must be 0 / 1 and edge_wt 1 / 2");
  HIP_OK(hipDeviceSynchronize());
  h->xcd_map = xcd_map;
  h->edge_wt = edge_wt;
  return 0;
}

int td_board_map(int n_boards, int kind, int xcd_map, int32_t* out) {
  if (n_boards < 1 || !out || kind < 0 || kind > 1) return fail("td_board_map: bad arguments");
  for (int i = 0; i < n_boards; ++i)
    out[i] = xcd_map ? xcd_board(i, n_boards) : i;
  return 0;
}

void td_py_seed(uint32_t* mt, uint32_t seed) { py_seed(mt, seed); }
void td_np_seed(uint32_t* mt, uint32_t seed) { np_seed(mt, seed); }
uint32_t td_mt_next(uint32_t* mt) { return MtRef{mt}.next(); }
int64_t td_py_randint(uint32_t* mt, int64_t a, int64_t b) { return MtRef{mt}.py_randint(a, b); }
int64_t td_np_randint(uint32_t* mt, int64_t lo, int64_t hi) { return MtRef{mt}.np_randint(lo, hi); }

}  // extern "C"
