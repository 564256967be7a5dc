/* tdstep.h -- C-ABI of the MI355X-native batched gym-TD step (libtdstep.so).
 *
 * The reference (LiuTed/gym-TD) is pure Python: its only boundary is the gym.Env
 * surface.  Each entry point below replaces one piece of that surface for a batch
 * of B independent boards that live in HBM; the Python mirror
 * (gym-td_amd/gym_TD) binds them with ctypes:
 *
 *   td_create / td_destroy     TDGymBasic.__init__            gym_TD/envs/TDGymBasic.py:18-28
 *                              TDDefense/TDAttack/TDMulti.__init__ (TDDefense.py:19-26,
 *                              TDAttack.py:18-22, TDMulti.py:16-31)
 *   td_set_config              paramConfig                    gym_TD/envs/TDParam.py:98-100
 *   td_seed                    TDGymBasic.seed                TDGymBasic.py:30-32 (+ the opponent's
 *                              `random` stream, TDGymBasic.py:84-86,98-100)
 *   td_reset                   TDGymBasic.reset               TDGymBasic.py:37-55
 *   td_step                    TDDefense.step / TDAttack.step / TDMulti.step
 *                              (TDDefense.py:34-87, TDAttack.py:27-56, TDMulti.py:46-138)
 *                              -> TDBoard.step/done/get_states (TDBoard.py:295-385, 85-144)
 *   td_layout_generate         TDRoadGen.create_road_v2       TDRoadGen.py:4-199 (+ map planes
 *                              TDBoard.py:31-59)
 *   td_layout_from_roads       TDBoard.__init__ map planes    TDBoard.py:31-59
 *   td_export_state / import   the board's Python attributes (enemies, towers, costs, map[6])
 *
 * Conventions
 *   - every array argument of td_step / td_reset is a caller-owned DEVICE pointer
 *     (e.g. a torch tensor's data_ptr()), work is enqueued on `stream` (a
 *     hipStream_t, NULL = default stream) and the call returns immediately;
 *   - one handle per stream/thread; handles are not thread-safe;
 *   - int return codes: 0 = OK, < 0 = error (td_last_error() has the message);
 *     nothing throws across the ABI;
 *   - per-board error bits (capacity overflow, invalid action, missing layout)
 *     are kept on the device, read them with td_get_flags().
 */
#ifndef TDSTEP_H_
#define TDSTEP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 3: td_step_io starts with its own size and ABI words, which td_step checks before
 * it reads anything else (an ABI-2 struct -- 14 pointers, no header -- is refused).
 * ABI 2: td_step_io.cooldowns.  ABI 1: the first release. */
#define TD_ABI_VERSION 3

enum td_mode { TD_MODE_DEF = 0, TD_MODE_ATK = 1, TD_MODE_2P = 2 };

enum td_board_flag {
  TD_FLAG_EN_OVERFLOW = 1, /* more than 128 live enemies: summon refused */
  TD_FLAG_TW_OVERFLOW = 2, /* more than 32 towers: build refused */
  TD_FLAG_BAD_ACTION = 4,  /* action outside the action space (the reference asserts) */
  TD_FLAG_NO_LAYOUT = 8,   /* auto-reset found no staged layout */
  TD_FLAG_BAD_MOVE = 16,   /* an enemy walked off the board (corrupt layout) */
  TD_FLAG_CLAIM_TIMEOUT = 32 /* a wait for the board's refill claim gave up after 1 s: the ring
                                guard left its ring short, or its episode end found no layout
                                (then TD_FLAG_NO_LAYOUT too); see td_guard_timeouts */
};

/* Game parameters: gym_TD/envs/TDParam.py:1-64 (Config) and :105-111 (HyperParameters).
 * Numbers are doubles so Python ints and floats both round-trip exactly. */
typedef struct td_config {
  double enemy_LP[4][2], enemy_speed[4][2], enemy_defense[4][2], enemy_cost[4][2];
  double tower_attack[4][2], tower_range[4][2], tower_splash_range[4][2];
  double tower_cost[4][2], tower_attack_interval[4][2];
  double tower_destruct_return, frozen_time, frozen_ratio;
  double attacker_init_cost, defender_init_cost, base_LP, max_cost;
  double reward_kill, penalty_leak, reward_time;
  double attacker_cost_init_rate, attacker_cost_final_rate, defender_cost_rate;
  double tower_distance, enemy_upgrade_at;
  double attacker_action_interval, defender_action_interval;
  int32_t max_enemy_lv, max_tower_lv, enemy_types, tower_types;
  int32_t max_episode_steps, max_cluster_length, max_num_of_roads, reserved;
} td_config;

/* Device outputs of one step.  Only obs/reward/done (and the action inputs the
 * mode needs) are required; every other pointer may be NULL.
 *   def_act   int64 [B] (discrete) or [B][6][L][L] (multi-action)   TD-def, TD-2p
 *   atk_act   int64 [B][3][8]                                       TD-atk, TD-2p
 *   obs       float [B][45][L][L]   reward double [B]   done uint8 [B]
 *   real_def  int64 [B] or [B][6][L][L]   real_atk int64 [B][3][8]   info['RealAction']
 *   fail_def  int32 [B]   fail_atk int32 [B][3] (-1 = no entry)       info['FailCode']
 *   win       int8 [B] (-1 = None)                                     info['Win']
 *   allow_next uint8 [B] (bit0 attacker_cd<=1, bit1 defender_cd<=1)   info['AllowNextMove']
 *             (bits 2-7 are always 0)
 *   ep_return double [B], ep_len int32 [B]: running episode return / length after this
 *             step (the finished episode's totals when done[b]).
 *   cooldowns uint8 [B]: the env's attacker_cd (bits 0-3) and defender_cd (bits 4-7) after the
 *             step (TDDefense.py:38-39,75, TDAttack.py:31-32,44), each saturated at 15
 *             (ABI 2; ABI 1 packed them into allow_next bits 2-7).
 *   size, abi: sizeof(td_step_io) and TD_ABI_VERSION as the caller was built (ABI 3;
 *             td_step_io_init sets both).  td_step reads these two words first and refuses,
 *             with no launch, a struct whose size or ABI differs from its own: a caller
 *             built against another layout of this struct is caught, not stepped. */
typedef struct td_step_io {
  uint32_t size;
  uint32_t abi;
  const int64_t* def_act;
  const int64_t* atk_act;
  float* obs;
  double* reward;
  uint8_t* done;
  int64_t* real_def;
  int64_t* real_atk;
  int32_t* fail_def;
  int32_t* fail_atk;
  int8_t* win;
  uint8_t* allow_next;
  double* ep_return;
  int32_t* ep_len;
  uint8_t* cooldowns;
} td_step_io;

typedef struct td_handle td_handle;

int td_abi_version(void);
/* sizeof(td_step_io) as this library was built (120 on LP64 at ABI 3). */
int td_step_io_size(void);
/* Device memory for a caller's output buffers (the observation above all), zeroed;
 * contiguous != 0: physically contiguous where the driver can give it
 * (hipDeviceMallocContiguous), else a plain allocation.  A contiguous observation stepped
 * 4-5 % faster than a default allocation at 10x10 / 65,536 and 20x20 / 30x30 boards in
 * one probe (profiles/r04/s24); TDEngine's choice is TD_CONTIG_OBS (gym_TD/engine.py).
 * The reference allocates its observation per call (np.zeros in TDBoard.get_states,
 * gym_TD/envs/TDBoard.py:85-112); no counterpart.  td_free_device releases it (after the
 * work that writes it is done). */
int td_alloc_device(size_t bytes, int device, int contiguous, void** out);
int td_free_device(void* p);
/* How td_alloc_device placed block p: 1 physically contiguous, 0 a plain allocation (a
 * contiguous request the driver refused falls back to one), -1 not a live td_alloc_device
 * block.  (A placement a caller records -- e.g. to key a measurement by it -- is this one,
 * not the request.) */
int td_alloc_is_contiguous(const void* p);
/* Zero *io and set its size / abi words (a C caller's initialiser; writes td_step_io_size()
 * bytes, so io must be this header's td_step_io). */
void td_step_io_init(td_step_io* io);
const char* td_last_error(void);
void td_config_default(td_config* cfg);

/* Device memory per board: ~8.2 KB + 18*L^2 B of state (records, both RNG streams, the
 * layout draw's scratch) plus a ring of 16 staged layouts of (8 + L^2 rounded up to 32)
 * words each -- ~18 KB at L = 10 (1.2 GB at 65,536 boards), ~84 KB at L = 30 (5.5 GB at
 * 65,536).  A failed allocation names the footprint in td_last_error(). */
/* mode: td_mode; multi_action: HyperParameters.allow_multiple_actions;
 * difficulty: built-in opponent level (TD-def: 0/1, TD-atk: 0/1/2, TD-2p: ignored);
 * map_size: 10/20/30 have specialised kernels, any 4 <= L <= 32 works. */
td_handle* td_create(const td_config* cfg, int map_size, int n_boards, int mode, int multi_action,
                     int difficulty, int device);
void td_destroy(td_handle* h);
/* paramConfig on a live engine (TDParam.py:98-100): values the reference reads live from
 * `config` change from the next step; enemies and towers keep the stats they were created
 * or upgraded with (TDElements.py:4-69, 134-170) and each board the max_cost / base_LP of
 * its last reset (TDBoard.py:66-72) -- the device keeps one constant block per config
 * epoch (up to 256 still referenced by live entities).  td_config_epoch: the current one. */
int td_set_config(td_handle* h, const td_config* cfg);
int td_config_epoch(td_handle* h);
int td_set_autoreset(td_handle* h, int on);
/* TDGymBasic(random_agent=...) (TDGymBasic.py:18-26): with random_agent = 0 the built-in
 * opponents draw from each board's numpy layout stream (np_random, :87-89,101-103,
 * 118-120,139-160,176-177,188-190,213-256) instead of its CPython stream; the destruct
 * branch's tower index stays on CPython random (:191, :287).  Play and reset() then
 * share the stream in order: with auto-reset on, a finished board's next layout is drawn
 * right after the step that ended its episode (a second kernel on the step's stream), as
 * gym's AsyncVectorEnv calls reset() there; nothing is staged ahead.  Switching to 0 is
 * refused while a board holds layouts an auto-reset refill drew ahead of play (set it
 * before the first reset, or re-seed with td_seed).  Both mode setters synchronise the
 * device first. */
int td_set_random_agent(td_handle* h, int random_agent);

/* Board b's layout stream = numpy.random.RandomState(np_seeds[b]) and its built-in
 * opponent stream = random.Random(py_seeds[b]).  Host arrays of n_boards entries. */
int td_seed(td_handle* h, const uint32_t* np_seeds, const uint32_t* py_seeds);
/* CPython `random.getstate()` import/export for one board: 624 words + position. */
int td_set_py_state(td_handle* h, int board, const uint32_t* mt625);
int td_get_py_state(td_handle* h, int board, uint32_t* mt625);
int td_set_np_state(td_handle* h, int board, const uint32_t* mt625);
int td_get_np_state(td_handle* h, int board, uint32_t* mt625);

/* Start a new episode on every board with host_mask[b] != 0 (NULL = all): draws
 * the layout from the board's numpy stream (on the device; with auto-reset on, a
 * layout staged ahead of time by the refill kernel is used), resets the board and
 * writes its initial observation into obs (device, may be NULL).  Synchronous.
 * Returns the number of boards whose road generation failed (the reference raises
 * or hangs there, TDRoadGen.py:177-189); those boards keep their previous state. */
int td_reset(td_handle* h, const uint8_t* host_mask, float* obs, void* stream);

/* Boards whose road generation failed in the last td_reset (ids into boards[0..cap)); returns the count. */
int td_last_reset_failures(td_handle* h, int32_t* boards, int cap);

/* Reset from explicit layout records (td_layout_words(L) uint32 each, host memory). */
int td_reset_layouts(td_handle* h, const uint32_t* recs, const int32_t* boards, int n, float* obs, void* stream);

/* One env step for all boards (asynchronous on `stream`).  Buffers need only their
 * element type's alignment; a 16-B-aligned obs (and, multi-action, 16-B-aligned flag
 * and real-action arrays) takes the line-aligned 16-B store path, any other the
 * per-element one (same bytes, slower). */
int td_step(td_handle* h, const td_step_io* io, void* stream);

/* Which step kernel td_step launches (one wave per board in all three; they differ in
 * occupancy and load schedule, not in results):
 *   TD_KERNEL_LARGE  td_step_kernel        several rounds of waves (7 per SIMD), live slots
 *                                          loaded once the header's counts are in;
 *   TD_KERNEL_SMALL  td_step_kernel_small  one round (8 waves per SIMD), 16 enemy + 16 tower
 *                                          slots prefetched with the header;
 *   TD_KERNEL_SMALL2 td_step_kernel_small2 as SMALL, plus a second wave per board that
 *                                          writes half of the observation;
 *   TD_KERNEL_AUTO   td_create's rule: SMALL2 up to half a round of boards, SMALL up to one
 *                    round, SMALL2 again above that -- at any batch for single-action TD-def
 *                    at L = 10, up to 3 rounds for the other L = 10 modes, 10 rounds at
 *                    L = 30 (single-action) and 8 rounds for TD-2p multi-action at L = 20 --
 *                    else LARGE (L = 10 / 20 / 30; other L only have LARGE).
 * The small kernels need a 16-B-aligned observation buffer; a td_step with any other
 * buffer runs LARGE.  (Forcing a kind is a test hook: td_set_step_kernel, td_diag.h.)
 * td_step_kernel returns the resolved kind, td_step_kernel_name the
 * kernel's name as rocprofv3 shows it ("td_step_kernel_small<10, 0, false>": L, mode,
 * multi-action scan). */
enum td_step_kernel_kind { TD_KERNEL_AUTO = 0, TD_KERNEL_LARGE = 1, TD_KERNEL_SMALL = 2, TD_KERNEL_SMALL2 = 3 };
int td_step_kernel(td_handle* h);
const char* td_step_kernel_name(td_handle* h);

/* Steps between launches of the layout refill kernel on the side streams (auto-reset;
 * default 64, 0 = none).  A pure performance knob: before every 15th step (and the first
 * step after a reset) the ring guard runs on the step stream and brings every board's
 * ring of 16 staged layouts to at least 15, so an episode end always finds its next
 * layout, whatever the interval.  The only board that misses one is a board whose draws
 * fail 65 times in a row (where the reference raises): it is flagged no_layout. */
int td_set_refill_interval(td_handle* h, int steps);

/* Kernel timing: every `every`-th td_step call from now on, up to max_launches of them,
 * binds a pair of timing events to its step kernel's own dispatch (hipExtLaunchKernel;
 * no marker packets); max_launches = 0 turns it off.  td_kernel_times waits for them
 * and writes each kernel's start-to-end duration in microseconds (the dispatch-packet
 * timestamps rocprofv3 reports); returns the count. */
int td_kernel_timing(td_handle* h, int max_launches, int every);
int td_kernel_times(td_handle* h, float* us, int cap);

/* Episodes finished by td_step since the last clear (SURVEY.md §8(b) td_episode_stats):
 * dev_out[0] = count, dev_out[1] = sum of their returns (f64, device memory, asynchronous
 * on `stream`; the sum is accumulated with atomics, so its rounding order is unspecified).
 * clear != 0 zeroes the accumulators after the copy.  The per-rank values are what the
 * multi-GPU driver gathers over RCCL. */
int td_episode_stats(td_handle* h, double* dev_out, int clear, void* stream);

/* Each board's last finished episode, the per-episode record a trainer collects
 * (train/main.py:155-166: total reward, length, win): dev_out = B records of 16 bytes,
 * { f64 return; i32 length; i32 win (1, 0, or -1 before the first finished episode) },
 * device memory, asynchronous on `stream`.  SURVEY.md §8(e): the per-board payload the
 * multi-GPU driver gathers over RCCL once per reporting interval. */
typedef struct td_episode_record {
  double ret;
  int32_t length;
  int32_t win;
} td_episode_record;
int td_episode_records(td_handle* h, td_episode_record* dev_out, void* stream);

/* The built-in opponent acting on its own between steps, as TDGymBasic's methods do when
 * called directly (TDGymBasic.py:81-108 random_enemy_lv0/1, :111-292 random_tower_lv0/1/2;
 * demo.py:78-79): side 0 = random_enemy_lv<level>, side 1 = random_tower_lv<level>, for the
 * boards in host_mask (NULL = all), on each board's opponent stream, with the reference's
 * cool-down check and update.  Synchronous. */
int td_opponent(td_handle* h, int side, int level, const uint8_t* host_mask, void* stream);

/* Layout records. */
int td_layout_words(int map_size);
int td_layout_from_roads(int map_size, int num_roads, const int32_t* cells, const int32_t* offsets, uint32_t* rec);
/* TDGymBasic.reset's draws on one numpy-legacy stream: num_roads = randint(1, 4),
 * then create_road_v2.  Returns 0 or a road-generation error code (>0). */
int td_layout_generate(uint32_t* np_state625, int map_size, int max_attempts, uint32_t* rec);

/* Board state, array-major for boards [b0, b0+count):
 *   hdr[count] (96 B each: see td_common.h TdHdr), en_lp f64[count][128], en_mg f64[count][128],
 *   en_inf u32[count][128] (cell | type<<12 | lv<<14 | slowdown<<16 | config epoch<<24),
 *   tw_cd f64[count][32], tw_inf u32[count][32] (cell | type<<12 | lv<<14 | build epoch<<16 |
 *   stats epoch<<24; imported entities take the current epoch), cells u32[count][L*L],
 *   opp_mt u32[count][626] (the opponent's CPython stream: 624 words, position, and the
 *   lazy-twist boundary -- words [w[625], 624) still hold the previous block).  Synchronous.
 *   The board's numpy layout stream is not part of the record (it belongs to the stream of
 *   layouts, staged ahead under auto-reset): save / restore it with td_get_np_state /
 *   td_set_np_state -- with random_agent=False it is also the built-in opponent's stream. */
size_t td_state_bytes(td_handle* h, int count);
int td_export_state(td_handle* h, int b0, int count, void* host_dst);
int td_import_state(td_handle* h, int b0, int count, const void* host_src);
int td_get_flags(td_handle* h, int32_t* host_flags);

/* Ring-guard waits for a board's refill claim that gave up after 1 s (a claim never given
 * back): the board is flagged TD_FLAG_CLAIM_TIMEOUT and its ring may run short.  Returns the
 * count since the last clear (clear != 0 zeroes it).  Synchronous. */
int td_guard_timeouts(td_handle* h, int clear);

/* Host-side RNG helpers (exposed for tests and for seeding from Python states). */
void td_py_seed(uint32_t* mt625, uint32_t seed);
void td_np_seed(uint32_t* mt625, uint32_t seed);
uint32_t td_mt_next(uint32_t* mt625);
int64_t td_py_randint(uint32_t* mt625, int64_t a, int64_t b);
int64_t td_np_randint(uint32_t* mt625, int64_t lo, int64_t hi);

#ifdef __cplusplus
}
#endif
#endif /* TDSTEP_H_ */
