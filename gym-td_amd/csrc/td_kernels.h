// td_kernels.h -- launch interface between the C-ABI (td_capi.hip) and the kernels (td_step.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "td_common.h"
#include "../../include/tdstep.h"

namespace td {

// opponent hot record: [0] position, [1] lazy-twist boundary, [2] pre-drawn count,
// [3] position of the first pre-drawn output, [4..4+HOT_CACHE) pre-drawn tempered outputs for
// positions [3] .. [3]+count-1.  The large kernel refills them (from its position on) only
// when fewer than HOT_REFILL remain unused; the small kernels every step.
constexpr int HOT_CACHE = 8, HOT_REFILL = 8;
constexpr int HOT_WORDS = 4 + HOT_CACHE;

struct StepArgs {
  int B, L, mode, multi, difficulty, autoreset;
  int opp_np;           // random_agent=False: the built-in opponents draw from np_mt (auto-reset off)
  int small;            // 0 td_step_kernel, 1 td_step_kernel_small, 2 td_step_kernel_small2
  int obs_wt;           // small kernel: observation stores write-through (the batch's obs fits the MALL)
  TdHdr* hdr;
  double* en_lp;
  double* en_mg;
  uint32_t* en_inf;
  double* tw_cd;
  uint32_t* tw_inf;
  uint32_t* cells;
  uint32_t* opp_mt;     // [B][626] CPython-random MT words of the built-in opponent ([624..625] unused)
  uint32_t* opp_hot;    // [B][HOT_WORDS] its position, lazy-twist boundary, count and next 8 draws
  uint32_t* np_mt;      // [B][625] numpy-legacy state of the layout stream (TDGymBasic.np_random)
  // Staged next-episode layouts: a ring of NSLOT records per board (slot_words
  // words each, 128-B aligned).  Layout number n of a board's stream lives in slot
  // n % NSLOT with word 0 = slot_tag(n) once it is complete; lay_tail counts the
  // layouts drawn (written by the refill / reset kernels only), lay_head the
  // layouts consumed (written by the step / reset kernels only).
  uint32_t* nxt;        // [B][NSLOT][slot_words]
  uint32_t* lay_head;   // [B]
  uint32_t* lay_tail;   // [B]
  uint32_t* lay_claim;  // [B] 1 while a refill wave draws the board's layouts
  int slot_words;
  int refill_grp;       // boards scanned per refill wave per pass (refill_group)
  int refill_waves;     // waves per refill launch (each walks ceil(B / refill_grp / refill_waves) groups)
  int refill_walks;     // walks per board per refill launch (a draw resumes in the next launch)
  uint8_t* scratch;     // [B][scratch_stride] a pending layout draw: RoadResume header + generator arrays
  size_t scratch_stride;
  uint8_t* reset_fail;  // [B] reset kernel: road generation failed (board left unchanged)
  uint32_t* guard_to;   // [1] ring-guard claim waits that gave up (td_guard_timeouts)
  const int32_t* ovr_idx;   // reset kernel, td_reset_layouts: [B] record index in ovr_rec, or -1
  const uint32_t* ovr_rec;  // caller-supplied layout records (layout_words(L) each)
  const TdDevCfg* cfg;   // the current constant block (= cfgs + epoch)
  const TdDevCfg* cfgs;  // [NCFG] one block per paramConfig epoch (entities keep their epoch's values)
  int epoch;
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
  uint8_t* cooldowns;
  double* ep_return;
  int32_t* ep_len;
  double* ep_stats;  // [2]: finished episodes, sum of their returns (accumulated by the step kernel)
  td_episode_record* last_ep;  // [B]: each board's last finished episode (written on done)
  const uint8_t* reset_mask;  // reset kernel only (nullptr = all boards)
  int xcd_map;   // block i steps board xcd_board(i, B) (else board i)
  int edge_wt;   // observation lines shared with a neighbouring board: 2 plain, 1 write-through (write_obs_lines)
};

constexpr int NXCD = 8;  // XCDs of an MI355X: block i runs on XCD i % 8

// The XCD-contiguous board map: block i (XCD i % 8, slot i / 8) steps board
// prefix(i % 8) + i / 8, so XCD x steps the contiguous range of boards after those of
// XCDs 0 .. x-1.  Neighbouring boards then share an L2: the lines of the small per-board
// arrays (header, hot record, reward, done, info) and the observation lines two boards
// share are written whole by one XCD instead of in pieces by several.
__host__ __device__ inline int xcd_board(int i, int B) {
  const int x = i & (NXCD - 1), q = B / NXCD, r = B % NXCD;
  return x * q + (x < r ? x : r) + i / NXCD;
}


// ev0 / ev1: optional timing events bound to the step kernel's dispatch (td_kernel_timing).
hipError_t launch_step(const StepArgs& a, hipStream_t s, bool reset, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// Small-batch step-kernel workgroups (one per board) resident at once on `cus` compute
// units, for the one-wave (td_step_kernel_small) or two-wave (td_step_kernel_small2) build.
int step_resident_boards(const StepArgs& a, int cus, int waves);
// random_agent=False with auto-reset: reset the boards the step just finished (a.done),
// drawing their layouts from the shared numpy stream now (same stream, after the step).
hipError_t launch_autoreset(const StepArgs& a, hipStream_t s);
// Config epochs referred to by live enemies / towers: bit e of used[NCFG / 32] (zeroed by the caller).
hipError_t launch_cfg_usage(const StepArgs& a, uint32_t* used, hipStream_t s);
// Draw staged layouts for every board whose ring has a free slot: a side-stream refill
// (guard = 0), or the ring guard on the step stream (guard = G: every ring below G
// layouts filled to G, draws run to the end; td_step.hip td_refill_kernel).
hipError_t launch_refill(const StepArgs& a, hipStream_t s, int guard = 0);
// The built-in opponent (side 0: random_enemy_lv<level>, 1: random_tower_lv<level>)
// on the boards in a.reset_mask (nullptr = all).
hipError_t launch_opponent(const StepArgs& a, int side, int level, hipStream_t s);

// Staged layouts per board: sixteen episodes of slack for the side refills, and the
// ring guard (td_refill_kernel) needs to run only every NSLOT - 1 steps.  (NSLOT = 4 with
// a guard every 3rd step: +4 % / +7-9 % per step at 8,192 / 4,096 boards, profiles/r03/s13.)
constexpr int NSLOT = 16;
__host__ __device__ inline uint32_t slot_tag(uint32_t n) { return 0x80000000u | (n & 0x7fffffffu); }
__host__ __device__ inline int slot_words(int L) { return (8 + L * L + 31) & ~31; }
// Boards scanned per refill wave when a refill launch has `waves` waves (at most 64:
// one ballot per wave).
__host__ __device__ inline int refill_group(int B, int waves) {
  const int g = (B + waves - 1) / waves;
  return g < 1 ? 1 : (g > 64 ? 64 : g);
}

constexpr int kRoadAttempts = 1000;  // bound of each create_road_v2 retry loop (reference: unbounded)
constexpr int kLayoutRetries = 64;   // auto-reset: failing draws skipped before giving up

constexpr uint64_t kTakeSpinTicks = 100000000ull;  // 1 s of the 100-MHz clock: longest wait for a refill wave

}  // namespace td
