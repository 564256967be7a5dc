// td_common.h -- device-side board record layout and the device constant block.
//
// Boards live in HBM as board-major records split into per-field arrays, one
// wavefront per board reads its own slice with coalesced loads:
//   hdr     TdHdr            [B]
//   en_lp   f64              [B][ECAP]   enemy LP            (Enemy.LP, TDElements.py:6)
//   en_mg   f64              [B][ECAP]   enemy margin        (Enemy.margin, :11)
//   en_inf  u32              [B][ECAP]   cell | type<<12 | lv<<14 | slowdown<<16 | cfg epoch<<24
//   tw_cd   f64              [B][TCAP]   tower cool-down     (Tower.cd, :54)
//   tw_inf  u32              [B][TCAP]   cell | type<<12 | lv<<14 | build epoch<<16 | stats epoch<<24
//   cells   u32              [B][L*L]    cell words (td_layout.h bit layout)
//   opp_mt  u32              [B][626]    CPython-random MT19937 of the built-in opponent (lazy twist)
//   nxt     u32              [B][8+L*L]  staged layout for the board's next episode
// Enemy / tower lists keep the reference's list order (index order).
#pragma once
#include <stdint.h>

namespace td {

constexpr int ECAP = 128;  // enemies alive per board (<=121 reachable with default config)
constexpr int TCAP = 32;   // towers per board (<=25 reachable with default config)
constexpr int NCH = 45;    // observation channels (TDBoard.py:146-154, default type/level counts)
// Opponent stream words per board: MT19937 state [0..623], position [624], and the
// lazy-twist boundary [625] (words [tw, 624) still hold the previous block).
constexpr int OPP_WORDS = 626;

enum Mode : int { MODE_DEF = 0, MODE_ATK = 1, MODE_2P = 2 };

// per-board error bits (TdHdr.flags)
enum : int {
  FLAG_EN_OVERFLOW = 1 << 0,
  FLAG_TW_OVERFLOW = 1 << 1,
  FLAG_BAD_ACTION = 1 << 2,
  FLAG_NO_LAYOUT = 1 << 3,
  FLAG_BAD_MOVE = 1 << 4,
  FLAG_CLAIM_TIMEOUT = 1 << 5,  // a wait for the board's refill claim gave up (1 s): its ring may run short
};

struct alignas(16) TdHdr {  // 96 bytes
  double cost_def, cost_atk;   // TDBoard.py:68-69
  double ep_return;            // running sum of this episode's rewards
  int32_t steps, base_LP;      // :76, :71
  int32_t atk_cd, def_cd;      // TDGymBasic.py:52-53
  int32_t n_en, n_tw;
  int32_t num_roads, end_cell;
  int32_t start_cell[3], maxdist;
  int32_t flags, episodes;
  double max_cost;             // captured at reset (TDBoard.py:70, passed by TDGymBasic.reset :43-53)
  int32_t max_base_LP;         // :72
  int32_t format;              // kHdrFormat on every board a kernel has reset (td_import_state checks it)
};
constexpr int32_t kHdrFormat = 0x54440002;  // "TD", header format 2 (max_cost / max_base_LP captured)
static_assert(sizeof(TdHdr) == 96, "TdHdr layout");

// Device constant block (built on the host from paramConfig-style values).  The device
// keeps a table of them (one per paramConfig epoch, td_capi.hip): enemies and towers
// carry the epoch of the block they were created / upgraded under, as the reference's
// Enemy / Tower objects keep the values they captured then (TDElements.py:4-43, 45-63,
// 134-170).
constexpr int NCFG = 256;  // epochs in the table (8-bit tags)
struct alignas(16) TdDevCfg {
  double e_lp[4][2], e_speed[4][2], e_def[4][2], e_cost[4][2];
  double t_atk[4][2], t_rge[4][2], t_dmg[4][2];
  double t_price[4][2];  // tower_cost: price to build (lv0) / upgrade to lv
  double t_intv[4][2];   // effective Tower.intv at lv (upgrade_tower arg swap, TDElements.py:163-169)
  double t_addcost[4][2];  // tower_attack_interval: what an upgrade adds to Tower.cost (the same swap)
  double destruct_return, frozen_ratio, max_cost, reward_kill, penalty_leak, reward_time;
  double atk_init_rate, atk_final_rate, def_rate, enemy_upgrade_at;
  double def_init_cost, atk_init_cost;
  int32_t frozen_time, base_LP, tower_distance, atk_interval;
  int32_t def_interval, max_episode_steps, max_cluster_length, max_tower_lv;
};

__host__ __device__ inline int cw_dist(uint32_t w) { return (int)((w >> 16) & 0xffu); }
__host__ __device__ inline int cw_dir(uint32_t w) { return (int)((w >> 8) & 3u); }
__host__ __device__ inline int cw_block(uint32_t w) { return (int)(w >> 24); }

__host__ __device__ inline uint32_t en_pack(int cell, int type, int lv, int slow, int ep) {
  return (uint32_t)cell | ((uint32_t)type << 12) | ((uint32_t)lv << 14) | ((uint32_t)slow << 16) | ((uint32_t)ep << 24);
}
__host__ __device__ inline int en_cell(uint32_t u) { return (int)(u & 0xfffu); }
__host__ __device__ inline int en_type(uint32_t u) { return (int)((u >> 12) & 3u); }
__host__ __device__ inline int en_lv(uint32_t u) { return (int)((u >> 14) & 1u); }
__host__ __device__ inline int en_slow(uint32_t u) { return (int)((u >> 16) & 0xffu); }  // frozen_time <= 255
__host__ __device__ inline int en_ep(uint32_t u) { return (int)(u >> 24); }
// ec: epoch the tower was built under (its base Tower.cost); eu: epoch of its current
// stats (the build, or the last upgrade: atk, rge, dmgrge, intv and the added cost)
__host__ __device__ inline uint32_t tw_pack(int cell, int type, int lv, int ec, int eu) {
  return (uint32_t)cell | ((uint32_t)type << 12) | ((uint32_t)lv << 14) | ((uint32_t)ec << 16) | ((uint32_t)eu << 24);
}
__host__ __device__ inline int tw_ec(uint32_t u) { return (int)((u >> 16) & 0xffu); }
__host__ __device__ inline int tw_eu(uint32_t u) { return (int)(u >> 24); }

}  // namespace td
