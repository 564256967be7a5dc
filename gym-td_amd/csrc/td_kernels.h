// td_kernels.h -- launch interface between the C-ABI (td_capi.hip) and the kernels (td_step.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "td_common.h"

namespace td {

struct StepArgs {
  int B, L, mode, multi, difficulty, autoreset;
  TdHdr* hdr;
  double* en_lp;
  double* en_mg;
  uint32_t* en_inf;
  double* tw_cd;
  uint32_t* tw_inf;
  uint32_t* cells;
  uint32_t* opp_mt;     // [B][625] CPython-random state of the built-in opponent
  uint32_t* nxt;        // [B][8 + L*L] staged next-episode layout (word 0 = magic while unconsumed)
  uint32_t* consumed;   // [B] layouts consumed so far (host refills when it catches up)
  const TdDevCfg* cfg;
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
  const uint8_t* reset_mask;  // reset kernel only (nullptr = all boards)
};

hipError_t launch_step(const StepArgs& a, hipStream_t s, bool reset);
hipError_t launch_stage_layouts(uint32_t* nxt, const uint32_t* recs, const int32_t* boards, int n, int words,
                                hipStream_t s);

}  // namespace td
