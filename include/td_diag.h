/* td_diag.h -- test and measurement hooks of libtdstep.so.  NOT part of the drop-in
 * surface (include/tdstep.h): no reference function corresponds to any of
 * them.  The parity tests use them to hold every step kernel to the oracle and to provoke
 * the refill protocol's failure paths; a production binding should not bind them.
 * The symbols live in the same library so that the tests exercise the shipped build. */
#ifndef TD_DIAG_H_
#define TD_DIAG_H_

#include "tdstep.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Force the step kernel (enum td_step_kernel_kind; TD_KERNEL_AUTO = td_create's rule).  The
 * three kernels give the same results: the parity tests run each of them.  Fails (and
 * changes nothing) for a small kernel at an L without one. */
int td_set_step_kernel(td_handle* h, int kind);

/* The board each step-kernel block steps (no GPU needed): out[i] for blocks i in
 * [0, n_boards): the XCD-contiguous map of every step kernel (block i runs on XCD i % 8 and
 * steps the (i / 8)-th board of that XCD's contiguous range).  kind 0 and 1 give the same map.
 * xcd_map = 0: block i = board i. */
int td_board_map(int n_boards, int kind, int xcd_map, int32_t* out);

/* How the step kernels place boards and store the two observation lines a board shares
 * with its neighbours (18,000 B per board at 10x10 is not a multiple of 128):
 *   xcd_map 1 (default): the XCD-contiguous board map; 0: block i = board i;
 *   edge_wt 2 (default): plain write-back stores, merged in the XCD's L2; 1: write-through.
 * Results are the same bytes for every policy (tests/test_gpu_store_policy.py); the defaults
 * are the fastest measured.  Synchronises the device. */
int td_set_store_policy(td_handle* h, int xcd_map, int edge_wt);

/* UNSAFE on a production handle: hold (held = 1) or give back (0) board b's refill claim, as
 * a refill wave drawing its layouts holds it, outside the claim protocol.  A claim left held
 * keeps the board's ring short: its next episode end is flagged no_layout and
 * TD_FLAG_CLAIM_TIMEOUT (tests/test_gpu_claims.py).  Synchronises the device. */
int td_debug_set_claim(td_handle* h, int board, int held);

#ifdef __cplusplus
}
#endif
#endif /* TD_DIAG_H_ */
