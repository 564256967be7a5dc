"""The RCCL path of bench.py on the one GPU of the box (verdict r04, item 6).

A spawned process (a launcher's rank 0 of a world of one: RANK / WORLD_SIZE / MASTER_*
in its environment) initialises the process group with bench.init_dist -- the call
bench.py makes per rank, ``init_process_group("nccl", device_id=...)`` -- steps a batch
with auto-reset through libtdstep.so and runs bench.collect on the tensors bench.py
builds: the all_reduce MAX of the clocks (f64 on the device) and the gathers of the
device-accumulated episode statistics (f64 [2]) and of the per-board record payload
(uint8 [B, 16], td_episode_records).  A group of one still runs every collective
(gym_TD.shard), so this is RCCL moving device tensors.  The parent checks the results
against the engine's own values (reference: the per-episode stats train/main.py:143-166
collects)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [{pkg!r}, {root!r}]
import bench
from gym_TD import params as P
from gym_TD.engine import TDEngine
import copy
coll = bench.init_dist(0, "nccl")
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1 and coll.type == "cuda"
cfg = copy.deepcopy(P.config)
cfg.base_LP = 1  # short episodes: records and stats are filled within the run
B = 512
seeds = np.arange(B) + 3000
eng = TDEngine(10, B, "def", False, 1, device=0, np_seeds=seeds, py_seeds=seeds, autoreset=True, cfg=cfg)
eng.reset_all()
eng.episode_stats(clear=True)
g = torch.Generator(device="cuda").manual_seed(5)
for k in range(200):
    eng.step(def_act=torch.randint(0, 601, (B,), device="cuda", generator=g, dtype=torch.int64))
torch.cuda.synchronize()
stats = eng.episode_stats(clear=False)
recs = eng.episode_records()
(el, ak, ss), per_rank, got, clocks = bench.collect(1.5, 2.5e-4, 3.5e-4, stats, recs, coll, 4.5e-5)
want = [r.cpu() for r in recs]
out = dict(clocks=[el, ak, ss], rank_clocks=clocks.tolist(), per_rank=per_rank.cpu().numpy().tolist(), stats=stats.cpu().numpy().tolist(),
           recs_equal=all(torch.equal(a.cpu(), b) for a, b in zip(got, want)),
           per_rank_device=str(per_rank.device), finished=int(stats[0].item()),
           with_record=int((want[2] >= 0).sum()))
eng.close()
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_nccl_world_of_one_runs_bench_collectives():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    code = _CHILD.format(pkg=os.path.join(ROOT, "gym-td_amd"), root=ROOT)
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    import json
    r = json.loads(line[len("RESULT "):])
    assert r["clocks"] == [1.5, 2.5e-4, 3.5e-4]  # MAX over one rank: the values themselves
    assert r["rank_clocks"] == [[1.5, 2.5e-4, 3.5e-4, 4.5e-5]]  # each rank's own clocks, gathered
    assert r["per_rank"] == [r["stats"]]  # gathered to rank 0 over RCCL, bit for bit
    assert r["per_rank_device"].startswith("cuda")
    assert r["recs_equal"]  # the per-board 16-B payload, gathered over RCCL
    assert r["finished"] > 0 and r["with_record"] > 0
