"""bench.py's N > 1 path end to end on the one GPU of the box.

``bench.py --gpus 2`` starts its two ranks itself (torch.distributed.run as a child process,
before anything touches the GPU); with TD_BENCH_DIST_BACKEND=gloo and TD_BENCH_SAME_DEVICE=1
both ranks step their half of the global batch on cuda:0 -- a rehearsal of the driver's
multi-GPU command, never a measured configuration.  The JSON line must describe what ran:
two ranks, strong scaling over the global batch, each rank's own clock and closing barrier
(outside its timed region), ``value`` = all boards' steps / the slowest rank's clock, and at
least MIN_SAMPLES sampled kernel launches per rank.  Reference: the process-level
AsyncVectorEnv these ranks replace (/root/reference/train/main.py:329-347)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_line():
    sys.path.insert(0, ROOT)
    import bench
    env = dict(os.environ, TD_BENCH_DIST_BACKEND="gloo", TD_BENCH_SAME_DEVICE="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    K = 20
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--global-batch", "2048",
                        "--steps", str(K), "--warmup", "5", "--burnin", "300", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size_reported"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 2048 and d["config"]["boards_per_gpu"] == 1024
    per = d["per_rank_ms_per_step"]
    assert len(per) == 2 and len(d["closing_barrier_us"]) == 2 and len(d["per_rank_avg_kernel_us"]) == 2
    assert d["ms_per_step"] == pytest.approx(max(per), rel=1e-9)  # the slowest rank's clock
    assert d["value"] == pytest.approx(2 * 1024 * K / (max(per) * K / 1e3), rel=1e-6)
    assert d["roofline"]["kernel_samples_per_rank"] >= bench.MIN_SAMPLES
    assert d["board_flags_nonzero"] == 0
    assert "cpu_baseline" not in d  # the CPU baseline is rank 0's at N = 1 only
