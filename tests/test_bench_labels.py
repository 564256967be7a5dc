"""bench.py's partition of the global batch over ranks and the labels of its JSON line
(BASELINE.json metric / configs[3]: 65,536 boards over the node, 65,536 / N per GPU)."""
import pytest

import bench


@pytest.mark.parametrize("world,per_gpu", [(1, 65536), (2, 32768), (4, 16384), (8, 8192)])
def test_strong_scaling_default_is_the_metric_batch(world, per_gpu):
    B, g, scaling = bench.partition("def-small", world)
    assert (B, g, scaling) == (per_gpu, 65536, "strong")
    assert bench.metric_label("def-small", g, scaling) == bench.BASELINE_METRIC


def test_weak_scaling_is_labelled():
    B, g, scaling = bench.partition("def-small", 8, boards_per_gpu=65536)
    assert (B, g, scaling) == (65536, 524288, "weak")
    lab = bench.metric_label("def-small", g, scaling)
    assert lab != bench.BASELINE_METRIC and "batch=524288" in lab and "weak" in lab


def test_other_batches_are_not_labelled_as_the_metric():
    B, g, scaling = bench.partition("def-small", 1, global_batch=8192)
    assert (B, g, scaling) == (8192, 8192, "strong")
    assert "batch=8192" in bench.metric_label("def-small", g, scaling)
    B, g, _ = bench.partition("def-large", 8)
    assert (B, g) == (16384, 131072)  # BASELINE configs[4]: 131,072 x 30x30 over 8 GPUs
    with pytest.raises(ValueError):
        bench.partition("def-small", 3)


def test_traffic_only_for_the_measured_build(tmp_path):
    # a record measured on other kernel sources, at another batch, of another kernel or with
    # the observation allocated another way is never quoted
    import json
    k = "td_step_kernel<10, 0, false>"
    assert bench.measured_traffic("def-small", 12345, k, "plain") == (None, None)
    assert len(bench.kernel_source_hash()) == 16
    rec = {"hbm_bytes_per_launch": 1.0e9, "read": 1.0e8, "write": 9.0e8, "round": "rX", "kernel": k,
           "kernel_src": bench.kernel_source_hash(), "obs_alloc": "contiguous"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"def-small_B65536": rec}))
    assert bench.measured_traffic("def-small", 65536, k, "contiguous", path=str(p))[0] == 1.0e9
    assert bench.measured_traffic("def-small", 65536, k, "plain", path=str(p)) == (None, None)
    assert bench.measured_traffic("def-small", 65536, "td_step_kernel_small<10, 0, false>", "contiguous",
                                  path=str(p)) == (None, None)
    p.write_text(json.dumps({"def-small_B65536": dict(rec, kernel_src="0" * 16)}))
    assert bench.measured_traffic("def-small", 65536, k, "contiguous", path=str(p)) == (None, None)


def test_world_must_match_gpus():
    # under a launcher, WORLD_SIZE must equal --gpus; without one, --gpus N > 1 launches N ranks
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(8, {}) is None
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == 8
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})


def test_mismatched_world_exits_nonzero():
    """bench.py under a launcher that started another rank count than --gpus says exits
    non-zero before it touches a GPU."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "1"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr


def test_gpus_n_starts_n_ranks(monkeypatch):
    """--gpus N > 1 with no launcher: torch.distributed.run with N processes on 127.0.0.1,
    started as a child (never an exec of this process), its status returned."""
    import subprocess
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 3
    monkeypatch.setattr(subprocess, "call", fake_call)
    assert bench.launch_ranks(4, ["--gpus", "4", "--steps", "5"]) == 3
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4" and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [bench.os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "5"][-4:]


def test_sampling_stride_follows_the_step_time():
    # the kernel is sampled inside the timed region; the stride keeps the events' cost
    # (EVENT_COST_US per sampled launch) under EVENT_PERTURB of the step, with >= 2 launches
    # between samples, but never fewer than MIN_SAMPLES samples per rank
    assert bench.event_every(20, 204.0) == 2  # the driver's line: 10 samples
    assert bench.event_every(20, 33.0) == 5  # 8,192 boards (the N = 8 share): 4 samples per rank
    assert bench.event_every(2000, 33.0) == 10
    assert bench.event_every(2000, 21.0) == 15
    assert bench.event_every(1, 210.0) == 1  # one timed step: one sample
    assert bench.event_every(20, None) == 5  # --warmup 0: EVENT_EVERY within the cap
    assert bench.event_every(200, None) == bench.EVENT_EVERY
    assert bench.event_every(20, 210.0, override=1) == 1
    for steps, us in ((20, 210.0), (20, 32.4), (300, 497.0), (2000, 21.0), (200, 300.0), (7, 18.0)):
        k = bench.event_every(steps, us)
        cap = max(1, steps // bench.MIN_SAMPLES)
        assert bench.EVENT_COST_US / (k * us) <= bench.EVENT_PERTURB or k == cap
        assert (steps + k - 1) // k >= min(steps, bench.MIN_SAMPLES)


class _Clock(object):
    """A fake clock that the stubbed steps / barrier advance by known amounts."""

    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_timed_region_excludes_the_closing_barrier():
    """The rank's elapsed time ends at its own synchronize after its steps: a closing barrier
    of known delay (a rank that waits for a slower one) is not in it, and is reported on its
    own; the opening barrier precedes the clock."""
    clk, calls = _Clock(), []

    def run():
        calls.append("run")
        clk.t += 0.004  # the K steps: 4 ms

    def sync():
        calls.append("sync")

    def barrier():
        calls.append("barrier")
        clk.t += 0.0025  # 2.5 ms waiting for the other ranks

    elapsed, barrier_s = bench.timed_region(run, sync, barrier, clock=clk)
    assert elapsed == pytest.approx(0.004, abs=1e-12)
    assert barrier_s == pytest.approx(0.0025, abs=1e-12)
    assert calls == ["sync", "barrier", "sync", "run", "sync", "barrier", "sync"]
    # world of one: no barrier at all, the same clock
    calls.clear()
    elapsed, barrier_s = bench.timed_region(run, sync, None, clock=clk)
    assert (round(elapsed, 12), barrier_s) == (0.004, 0.0)
    assert calls == ["sync", "sync", "run", "sync"]


def test_timed_region_real_clock_with_a_slow_barrier():
    """The same with the real clock and a sleeping barrier (20 ms) around 5-ms steps."""
    import time
    elapsed, barrier_s = bench.timed_region(lambda: time.sleep(0.005), lambda: None, lambda: time.sleep(0.02))
    assert 0.005 <= elapsed < 0.019 and barrier_s >= 0.02


def test_kernel_longer_than_the_step_withholds_the_fraction():
    assert bench.kernel_vs_step(225.9, 221.8)[0] is True
    assert "exceeds the timed region" in bench.kernel_vs_step(225.9, 221.8)[1]
    assert bench.kernel_vs_step(215.0, 221.8) == (False, None)
    assert bench.kernel_vs_step(float("nan"), 221.8) == (False, None)


def test_cpu_baseline_uses_every_core_of_the_affinity_mask():
    import os
    assert bench.host_cores() == len(os.sched_getaffinity(0))
    q = bench.cpu_quota()
    assert q is None or q > 0
    threads, affinity, quota = bench.baseline_threads()
    assert affinity == len(os.sched_getaffinity(0)) and quota == q
    assert threads == (affinity if not q else max(1, min(affinity, int(q))))


def test_baseline_note_states_cores_and_projection():
    n = bench.baseline_note(8.0e6, 16, 256, 16.0)
    assert n["affinity_cores"] == 256 and n["cpu_quota_cores"] == 16.0
    assert n["value_per_core"] == 0.5e6
    assert n["all_affinity_cores_projection"]["value"] == 128.0e6
    assert "not measured" in n["all_affinity_cores_projection"]["note"]
