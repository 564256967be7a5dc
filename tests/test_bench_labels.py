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


def test_traffic_only_for_the_measured_build(tmp_path, monkeypatch):
    # a record measured on other kernel sources (or at another batch) is never quoted
    assert bench.measured_traffic("def-small", 12345) == (None, None)
    assert len(bench.kernel_source_hash()) == 16


@pytest.mark.parametrize("world,kernel", [(1, "td_step_kernel<10, DEF>"), (2, "td_step_kernel<10, DEF>"),
                                          (4, "td_step_kernel<10, DEF>"), (8, "td_step_kernel_small<10, DEF>")])
def test_roofline_names_the_kernel_that_runs(world, kernel, monkeypatch):
    # td_create's rule on a 256-CU MI355X: one round of waves (8 per SIMD) -> small kernel,
    # half a round -> two waves per board
    monkeypatch.delenv("TD_SMALL", raising=False)
    B, _, _ = bench.partition("def-small", world)
    assert bench.step_kernel_name(10, "def", B, 256) == kernel
    assert bench.step_kernel_name(10, "def", 4096, 256) == "td_step_kernel_small2<10, DEF>"
    assert bench.step_kernel_name(20, "2p", 16384, 256) == "td_step_kernel<20, 2P>"
