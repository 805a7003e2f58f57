"""CPU checks of bench.py's contract pieces that need no GPU: defaults (C2, 16 timed iterations, 2
warmup, N = 1, strong packet-shard scaling), the roofline arithmetic and the host-thread count."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_defaults_are_the_c2_contract(bench):
    a = bench.parse([])
    assert (a.workload, a.steps, a.warmup, a.gpus) == ("c2", 16, 2, 1)
    assert (a.photons, a.width, a.height, a.max_depth, a.radius, a.alpha) == (1_000_000, 512, 512, 5, 0.01, 0.5)
    assert (a.scaling, a.shard_mode, a.pipeline, a.split, a.kernel) == ("strong", "packets", 1, 256, 0)
    c5 = bench.parse(["--workload", "c5"])
    assert (c5.steps, c5.photons, c5.width) == (10, 50_000_000, 1024)


def test_roofline_fraction_is_achieved_over_peak(bench):
    class WL:
        def segments_per_gather(self):
            return 1000

    a = bench.parse(["--split", "4"])
    st = {"n_segments": 640, "node_visits": 1000, "beam_evals": 3000, "queued_pairs": 500}
    r = bench.roofline(st, a, WL(), 2.0, None, None)
    items = (640 + 63) // 64 * 4
    # 112 B per queued pair: three SegRec planes, the record carries the power (128 B split layout)
    # a node visit reads one 128-B Node4 record (4-wide walk), a staged beam line 64 B
    alg = 128.0 * 1000 + 64.0 * 3000 + items * 64 * (40 + 12) + 112.0 * 500 + 640 * 12 * (4 + 1)
    # without the PMC passes: the HBM roofline of the requested bytes
    assert r["bound"] == "hbm" and r["hbm"]["requested_bytes_per_launch"] == alg
    a_split = bench.parse(["--split", "4", "--split-records", "1"])
    r_split = bench.roofline(st, a_split, WL(), 2.0, None, None)
    assert r_split["hbm"]["requested_bytes_per_launch"] == alg + 16.0 * 500
    assert r["achieved"] == pytest.approx(alg / 2e-3 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"]) and r["unit"] == "GB/s" and r["traffic"] is None
    # with them: VALU issue binds; frac = instructions / (256 CU x 4 SIMD / 2 x clocks), HBM kept aside
    issue = {"SQ_INSTS_VALU": 3.0e9, "clocks": 2.0e7, "valu_issue_frac": 3.0e9 / (512 * 2.0e7)}
    pmc = {"traffic_bytes_per_launch": 4.0e9, "kernel_ms": 10.0, "source": "test", "issue": issue}
    r = bench.roofline(st, a, WL(), 2.0, pmc, None)
    assert r["bound"] == "valu_issue" and r["traffic"] == 4.0e9
    assert r["achieved"] == pytest.approx(3.0e9 / 1e-2 / 1e9)
    assert r["peak"] == pytest.approx(512 * 2.0e7 / 1e-2 / 1e9)  # 2 GHz
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"]) == pytest.approx(issue["valu_issue_frac"])
    assert r["hbm"]["traffic_GBps"] == pytest.approx(4.0e9 / 1e-2 / 1e9)
    assert r["hbm"]["traffic_over_requested"] == pytest.approx(4.0e9 / alg)
    pmc["l2"] = {"TCC_HIT_sum": 3.0, "TCC_MISS_sum": 1.0, "hit_rate": 0.75}
    assert bench.roofline(st, a, WL(), 2.0, pmc, None)["l2"]["hit_rate"] == 0.75


def test_host_threads_positive(bench):
    n, note = bench.host_threads()
    assert n >= 1 and "affinity" in note


def test_late_step_is_the_smallest_radius_iteration(bench):
    """counters_last_iteration and the CPU sample go to the smallest radius the line times: C2's
    iteration 15 whenever 16 or more steps are timed (the driver's 20 steps re-time 0-3 after it)."""
    class WL:
        def iteration(self, k):
            return k % 16

    assert bench.late_step(WL(), 20) == 15
    assert bench.late_step(WL(), 16) == 15
    assert bench.late_step(WL(), 5) == 4

    class Synthetic:
        iteration = None

    assert bench.late_step(Synthetic(), 7) == 6
