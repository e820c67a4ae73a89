"""The committed PMC summaries that bench.py prices its roofline with (profiles/pmc_traffic.json,
profiles/pmc_issue.json) are present for the headline workload, come from exactly one profiled pass,
and give fractions <= 1 at the measured pass time (profiles/r02/bench_teapot.json)."""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD = "teapot.scene 1920x1080 2048spp 16 bounces sort=on"


def _bench():
    # imported on use: bench.py sets GPU_MAX_HW_QUEUES at import, which a GPU run's collection of this
    # module must not do
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    return importlib.import_module("bench")


def _bench_line():
    with open(os.path.join(REPO, "profiles", "r02", "bench_teapot.json")) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_traffic_profile_is_one_pass():
    d = _bench().load_pmc(WORKLOAD)
    assert d is not None and d["passes_profiled"] == 1
    assert d["trace_launches"] == 16                      # one pass of 16 bounces
    assert 0 < d["trace_bytes_per_launch"] < d["pass_bytes"]


def test_issue_profile_and_valu_fraction():
    bench = _bench()
    d = bench.load_issue(WORKLOAD)
    assert d is not None and d["passes_profiled"] == 1
    v_all, v_trace = d["per_pass"]["SQ_INSTS_VALU"], d["trace_per_pass"]["SQ_INSTS_VALU"]
    assert 0 < v_trace < v_all
    ms_pass = _bench_line()["ms_per_step"]
    frac = v_all / (ms_pass / 1e3) / 1e9 / bench.VALU_PEAK_GWIS
    assert 0.0 < frac <= 1.0
    assert bench.VALU_PEAK_GWIS == 1228.8


def test_bench_line_fractions_at_most_one():
    roof = _bench_line()["roofline"]
    assert 0 < roof["frac"] <= 1 and 0 < roof["traffic_frac"] <= 1
    assert 0 < roof["l2"]["frac"] <= 1 and 0 < roof["frame"]["frac"] <= 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
