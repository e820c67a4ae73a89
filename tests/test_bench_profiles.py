"""The committed PMC summaries that bench.py prices its roofline with (profiles/pmc_traffic.json,
profiles/pmc_issue.json) are present for the headline workload, come from exactly one profiled pass,
and give fractions <= 1 at the measured pass time (the closing bench lines measured with them: profiles/r06/final)."""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD = "teapot.scene 1920x1080 2048spp 16 bounces sort=on"
FINAL = os.path.join(REPO, "profiles", "r06", "final")   # the closing measurement of this round


def _bench():
    # imported on use: bench.py sets GPU_MAX_HW_QUEUES at import, which a GPU run's collection of this
    # module must not do
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    return importlib.import_module("bench")


def _bench_line():
    with open(os.path.join(FINAL, "bench_teapot.json")) as f:
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
    t = roof["timed"]                                   # round 5: the trace kernel inside the timed step
    assert 0 < t["ms_per_step"] <= t["step_ms"] and 0 < t["frac"] <= 1 and 0 < t["measured_frac"] <= 1
    assert 0 < t["valu_frac"] <= 1


def test_closing_headline_is_the_timed_step():
    """Round 6 (verdict r05 item 3): the closing lines' headline achieved / frac are the timed-step figures: frac x peak
    x the kernel's time per step recomputes the step's algorithmic trace bytes, and that time fits in ms_per_step.  The
    exclusive-launch figures sit under `exclusive`, and the PMC record is the measured revision's."""
    rev = open(os.path.join(FINAL, "REVISION")).read().strip()
    for name in ("bench_teapot.json", "bench_teapot_steps20.json"):
        line = _final_lines()[name]
        roof = line["roofline"]
        assert roof["regime"] == "timed step" and roof["frac"] == roof["timed"]["frac"]
        assert 0 < roof["kernel_ms_per_step"] <= line["ms_per_step"]
        rebuilt = roof["frac"] * roof["peak"] * 1e9 * roof["kernel_ms_per_step"] / 1e3
        assert abs(rebuilt - roof["bytes_per_step"]) / roof["bytes_per_step"] < 3e-3, name
        assert roof["exclusive"]["ms_per_launch"] * roof["exclusive"]["launches"] > line["ms_per_step"]   # another regime
    assert _bench().load_pmc(WORKLOAD)["run"].startswith("rev " + rev)


def test_roofline_restated_on_exclusive_launches():
    """bench.roofline: the exclusive-launch figures (round 3) are a labelled secondary field -- achieved =
    algorithmic bytes (scene once per XCD) / the exclusive launch duration; traffic_frac = the PMC bytes over
    the same duration; the shared-chip spans only in `shared`."""
    bench = _bench()
    counted = {"live_segments": 79_000_000, "generated_rays": 41_472_000, "nodes_popped": 800_000_000,
               "internal_visits": 680_000_000, "triangle_tests": 300_000_000}
    excl = {"launches": 16, "ms_per_launch": 0.7, "trace_ms": 11.2, "kernel_ms": 15.0, "counted": counted}
    scene_bytes = 32 * 252_099 + 48 * 126_050
    roof = bench.roofline(excl, counted, 16, 2.3, scene_bytes, 0, WORKLOAD, 0.14, 20)
    ex = roof["exclusive"]
    comp = (24 * (79_000_000 - 41_472_000) + 8 * 79_000_000 + 16 * 8 * scene_bytes) / 16
    assert ex["bytes_per_launch"] == int(comp)
    assert abs(ex["achieved"] - comp / 0.7e-3 / 1e9) < 0.1
    assert abs(ex["frac"] - ex["achieved"] / 8000.0) < 1e-4
    assert roof["shared"]["ms_per_launch"] == 2.3 and ex["ms_per_launch"] == 0.7
    pmc = bench.load_pmc(WORKLOAD)
    if pmc:
        assert abs(ex["traffic_frac"] - pmc["trace_bytes_per_launch"] / 0.7e-3 / 1e9 / 8000.0) < 1e-3
    assert roof["logical_per_step"]["achieved"] > 0


def test_roofline_headline_fits_the_step():
    """Round 6 (verdict r05 item 3): the headline achieved / frac / traffic / traffic_frac are the timed-step
    figures: frac x peak x the kernel's time per step = the step's algorithmic trace bytes, that time is at most
    ms_per_step, and traffic_frac prices the measured bytes of one pass over the same time."""
    bench = _bench()
    counted = {"live_segments": 20 * 79_000_000, "generated_rays": 20 * 41_472_000, "nodes_popped": 1,
               "internal_visits": 1, "triangle_tests": 1}
    excl = {"launches": 16, "ms_per_launch": 0.7, "trace_ms": 11.2, "kernel_ms": 15.0, "counted": counted}
    scene_bytes = 32 * 252_099 + 48 * 126_050
    elapsed, steps = 0.118, 20
    roof = bench.roofline(excl, counted, 20 * 16, 2.3, scene_bytes, 0, WORKLOAD, elapsed, steps)
    t = roof["timed"]
    assert roof["regime"] == "timed step" and roof["frac"] == t["frac"] and roof["achieved"] == t["achieved"]
    step_ms = elapsed / steps * 1e3
    assert 0 < roof["kernel_ms_per_step"] <= step_ms
    alg_step = bench.compulsory_trace_bytes(counted, scene_bytes, 20 * 16, per_xcd=True) / steps
    assert roof["bytes_per_step"] == int(alg_step)
    assert abs(roof["frac"] * roof["peak"] * 1e9 * roof["kernel_ms_per_step"] / 1e3 - alg_step) / alg_step < 2e-3
    # at most the step's algorithmic bytes at the HBM peak over the whole step
    assert roof["frac"] * roof["peak"] * 1e9 * roof["kernel_ms_per_step"] / 1e3 <= alg_step * 1.002
    # the timed regime's own PMC records (the driver's 20 concurrent passes) price it where they exist
    pmc = bench.load_pmc(WORKLOAD + bench.TIMED_PMC) or bench.load_pmc(WORKLOAD)
    assert roof["traffic"] == t["measured_bytes_per_step"]
    assert abs(roof["traffic_frac"] - pmc["trace_bytes_per_launch"] * pmc["trace_launches"] / pmc["passes_profiled"] /
               (roof["kernel_ms_per_step"] / 1e3) / 1e9 / 8000.0) < 2e-3
    iss = bench.load_issue(WORKLOAD + bench.TIMED_PMC)
    if iss:
        assert t["regime"] == "the driver's 20 concurrent passes" and iss["passes_profiled"] == 20
        assert t["wave_cycle_share"] == round(iss["trace_per_pass"]["SQ_WAVE_CYCLES"] / iss["per_pass"]["SQ_WAVE_CYCLES"], 4)
        assert 0 < t["wave_cycle_share"] < t["one_pass"]["wave_cycle_share"] < 1


def _final_lines():
    d = FINAL
    out = {}
    for f in sorted(os.listdir(d)):
        if f.startswith("bench_") and f.endswith(".json"):
            with open(os.path.join(d, f)) as fh:
                out[f] = json.loads(fh.read().strip().splitlines()[-1])
    return out


def test_closing_lines_every_config_bit_exact():
    """The closing measurement (FINAL): a line per BASELINE config, each with its pass-0
    framebuffer hash equal to the oracle's and its fractions at most one."""
    lines = _final_lines()
    for name in ("bench_cornell.json", "bench_cornell_plus.json", "bench_spheres.json", "bench_teapot.json",
                 "bench_teapotnosort.json", "bench_lamp.json", "bench_lampnosort.json", "bench_teapot_steps20.json"):
        assert name in lines, name
        d = lines[name]
        assert d["bit_exact_vs_oracle"] is True, name
        assert d["value"] > 0 and d["ms_per_step"] > 0
        roof = d.get("roofline")
        if roof and roof.get("frac") is not None:   # traced configs (spheres has no trace kernel)
            assert 0 < roof["frac"] <= 1, name
            if roof.get("traffic_frac") is not None:   # configs with a committed PMC record (not cornell)
                assert 0 < roof["traffic_frac"] <= 1, name
                assert 0 < roof["frame"]["frac"] <= 1 and 0 < roof["valu"]["frac"] <= 1, name
    assert lines["bench_teapot_steps20.json"]["steps"] == 20 and lines["bench_teapot_steps20.json"]["warmup"] == 5


def test_closing_exclusive_launch_agrees_with_the_profiler():
    """The bench's exclusive trace launch duration (device wall clock, one atomic per workgroup) and the
    profiler's average dispatch duration of the same launches agree within 10 %."""
    roof = _final_lines()["bench_teapot.json"]["roofline"]
    ex = roof.get("exclusive", roof)          # round 6: the exclusive figures moved under `exclusive`
    a, b = ex["ms_per_launch"], ex["pmc_run"]["ms_per_launch"]
    assert abs(a - b) / b < 0.10, (a, b)


def test_results_table_from_committed_files():
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "results_table.py"),
                          FINAL], capture_output=True, text=True, check=True).stdout
    rows = [r for r in out.splitlines() if r.startswith("| ") and " | 1 | " in r]
    assert len(rows) == 7, out                      # 5 configs, teapot and lamp in both sort modes
    assert all("| True |" in r for r in rows)


def test_roofline_per_launch_table_recomputes():
    """Round 4: the per-launch table (rt_renderer_launch_profile) of the closing line: every launch's fraction
    follows from its own bytes and duration, heavy + tail cover the launches, and the measured bytes come from the
    committed PMC record of the same revision."""
    bench = _bench()
    roof = _bench_line()["roofline"]
    rows = roof["per_launch"]
    assert len(rows) == 16 and [r["bounce"] for r in rows] == list(range(16))
    for r in rows:
        assert abs(r["frac"] - r["algorithmic_bytes"] / (r["ms"] / 1e3) / 1e9 / bench.HBM_PEAK_GBS) < 2e-4
    assert roof["heavy"]["launches"] + roof["tail"]["launches"] == 16
    assert roof["heavy"]["live"] + roof["tail"]["live"] == sum(r["live"] for r in rows)
    pmc = bench.load_pmc(WORKLOAD)
    assert [r["measured_bytes"] for r in rows] == pmc["trace_bytes_by_launch"]
    assert pmc["run"].startswith("rev ")


def test_timed_regime_fits_the_step():
    """Round 5 (roofline.timed): the trace kernel's time per step is its wave-residency share of a pass times
    ms_per_step, so it never exceeds the step, and every fraction recomputes from the bytes / instructions
    per pass over that time."""
    bench = _bench()
    counted = {"live_segments": 20 * 79_000_000, "generated_rays": 20 * 41_472_000}
    scene_bytes = 32 * 252_099 + 48 * 126_050
    iss = {"per_pass": {"SQ_WAVE_CYCLES": 4.0e9, "SQ_INSTS_VALU": 3.6e9},
           "trace_per_pass": {"SQ_WAVE_CYCLES": 3.0e9, "SQ_INSTS_VALU": 3.0e9}, "run": "synthetic"}
    pmc = {"trace_bytes_per_launch": 250e6, "trace_launches": 16, "passes_profiled": 1}
    t = bench.timed_regime(iss, pmc, counted, 20 * 16, scene_bytes, 0.128, 20)
    assert t["wave_cycle_share"] == 0.75 and t["ms_per_step"] <= t["step_ms"]
    secs = 0.75 * 0.128 / 20
    alg = bench.compulsory_trace_bytes(counted, scene_bytes, 20 * 16, per_xcd=True) / 20
    assert abs(t["frac"] - alg / secs / 1e9 / bench.HBM_PEAK_GBS) < 1e-4
    assert abs(t["measured_frac"] - 16 * 250e6 / secs / 1e9 / bench.HBM_PEAK_GBS) < 1e-4
    assert abs(t["valu_frac"] - 3.0e9 / secs / 1e9 / bench.VALU_PEAK_GWIS) < 1e-4
    assert bench.timed_regime({"per_pass": {}, "trace_per_pass": {}}, pmc, counted, 320, scene_bytes, 0.128, 20) is None
