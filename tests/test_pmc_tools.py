"""The PMC summary tools that feed bench.py's roofline (tools/pmc_summary.py, tools/stall_summary.py) on a
synthetic rocprofv3 counter CSV: per-launch trace bytes are the trace dispatches' sum divided by their count,
per-pass figures are divided by the passes profiled (fill_live_kernel dispatches) — round 1's summary divided
two profiled passes by one pass's bounces — and 128-B read requests are priced at 128 B."""
import csv
import json
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = "pytest_synthetic"
HEADER = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size", "Kernel_Id",
          "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count",
          "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
TRACE = "void (anonymous namespace)::trace_kernel<true, false, 0>(DevScene, PassArgs)"
FILL = "(anonymous namespace)::fill_live_kernel(unsigned int*, unsigned int, int)"
SHADE = "void (anonymous namespace)::shade_kernel<true, false, 0, false, false>(DevScene)"

# two profiled passes: per pass one fill_live, two trace launches and one shade launch
DISPATCHES = [FILL, TRACE, SHADE, TRACE, FILL, TRACE, SHADE, TRACE]


def _write(group_dir, counters):
    os.makedirs(group_dir, exist_ok=True)
    with open(os.path.join(group_dir, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HEADER)
        for i, name in enumerate(DISPATCHES, 1):
            for cname, value in counters(name, i).items():
                w.writerow([i, i, "Agent 2", 1, 1, 1, 256, 1, name, 256, 0, 0, 8, 0, 16, cname, value,
                            1000 * i, 1000 * i + 500])


@pytest.fixture()
def synthetic():
    out = os.path.join(REPO, "gpurun_out")
    dirs = [os.path.join(out, "pmc_%s_%d" % (TAG, k)) for k in (1, 2, 3)]
    # traffic: each trace launch reads 10 requests of 128 B and 4 of 64 B, writes 3 of 64 B + 1 of 32 B;
    # every other kernel 1 x 128 B read
    _write(dirs[0], lambda n, i: {"TCC_EA0_RDREQ_sum": 14 if n == TRACE else 1,
                                  "TCC_EA0_RDREQ_128B_sum": 10 if n == TRACE else 1,
                                  "TCC_EA0_RDREQ_64B_sum": 4 if n == TRACE else 0,
                                  "TCC_EA0_RDREQ_32B_sum": 0})
    _write(dirs[1], lambda n, i: {"TCC_EA0_WRREQ_sum": 4 if n == TRACE else 0,
                                  "TCC_EA0_WRREQ_64B_sum": 3 if n == TRACE else 0})
    # instruction counts: 100 VALU per trace launch, 10 per other dispatch
    _write(dirs[2], lambda n, i: {"SQ_INSTS_VALU": 100 if n == TRACE else 10, "SQ_INSTS_SALU": 1,
                                  "SQ_WAVE_CYCLES": 1000, "SQ_WAVES": 4})
    yield
    for d in dirs:
        shutil.rmtree(d, ignore_errors=True)


def _run(tool, args):
    return subprocess.run([sys.executable, os.path.join(REPO, "tools", tool)] + args, cwd=os.path.join(REPO, "tools"),
                          capture_output=True, text=True, check=True)


def test_traffic_summary_per_launch_and_per_pass(synthetic, tmp_path):
    path = str(tmp_path / "traffic.json")
    _run("pmc_summary.py", [TAG, "--json", path, "--workload", "w", "--run", "synthetic"])
    rec = json.load(open(path))["w"]
    assert rec["passes_profiled"] == 2 and rec["trace_launches"] == 4
    per_trace_read = 10 * 128 + 4 * 64
    per_trace_write = 3 * 64 + 1 * 32
    assert rec["trace_bytes_per_launch"] == per_trace_read + per_trace_write
    # per pass: 2 trace launches + fill_live + shade (one 128-B read each)
    assert rec["pass_bytes"] == 2 * (per_trace_read + per_trace_write) + 2 * 128


def test_issue_summary_per_pass(synthetic, tmp_path):
    path = str(tmp_path / "issue.json")
    _run("stall_summary.py", ["%s" % TAG, "--json", path, "--workload", "w", "--run", "synthetic"])
    rec = json.load(open(path))["w"]
    assert rec["passes_profiled"] == 2
    assert rec["trace_per_pass"]["SQ_INSTS_VALU"] == 2 * 100
    assert rec["per_pass"]["SQ_INSTS_VALU"] == 2 * 100 + 2 * 10
