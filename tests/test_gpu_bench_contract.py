"""bench.py's output contract on the GPU: one JSON line on stdout with the driver's keys, whatever
native libraries print (a short run: one timed pass, no extra legs)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "render_wall_ms", "bit_exact_vs_oracle"}


def test_bench_prints_one_json_line():
    out = subprocess.run([sys.executable, "bench.py", "--scene", "cornell", "--steps", "2", "--warmup", "1",
                          "--no-extras"], cwd=REPO, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["higher_is_better"] is True
    assert rec["unit"] == "Mrays/s" and rec["dtype"] == "f32" and rec["scaling"] in ("weak", "strong")
    assert isinstance(rec["config"], dict) and "workload" in rec["config"]
