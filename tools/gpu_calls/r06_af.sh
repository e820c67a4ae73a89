#!/bin/bash
# Round 6, call AF: the whole 1080p teapot frame (103 passes, sort on) against the oracle's frame hash, through the
# GPU test and through bench.py's full-frame line.
export TMPDIR=/tmp
O=gpurun_out/r06af; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_baseline_sizes.py -k "frame" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_teapot.json 2> $O/bench_teapot.err || { tail $O/bench_teapot.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench_teapot.json')); print(j['value'], j['render_wall_ms'], j['parity'])"
