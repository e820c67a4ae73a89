#!/bin/bash
# Round 6, call AG: both whole 1080p teapot frames against the oracle's frame hashes (GPU test), and the closing
# full-frame teapot lines (sort on / off) that now carry the frame parity.
export TMPDIR=/tmp
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_baseline_sizes.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench_teapot.json 2> $O/bench_teapot.err || { tail $O/bench_teapot.err; exit 1; }
timeout -k 10 900 python bench.py --scene teapot --no-sort > $O/bench_teapotnosort.json 2> $O/bench_teapotnosort.err || { tail $O/bench_teapotnosort.err; exit 1; }
for f in bench_teapot bench_teapotnosort; do
  python3 -c "import json; j=json.load(open('$O/$f.json')); print('$f', j['value'], j['render_wall_ms'], j['parity']['bit_exact_vs_oracle'], j['parity'].get('frame_bit_exact_vs_oracle'), j['cpu_baseline']['value'])"
done
