#!/bin/bash
# Round 6, call Y: the whole GPU suite and smoke at HEAD, then the driver's bench command.
# driver's bench command.
export TMPDIR=/tmp
O=gpurun_out/r06y2; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['bit_exact_vs_oracle'], j['roofline']['frac'])"
