#!/bin/bash
# Round 6 session 2, call H6: bench.py's new config.passes_in_flight -- the GPU tests that run bench.py, then the
# driver's line and the --dist line.
export TMPDIR=/tmp
O=gpurun_out/r06h6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_contract.py tests/test_gpu_bench_world2.py tests/test_gpu_dist_rccl.py \
  tests/test_gpu_multi_renderer.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_bench_tests.log 2>&1 || { tail -40 $O/gpu_bench_tests.log; exit 1; }
tail -2 $O/gpu_bench_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --dist --steps 20 --warmup 5 --no-extras > $O/bench_dist.json 2> $O/bench_dist.err || { tail -20 $O/bench_dist.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_dist'):
    j = json.load(open('$O/%s.json' % f)); print(f, j['ms_per_step'], j['bit_exact_vs_oracle'], j['config']['passes_in_flight'])"
