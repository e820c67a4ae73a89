#!/bin/bash
# Round 6, call Z: the torch.distributed path on the renderer's HIP runtime (librtamd loaded before torch) -- which
# runtime each way maps, a 13-pass share A/B, and the world-2 bench test with it.
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
for lf in 0 1; do
  RTAMD_LIB_FIRST=$lf timeout -k 10 300 python bench.py --dist --steps 13 --warmup 2 --no-extras > $O/b13_lf$lf.json 2> $O/b13_lf$lf.err || { tail $O/b13_lf$lf.err; exit 1; }
  python3 -c "import json; j=json.load(open('$O/b13_lf$lf.json')); print('lib_first=$lf', j['ms_per_step'], j['bit_exact_vs_oracle'], j['config']['hip_runtime'])"
done
timeout -k 10 900 python tools/ab.py 4 default default@RTAMD_LIB_FIRST=1 -- --steps 13 --warmup 2 --dist --no-extras > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -3 $O/ab13.txt
RTAMD_LIB_FIRST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_world2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/world2.log 2>&1 || { tail -30 $O/world2.log; exit 1; }
tail -1 $O/world2.log
