#!/bin/bash
# Round 6, call V: GScan (the reorder scan folded into the shade and scatter kernels) -- parity, then A/B against RTAMD_GSCAN=0.
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_random_configs.py tests/test_gpu_tiles.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python tools/ab.py 4 default default@RTAMD_GSCAN=0 -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -3 $O/ab20.txt
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_GSCAN=0 -- --steps 13 --warmup 2 --inlib > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -3 $O/ab13.txt
