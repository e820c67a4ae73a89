#!/bin/bash
# Round 6, call AE: both trace step bodies on every lane, results selected by kind (RT_FLAT_KIND=1: no exec-mask
# branch per step; static -9 SALU, -7 branches, +4 VALU) -- parity through the variant library, then A/B.
export TMPDIR=/tmp
O=gpurun_out/r06ae; mkdir -p $O
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/flat/librtamd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_random_configs.py tests/test_gpu_edge_scenes.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python tools/ab.py 4 default flat -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -3 $O/ab20.txt
timeout -k 10 600 python tools/ab.py 3 default flat -- --steps 13 --warmup 2 --inlib > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -3 $O/ab13.txt
