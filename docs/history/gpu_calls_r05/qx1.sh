#!/bin/bash
# r05: the reorder key's quantisation in fp32 (qb; exhaustively equal to the double form) and the XCD-contiguous
# accumulation blocks (default = both) against the previous build (base)
export TMPDIR=/tmp
OUT=gpurun_out/r5_qx1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python tools/launch_ab.py 3 base qb default > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -4 $OUT/launch.txt
timeout -k 10 1000 python tools/ab.py 4 base qb default -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
timeout -k 10 1000 python tools/ab.py 2 base qb default -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
