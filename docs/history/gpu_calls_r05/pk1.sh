#!/bin/bash
# r05: packed Moller-Trumbore on a paired triangle record (later bounces): parity, launch and batch A/B vs flat
export TMPDIR=/tmp
OUT=gpurun_out/r5_pk1; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python tools/launch_ab.py 3 flat default > $OUT/launch_ab.txt 2>&1 || { tail $OUT/launch_ab.txt; exit 1; }
tail -3 $OUT/launch_ab.txt
timeout -k 10 900 python tools/ab.py 4 flat default -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -3 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 2 flat default -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -3 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 flat default -- --scene lamp --steps 20 --warmup 3 > $OUT/ablamp.txt 2>&1 || { tail $OUT/ablamp.txt; exit 1; }
tail -3 $OUT/ablamp.txt
