#!/bin/bash
# r05: slimmer ray state (radiance kept in acc[ray id], 40 instead of 52 B per live ray): parity + A/B vs HEAD
export TMPDIR=/tmp
OUT=gpurun_out/r5_st1; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python tools/launch_ab.py 3 base default sh8 > $OUT/launch_ab.txt 2>&1 || { tail $OUT/launch_ab.txt; exit 1; }
tail -3 $OUT/launch_ab.txt
timeout -k 10 900 python tools/ab.py 4 base default sh8 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -3 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 2 base default -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -3 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 base default -- --scene lamp --steps 20 --warmup 3 > $OUT/ablamp.txt 2>&1 || { tail $OUT/ablamp.txt; exit 1; }
tail -3 $OUT/ablamp.txt
