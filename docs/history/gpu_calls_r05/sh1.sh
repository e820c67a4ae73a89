#!/bin/bash
# r05: shade_kernel at 8 waves/SIMD (waves_per_eu floor; 7 by its SGPR count) after the slim state
export TMPDIR=/tmp
OUT=gpurun_out/r5_sh1; mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/sh8/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 900 python tools/ab.py 5 default sh8 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -3 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 3 default sh8 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -3 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 default sh8 -- --scene lamp --steps 20 --warmup 3 > $OUT/ablamp.txt 2>&1 || { tail $OUT/ablamp.txt; exit 1; }
tail -3 $OUT/ablamp.txt
timeout -k 10 900 python tools/ab.py 2 default sh8 -- --scene cornell_plus > $OUT/abcp.txt 2>&1 || { tail $OUT/abcp.txt; exit 1; }
tail -3 $OUT/abcp.txt
