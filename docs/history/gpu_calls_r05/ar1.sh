#!/bin/bash
# r05: trace ray registers in the state-record layout {o.x d.x o.y d.y}{o.z d.z} (default) and the asynchronous
# refill (async: a refilled lane's ray loads overlap the next step's record loads) against the previous build (base)
export TMPDIR=/tmp
OUT=gpurun_out/r5_ar1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/async/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity_async.log 2>&1 || { tail -30 $OUT/parity_async.log; exit 1; }
tail -1 $OUT/parity_async.log
timeout -k 10 600 python tools/launch_ab.py 3 base default async > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -4 $OUT/launch.txt
timeout -k 10 1000 python tools/ab.py 3 base default async -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
timeout -k 10 1000 python tools/ab.py 2 base default async -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
