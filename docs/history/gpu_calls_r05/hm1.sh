#!/bin/bash
# r05: home-indexed radiance (acc[home] = the bounce-1 slot for rays that survive bounce 0) vs acc[ray id]
export TMPDIR=/tmp
OUT=gpurun_out/r5_hm1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_world2.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 600 python tools/launch_ab.py 3 default default@RTAMD_HOME=0 > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -3 $OUT/launch.txt
timeout -k 10 900 python tools/ab.py 3 default default@RTAMD_HOME=0 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -3 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 2 default default@RTAMD_HOME=0 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -3 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 default default@RTAMD_HOME=0 -- --scene cornell_plus > $OUT/abcp.txt 2>&1 || { tail $OUT/abcp.txt; exit 1; }
tail -3 $OUT/abcp.txt
timeout -k 10 900 python tools/ab.py 1 default default@RTAMD_HOME=0 -- --scene lamp --steps 10 --warmup 3 > $OUT/ablamp.txt 2>&1 || { tail $OUT/ablamp.txt; exit 1; }
tail -3 $OUT/ablamp.txt
