#!/bin/bash
# r05: sparse tail waves (at most K rays per wave when few rays live): parity, exclusive launches, batches
export TMPDIR=/tmp
OUT=gpurun_out/r5_sp1; mkdir -p $OUT
V=$PWD/cuda-raytracer_amd/build_var
RTAMD_LIB=$V/sp8/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity_sp8.log 2>&1 || { tail -30 $OUT/parity_sp8.log; exit 1; }
tail -1 $OUT/parity_sp8.log
timeout -k 10 600 python tools/launch_ab.py 3 default sp4 sp8 sp16 sp8w > $OUT/launch_ab.txt 2>&1 || { tail $OUT/launch_ab.txt; exit 1; }
tail -6 $OUT/launch_ab.txt
timeout -k 10 900 python tools/ab.py 3 default sp8 sp16 sp8w -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -5 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 3 default sp8 sp16 sp8w -- --steps 13 --warmup 3 > $OUT/ab13.txt 2>&1 || { tail $OUT/ab13.txt; exit 1; }
tail -5 $OUT/ab13.txt
timeout -k 10 900 python tools/ab.py 2 default sp8 sp16 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
