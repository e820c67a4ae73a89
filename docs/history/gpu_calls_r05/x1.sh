#!/bin/bash
# r05: GPU tests with the ADVICE fixes + XCD-affine trace order + overlapped in-library exchange,
# record-uniformity profile, then A/B of the order (off / bounce 1 / all).
export TMPDIR=/tmp
OUT=gpurun_out/r5_x1; mkdir -p $OUT
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== prof $(date +%T)"
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prof/librtamd.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-extras > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep RT_PROFILE $OUT/prof.err
echo "== ab20 $(date +%T)"
timeout -k 10 900 python tools/ab.py 3 default@RTAMD_XCDA=0 default default@RTAMD_XCDA=1 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
echo "== abfull $(date +%T)"
timeout -k 10 900 python tools/ab.py 2 default@RTAMD_XCDA=0 default -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -3 $OUT/abfull.txt
