#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/r5_w2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_world2.py tests/test_gpu_queue_sharing.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log
