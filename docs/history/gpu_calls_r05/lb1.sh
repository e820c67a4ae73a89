#!/bin/bash
# r05: the in-library multi-device render at N > 1 on one GPU through the loopback transport
export TMPDIR=/tmp
OUT=gpurun_out/r5_lb1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x -k "multi_device" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "PASS|FAIL" $OUT/tests.log | tail -20; tail -1 $OUT/tests.log
