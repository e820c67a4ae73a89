#!/bin/bash
# r05: per-kernel times of a lamp pass alone (sort on), for where lamp's time goes
export TMPDIR=/tmp
OUT=gpurun_out/r5_lk1; mkdir -p $OUT
PK_SCENE=lamp_available.scene PK_IMAGE=1920,1080,4096,32 PK_RUNS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/pass_kernels.py > $OUT/pk.log 2>&1 || { tail $OUT/pk.log; exit 1; }
grep "run " $OUT/pk.log
python3 tools/trace_summary.py trace $OUT/prof/run_kernel_trace.csv 32 > $OUT/summary.txt 2>&1 || { tail $OUT/summary.txt; exit 1; }
head -16 $OUT/summary.txt
