#!/bin/bash
# r05: per-kernel times of teapot pass 0 alone, sort on and sort off
export TMPDIR=/tmp
OUT=gpurun_out/r5_pk2; mkdir -p $OUT
for s in 1 0; do
  PK_SORT=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$s -o run --output-format csv -- python3 tools/pass_kernels.py > $OUT/pk$s.log 2>&1 || { tail $OUT/pk$s.log; exit 1; }
  python3 tools/trace_summary.py trace $OUT/prof$s/run_kernel_trace.csv > $OUT/summary$s.txt 2>&1 || { tail $OUT/summary$s.txt; exit 1; }
  grep "run 3" $OUT/pk$s.log
  head -13 $OUT/summary$s.txt
done
