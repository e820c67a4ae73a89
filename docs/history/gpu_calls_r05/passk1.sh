#!/bin/bash
# r05: per-kernel times of teapot pass 0 alone (home-indexed radiance), then the 13/26-pass share probe
export TMPDIR=/tmp
OUT=gpurun_out/r5_pk1; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/pass_kernels.py > $OUT/pk.log 2>&1 || { tail $OUT/pk.log; exit 1; }
cat $OUT/pk.log | grep "run "
python3 tools/trace_summary.py trace $OUT/prof/run_kernel_trace.csv > $OUT/summary.txt 2>&1 || { tail $OUT/summary.txt; exit 1; }
head -16 $OUT/summary.txt
timeout -k 10 600 python tools/share_probe.py 13 26 > $OUT/share_probe.txt 2>&1 || { tail $OUT/share_probe.txt; exit 1; }
cat $OUT/share_probe.txt
