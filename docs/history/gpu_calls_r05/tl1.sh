#!/bin/bash
# r05: smaller trace grids for the tail bounces (fewer long-resident straggler workgroups in the shared chip)
export TMPDIR=/tmp
OUT=gpurun_out/r5_tl1; mkdir -p $OUT
V="default default@RTAMD_TAIL_FROM=2,RTAMD_TAIL_PCT=50 default@RTAMD_TAIL_FROM=2,RTAMD_TAIL_PCT=25 default@RTAMD_TAIL_FROM=3,RTAMD_TAIL_PCT=25 default@RTAMD_TAIL_FROM=2,RTAMD_TAIL_PCT=10"
timeout -k 10 1000 python tools/ab.py 3 $V -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -6 $OUT/ab20.txt
timeout -k 10 1000 python tools/ab.py 2 $V -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -6 $OUT/abfull.txt
