#!/bin/bash
# r05: reorder grid cap (scatter / fused replay / histogram workgroups: default 8 per CU = 2048) -- fewer concurrent
# workgroups, fewer partially written run frontiers in L2
export TMPDIR=/tmp
OUT=gpurun_out/r5_sgr1; mkdir -p $OUT
timeout -k 10 600 python tools/launch_ab.py 3 default sg512 sg1024 > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -4 $OUT/launch.txt
timeout -k 10 1000 python tools/ab.py 3 default sg512 sg1024 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
timeout -k 10 1000 python tools/ab.py 2 default sg512 sg1024 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
