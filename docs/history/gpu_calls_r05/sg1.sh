#!/bin/bash
# r05: staggered-start knobs after the home-indexed radiance (default: group 4, one pass every 4 ms)
export TMPDIR=/tmp
OUT=gpurun_out/r5_sg1; mkdir -p $OUT
V="default default@RTAMD_STAGGER_US=2500 default@RTAMD_STAGGER_US=5500 default@RTAMD_STAGGER_GROUP=6 default@RTAMD_STAGGER_GROUP=2"
timeout -k 10 1000 python tools/ab.py 2 $V -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -6 $OUT/abfull.txt
timeout -k 10 1000 python tools/ab.py 3 $V -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -6 $OUT/ab20.txt
timeout -k 10 1000 python tools/ab.py 2 default if24@RTAMD_HW_QUEUES=28 default@RTAMD_HW_QUEUES=28 -- > $OUT/abif.txt 2>&1 || { tail $OUT/abif.txt; exit 1; }
tail -4 $OUT/abif.txt
