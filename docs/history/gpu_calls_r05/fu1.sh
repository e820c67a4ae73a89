#!/bin/bash
# r05: which bounces take the fused replay now that the replay runs at 8 waves and the state is 40 B
export TMPDIR=/tmp
OUT=gpurun_out/r5_fu1; mkdir -p $OUT
timeout -k 10 900 python tools/ab.py 3 default default@RTAMD_FUSED=3 default@RTAMD_FUSED=1 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 2 default default@RTAMD_FUSED=3 default@RTAMD_FUSED=1 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 default default@RTAMD_FUSED=3 default@RTAMD_FUSED=1 -- --scene cornell_plus > $OUT/abcp.txt 2>&1 || { tail $OUT/abcp.txt; exit 1; }
tail -4 $OUT/abcp.txt
timeout -k 10 900 python tools/ab.py 1 default default@RTAMD_FUSED=3 -- --scene lamp --steps 10 --warmup 3 > $OUT/ablamp.txt 2>&1 || { tail $OUT/ablamp.txt; exit 1; }
tail -3 $OUT/ablamp.txt
