#!/bin/bash
# Round 6, call S: one more launch per bounce (RTAMD_SHADE_HIST=0) -- does launch count matter in the shared regime?
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 600 python tools/ab.py 4 default default@RTAMD_SHADE_HIST=0 -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -3 $O/ab20.txt
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_SHADE_HIST=0 -- --steps 13 --warmup 2 --inlib > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -3 $O/ab13.txt
