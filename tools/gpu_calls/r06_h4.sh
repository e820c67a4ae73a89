#!/bin/bash
# Round 6 session 2, call H4: attribute the torch.distributed path's 20-pass batch (6.16 vs 5.92 ms/pass, call H3):
# the plain path at 16 passes in flight, and the in-library path (rt_multi at N = 1, system HIP runtime, 16 in flight).
export TMPDIR=/tmp
O=gpurun_out/r06h4; mkdir -p $O
timeout -k 10 400 python tools/ab.py 3 default default@RTAMD_INFLIGHT=16 -- --steps 20 --warmup 5 > $O/ab_plain.txt 2>&1 || { tail -20 $O/ab_plain.txt; exit 1; }
tail -3 $O/ab_plain.txt
timeout -k 10 400 python tools/ab.py 3 default default@RTAMD_HW_QUEUES=32 -- --inlib --steps 20 --warmup 5 > $O/ab_inlib.txt 2>&1 || { tail -20 $O/ab_inlib.txt; exit 1; }
tail -3 $O/ab_inlib.txt
