#!/bin/bash
# Round 6, call O: passes in flight = hardware queues, fewer of both (dispatch latency collapses above ~4-8 active
# queues, profiles/r06/launch_latency_vs_queues.txt), 20 steps and 13-pass batches.
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 700 python tools/ab.py 3 default default@RTAMD_HW_QUEUES=8,RTAMD_INFLIGHT=8 default@RTAMD_HW_QUEUES=12,RTAMD_INFLIGHT=12 \
  default@RTAMD_HW_QUEUES=16,RTAMD_INFLIGHT=16 -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -5 $O/ab20.txt
timeout -k 10 500 python tools/ab.py 3 default default@RTAMD_HW_QUEUES=8,RTAMD_INFLIGHT=8 default@RTAMD_HW_QUEUES=12,RTAMD_INFLIGHT=12 \
  -- --steps 13 --warmup 2 > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -4 $O/ab13.txt
