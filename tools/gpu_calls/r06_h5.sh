#!/bin/bash
# Round 6 session 2, call H5: the torch.distributed path's 20-pass batch with 20 / 17 passes in flight on fewer
# hardware queues than streams (does the 20-in-flight cliff of call H3 come from the queues the process holds?).
export TMPDIR=/tmp
O=gpurun_out/r06h5; mkdir -p $O
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_INFLIGHT=20,RTAMD_HW_QUEUES=22 default@RTAMD_INFLIGHT=20,RTAMD_HW_QUEUES=24 \
  default@RTAMD_INFLIGHT=17 -- --dist --steps 20 --warmup 5 > $O/ab_dist20.txt 2>&1 || { tail -20 $O/ab_dist20.txt; exit 1; }
tail -6 $O/ab_dist20.txt
