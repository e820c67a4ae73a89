#!/bin/bash
# Round 6 session 2, call H3: the torch.distributed path's 20-step batch (the driver's SCALE shape per rank) on one
# GPU, passes in flight x hardware queues, against the 1-GPU default line.
export TMPDIR=/tmp
O=gpurun_out/r06h3; mkdir -p $O
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_HW_QUEUES=32 default@RTAMD_INFLIGHT=18,RTAMD_HW_QUEUES=32 \
  default@RTAMD_INFLIGHT=20,RTAMD_HW_QUEUES=32 -- --dist --steps 20 --warmup 5 > $O/ab_dist20.txt 2>&1 || { tail -20 $O/ab_dist20.txt; exit 1; }
tail -6 $O/ab_dist20.txt
timeout -k 10 300 python tools/ab.py 3 default -- --steps 20 --warmup 5 > $O/ab_plain20.txt 2>&1 || { tail -20 $O/ab_plain20.txt; exit 1; }
tail -3 $O/ab_plain20.txt
