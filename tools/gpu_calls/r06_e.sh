#!/bin/bash
# Round 6, call E: short-run stagger on the share paths (16 in flight; torch.distributed RCCL at world 1), A/B.
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 700 python tools/ab.py 3 default default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=1500 \
  default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=2000 default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=3000 \
  -- --steps 13 --warmup 2 --dist > $O/ab_share13_dist.txt 2>&1 || { tail -20 $O/ab_share13_dist.txt; exit 1; }
tail -5 $O/ab_share13_dist.txt
timeout -k 10 500 python tools/ab.py 3 default default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=2000 \
  -- --steps 26 --warmup 2 --dist > $O/ab_share26_dist.txt 2>&1 || { tail -20 $O/ab_share26_dist.txt; exit 1; }
tail -3 $O/ab_share26_dist.txt
