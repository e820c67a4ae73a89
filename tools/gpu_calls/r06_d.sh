#!/bin/bash
# Round 6, call D: stagger for runs shorter than the passes in flight (a rank's 13-pass share at N = 8), A/B.
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=1000 \
  default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=2000 default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=4000 \
  default@RTAMD_STAGGER_SHORT=1,RTAMD_STAGGER_US=2000,RTAMD_STAGGER_GROUP=2 \
  -- --steps 13 --warmup 2 > $O/ab_share13.txt 2>&1 || { tail -20 $O/ab_share13.txt; exit 1; }
tail -7 $O/ab_share13.txt
