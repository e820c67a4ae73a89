#!/bin/bash
# Round 6, call F: the short-run stagger as the default -- 13-pass share (plain and dist), cornell_plus frame
# (13 passes of 512^2), the 20-step line (unchanged rule), against RTAMD_STAGGER_SHORT_US=0 (round 5's rule).
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 500 python tools/ab.py 3 default default@RTAMD_STAGGER_SHORT_US=0 -- --steps 13 --warmup 2 --dist > $O/ab13_dist.txt 2>&1 || { tail $O/ab13_dist.txt; exit 1; }
tail -2 $O/ab13_dist.txt
timeout -k 10 400 python tools/ab.py 5 default default@RTAMD_STAGGER_SHORT_US=0 -- --scene cornell_plus > $O/ab_cornell_plus.txt 2>&1 || { tail $O/ab_cornell_plus.txt; exit 1; }
tail -2 $O/ab_cornell_plus.txt
timeout -k 10 400 python tools/ab.py 3 default default@RTAMD_STAGGER_SHORT_US=0 -- --scene lamp --steps 13 --warmup 2 > $O/ab_lamp13.txt 2>&1 || { tail $O/ab_lamp13.txt; exit 1; }
tail -2 $O/ab_lamp13.txt
