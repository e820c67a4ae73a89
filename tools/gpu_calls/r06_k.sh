#!/bin/bash
# Round 6, call K: tail bounces' shade/reorder grids capped (RTAMD_TAIL_GRID) -- concurrent-tail probe, 13-pass share,
# 20 steps.
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
for g in 0 256 64; do
  RTAMD_TAIL_GRID=$g PROBE_TAG=grid$g timeout -k 10 300 python tools/tail_probe.py 1 6 >> $O/tail_probe.json 2> $O/tail_probe_$g.err || { tail $O/tail_probe_$g.err; exit 1; }
done
cat $O/tail_probe.json | cut -c1-150
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_TAIL_GRID=256 default@RTAMD_TAIL_GRID=64 default@RTAMD_TAIL_GRID=64,RTAMD_TAIL_FROM=3 \
  -- --steps 13 --warmup 2 --dist > $O/ab13.txt 2>&1 || { tail $O/ab13.txt; exit 1; }
tail -5 $O/ab13.txt
timeout -k 10 600 python tools/ab.py 3 default default@RTAMD_TAIL_GRID=256 default@RTAMD_TAIL_GRID=64 \
  -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -4 $O/ab20.txt
