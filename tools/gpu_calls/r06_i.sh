#!/bin/bash
# Round 6, call I: do concurrent tails slow each other?  Device-clock timelines of batches of 1, 2, 4, 6 passes
# started together (no stagger below 8 passes), plain path.
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
for n in 1 2 4 6; do
  RTAMD_TIMELINE=1 timeout -k 10 300 python bench.py --steps $n --warmup 1 --no-cpu-baseline --no-counters > $O/b$n.json 2> $O/b$n.err || { tail $O/b$n.err; exit 1; }
  python3 tools/pass_timeline.py $O/b$n.err $n | tee $O/timeline$n.txt
done
