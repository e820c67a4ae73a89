#!/bin/bash
# Round 6, call X: would batched tails pay?  One pass over k x the rays (its tail on one queue) vs k passes together.
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 500 python tools/batch_tail_probe.py 1 2 4 6 > $O/batch_tail.txt 2>&1 || { tail $O/batch_tail.txt; exit 1; }
cat $O/batch_tail.txt
timeout -k 10 300 python tools/tail_probe.py 1 2 4 6 > $O/tail_probe.txt 2>&1 || { tail $O/tail_probe.txt; exit 1; }
grep -h "timeline pass\|passes" $O/tail_probe.txt | tail -30
