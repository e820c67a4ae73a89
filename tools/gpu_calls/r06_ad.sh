#!/bin/bash
# Round 6, call AD: the later-bounce shade launches hold 15 % of the timed regime's wave residency with 8192 mostly idle
# waves each (grid sized for the pass's first bounce): shade grids of 4 / 2 workgroups per CU instead of 8.
export TMPDIR=/tmp
O=gpurun_out/r06ad; mkdir -p $O
timeout -k 10 900 python tools/ab.py 4 default sbpc4 sbpc2 -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -4 $O/ab20.txt
