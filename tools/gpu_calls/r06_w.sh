#!/bin/bash
# Round 6, call W: GScan with the plain scatter held at 8 waves/SIMD (its prologue took it to 106 SGPRs, 7 waves).
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 900 python tools/ab.py 5 default default@RTAMD_GSCAN=0 swpe8 -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -4 $O/ab20.txt
