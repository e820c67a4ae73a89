#!/bin/bash
# Round 6, call U: where GScan's time goes -- its shade-kernel work (group-sum atomics, fences, ticket, last-workgroup
# scan) in "shadow" variants that still take their offsets from the scan launch.
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 900 python tools/ab.py 3 default@RTAMD_GSCAN=0 sh_full sh_noatom sh_nofence sh_neither default -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -7 $O/ab20.txt
