#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python tools/tail_probe.py 1 2 4 6 > $O/tail_probe.json 2> $O/tail_probe.err || { tail $O/tail_probe.err; exit 1; }
cat $O/tail_probe.json
