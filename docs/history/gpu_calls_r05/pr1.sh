#!/bin/bash
# r05 timing probes (wrong images, timing only): the later-bounce shade's scattered radiance stores (accslot)
# and the f64 bucket quantisation (bf32)
export TMPDIR=/tmp
OUT=gpurun_out/r5_pr1; mkdir -p $OUT
timeout -k 10 600 python tools/launch_ab.py 3 default accslot bf32 both > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -5 $OUT/launch.txt
timeout -k 10 900 python tools/ab.py 3 default accslot bf32 both -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -5 $OUT/ab20.txt
