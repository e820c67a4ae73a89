# Round 4: runtime knobs re-checked after the cheaper shade -- fused reorder at bounces 0-1 / every bounce,
# pass stagger 2 / 6 ms (4), first group of 8 (4) -- interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_knob1
mkdir -p $OUT
timeout -k 10 900 python tools/ab.py 4 default default@RTAMD_FUSED=3 default@RTAMD_FUSED=1 default@RTAMD_STAGGER_US=2000 default@RTAMD_STAGGER_US=6000 default@RTAMD_STAGGER_GROUP=8 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -7 $OUT/ab_steps20.txt
echo done
