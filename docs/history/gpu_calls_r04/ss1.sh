# Round 4: tail bounces without the scan launch -- the scatter derives its bucket runs from the per-tile
# counts (RTAMD_SELF_SCAN = first such bounce): parity at 1 and 6, timeline at 6, interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_ss1
mkdir -p $OUT
for f in 1 6; do
RTAMD_SELF_SCAN=$f timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -v --timeout 200 --timeout-method thread > $OUT/parity_$f.log 2>&1 || { tail -30 $OUT/parity_$f.log; exit 1; }
tail -1 $OUT/parity_$f.log
done
RTAMD_SELF_SCAN=6 RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_ss6.json 2> $OUT/tl_ss6.err || { tail $OUT/tl_ss6.err; exit 1; }
cut -c1-160 $OUT/tl_ss6.json
timeout -k 10 800 python tools/ab.py 4 default default@RTAMD_SELF_SCAN=4 default@RTAMD_SELF_SCAN=6 default@RTAMD_SELF_SCAN=8 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -5 $OUT/ab_steps20.txt
echo done
