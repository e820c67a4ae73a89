# Round 4: the reorder's scan fused into the shade kernel's last workgroup from bounce RTAMD_SCAN_FUSE on
# (one launch fewer per bounce in every pass's dependent chain): parity at 0 (every bounce) and 2,
# the device-clock timeline at 2, interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_sf1
mkdir -p $OUT
for f in 0 2; do
RTAMD_SCAN_FUSE=$f timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -v --timeout 200 --timeout-method thread > $OUT/parity_$f.log 2>&1 || { tail -30 $OUT/parity_$f.log; exit 1; }
tail -1 $OUT/parity_$f.log
done
RTAMD_SCAN_FUSE=2 RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_sf2.json 2> $OUT/tl_sf2.err || { tail $OUT/tl_sf2.err; exit 1; }
cut -c1-160 $OUT/tl_sf2.json
timeout -k 10 800 python tools/ab.py 4 default default@RTAMD_SCAN_FUSE=2 default@RTAMD_SCAN_FUSE=1 default@RTAMD_SCAN_FUSE=4 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -5 $OUT/ab_steps20.txt
echo done
