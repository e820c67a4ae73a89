# Round 4: bounce launch grids sized by the live rays of earlier runs (RTAMD_LIVE_HINTS, default on):
# the GPU suite (incl. undersized-grid parity), the device-clock timeline, interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_lh1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_lh.json 2> $OUT/tl_lh.err || { tail $OUT/tl_lh.err; exit 1; }
cut -c1-160 $OUT/tl_lh.json
timeout -k 10 800 python tools/ab.py 4 default default@RTAMD_LIVE_HINTS=0 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -3 $OUT/ab_steps20.txt
timeout -k 10 500 python tools/ab.py 2 default default@RTAMD_LIVE_HINTS=0 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -3 $OUT/ab_frame.txt
echo done
