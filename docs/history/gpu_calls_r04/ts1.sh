# Round 4: tail bounces of every pass on a high-priority stream of its context (RTAMD_TAIL_STREAM = first
# tail bounce): parity with it on, interleaved A/B at 20 steps, and the device-clock timeline of one variant
export TMPDIR=/tmp
OUT=gpurun_out/r4_ts1
mkdir -p $OUT
RTAMD_TAIL_STREAM=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
RTAMD_TAIL_STREAM=2 GPU_MAX_HW_QUEUES=32 RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_ts2.json 2> $OUT/tl_ts2.err || { tail $OUT/tl_ts2.err; exit 1; }
cut -c1-160 $OUT/tl_ts2.json
timeout -k 10 800 python tools/ab.py 4 default default@RTAMD_TAIL_STREAM=2 default@RTAMD_TAIL_STREAM=2,GPU_MAX_HW_QUEUES=32 default@RTAMD_TAIL_STREAM=2,RTAMD_INFLIGHT=14,GPU_MAX_HW_QUEUES=32 default@RTAMD_TAIL_STREAM=1,GPU_MAX_HW_QUEUES=32 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
