# Round 4: tail bounces on a second (normal-priority) stream per context, the heavy bounces' stream
# masked off every RTAMD_TAIL_RESERVE-th CU so the tail launches find free slots: parity, timeline, A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_ts2
mkdir -p $OUT
RTAMD_TAIL_STREAM=2 RTAMD_TAIL_RESERVE=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
RTAMD_TAIL_STREAM=2 RTAMD_TAIL_RESERVE=16 GPU_MAX_HW_QUEUES=32 RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_r16.json 2> $OUT/tl_r16.err || { tail $OUT/tl_r16.err; exit 1; }
cut -c1-160 $OUT/tl_r16.json
timeout -k 10 800 python tools/ab.py 3 default default@RTAMD_TAIL_STREAM=2,GPU_MAX_HW_QUEUES=32 default@RTAMD_TAIL_STREAM=2,RTAMD_TAIL_RESERVE=16,GPU_MAX_HW_QUEUES=32 default@RTAMD_TAIL_STREAM=2,RTAMD_TAIL_RESERVE=8,GPU_MAX_HW_QUEUES=32 default@RTAMD_TAIL_STREAM=3,RTAMD_TAIL_RESERVE=16,GPU_MAX_HW_QUEUES=32 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
