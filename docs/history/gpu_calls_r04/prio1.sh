# Round 4: issue priority for the tail bounces' waves (RTAMD_TAIL_PRIO = first bounce, RTAMD_PRIO_LEVEL =
# level, +4: shade waves too): parity with the knob on, interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_prio1
mkdir -p $OUT
RTAMD_TAIL_PRIO=1 RTAMD_PRIO_LEVEL=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 900 python tools/ab.py 4 default default@RTAMD_TAIL_PRIO=2 default@RTAMD_TAIL_PRIO=2,RTAMD_PRIO_LEVEL=6 default@RTAMD_TAIL_PRIO=1 default@RTAMD_TAIL_PRIO=0,RTAMD_PRIO_LEVEL=1 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
