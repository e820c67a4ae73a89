# Round 3: passes in flight with the staggered start, 20-pass batch and full frame
export TMPDIR=/tmp
OUT=gpurun_out/r3_inflight
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 900 python tools/ab.py 5 default default@RTAMD_INFLIGHT=16 default@RTAMD_INFLIGHT=12 default@RTAMD_INFLIGHT=16,RTAMD_STAGGER_US=3000 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 2 default default@RTAMD_INFLIGHT=16 > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
echo done
