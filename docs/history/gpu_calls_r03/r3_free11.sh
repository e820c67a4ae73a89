# Round 3: order-free trace only on the tail bounces (latency-bound): frame, 20 steps, 13-pass share
export TMPDIR=/tmp
OUT=gpurun_out/r3_free11
mkdir -p $OUT
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 2 default@RTAMD_EXACT_TRACE=1 default@RTAMD_FREE_FROM=2 default@RTAMD_FREE_FROM=4 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_EXACT_TRACE=1 default@RTAMD_FREE_FROM=2 default@RTAMD_FREE_FROM=4 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
AB_ARGS="--no-extras --steps 13 --dist" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_EXACT_TRACE=1 default@RTAMD_FREE_FROM=2 default@RTAMD_FREE_FROM=4 > $OUT/ab_13.txt 2>&1; tail -4 $OUT/ab_13.txt
echo done
