# Round 3: 24 passes in flight (28 hardware queues) with the shaped stagger, full frame
export TMPDIR=/tmp
OUT=gpurun_out/r3_if24
mkdir -p $OUT
AB_ARGS="--no-extras" timeout -k 10 900 python tools/ab.py 3 default if24@GPU_MAX_HW_QUEUES=28 default@GPU_MAX_HW_QUEUES=28 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 600 python tools/ab.py 2 default if24@GPU_MAX_HW_QUEUES=28 > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
echo done
