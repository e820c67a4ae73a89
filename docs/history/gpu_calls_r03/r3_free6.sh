# Round 3: why the order-free frame is slower with many passes in flight: lamp/teapot full frame
# free (8 waves, bounce-0 spills) vs free (7 waves at bounce 0, no spills) vs reference order;
# and the free kernel at 4 passes in flight
export TMPDIR=/tmp
OUT=gpurun_out/r3_free6
mkdir -p $OUT
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 1 default@RTAMD_EXACT_TRACE=1 wpe7 default@RTAMD_INFLIGHT=4 > $OUT/ab_lamp.txt 2>&1; tail -4 $OUT/ab_lamp.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 2 default@RTAMD_EXACT_TRACE=1 wpe7 default > $OUT/ab_teapot.txt 2>&1; tail -4 $OUT/ab_teapot.txt
echo done
