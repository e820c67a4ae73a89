# Round 3: with the root step at refill, the whole GPU suite on the default build, then the refill
# thresholds re-checked (later bounces 16/24/32 idle lanes, bounce 0 32/48/64)
export TMPDIR=/tmp
OUT=gpurun_out/r3_refill2
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 default ref16 ref32 rf48 rf32 > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 3 default ref16 ref32 rf48 rf32 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
echo done
