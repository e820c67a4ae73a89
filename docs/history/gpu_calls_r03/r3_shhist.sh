# Round 3: the reorder histogram counted in the shade kernel: parity, A/B
export TMPDIR=/tmp
OUT=gpurun_out/r3_shhist
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 700 python tools/ab.py 5 default@RTAMD_SHADE_HIST=0 default > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_SHADE_HIST=0 default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 default@RTAMD_SHADE_HIST=0 default > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
AB_ARGS="--no-extras --scene cornell_plus" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_SHADE_HIST=0 default > $OUT/ab_cp.txt 2>&1; tail -3 $OUT/ab_cp.txt
echo done
