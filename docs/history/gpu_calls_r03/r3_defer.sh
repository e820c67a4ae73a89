# Round 3: a fresh ray's setup deferred past the next step (RT_DEFER_SETUP=1: its ray loads overlap the
# step's record loads): parity, then A/B against the root-step build (build_var/root) and the
# refactored default (build_var/newdef)
export TMPDIR=/tmp
OUT=gpurun_out/r3_defer
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/defer/librtamd.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_defer.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests_defer.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 root newdef defer > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 4 root newdef defer > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 root newdef defer > $OUT/ab_lamp.txt 2>&1; tail -4 $OUT/ab_lamp.txt
echo done
