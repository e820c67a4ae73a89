# Round 3: bounce 0 only, a second (depth-1) step at refill from scalar registers (RT_ROOT2_FIRST=1,
# build_var/r2f): parity, then A/B against the default build
export TMPDIR=/tmp
OUT=gpurun_out/r3_r2f
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/r2f/librtamd.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_r2f.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests_r2f.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 5 default r2f > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 5 default r2f > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default r2f > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
echo done
