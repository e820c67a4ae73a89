# Round 3: the root's step at refill (RT_ROOT_STEP=1, build_var/root): parity, then A/B against HEAD's
# library (build_var/head) and the refactored default
export TMPDIR=/tmp
OUT=gpurun_out/r3_root
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/root2/librtamd.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_root2.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests_root2.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 3 head default root root2 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 4 head default root root2 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 head root root2 > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
echo done
