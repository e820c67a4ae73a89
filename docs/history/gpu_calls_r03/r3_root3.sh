# Round 3: the top BVH levels stepped at refill on an LDS copy of their records (RT_ROOT_STEP=3,
# RT_TOP_LEVELS 3/4/5): parity of the 4-level build, then A/B against the root-only step (build_var/root)
export TMPDIR=/tmp
OUT=gpurun_out/r3_root3
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/root3/librtamd.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_root3.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests_root3.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 head root root3k3 root3 root3k5 > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 4 head root root3k3 root3 root3k5 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 head root root3 root3k5 > $OUT/ab_lamp.txt 2>&1; tail -5 $OUT/ab_lamp.txt
echo done
