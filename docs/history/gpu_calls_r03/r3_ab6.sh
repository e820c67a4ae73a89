# Round 3: the stack top read beside the record loads (RT_PREPOP): parity of the variant, A/B
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab6
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prepop/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace_rays.py tests/test_gpu_baseline_sizes.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_prepop.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests_prepop.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 4 default prepop > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 400 python tools/ab.py 4 default prepop > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 400 python tools/ab.py 2 default prepop > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
echo done
