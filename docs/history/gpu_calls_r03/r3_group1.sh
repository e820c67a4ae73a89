# Round 3: 16-lanes-per-ray tail trace (trace_group_kernel): parity with it on every bounce >= 1, with its
# reference-order fallback forced, the default threshold, then A/B of the threshold
export TMPDIR=/tmp
OUT=gpurun_out/r3_group1
mkdir -p $OUT
T="tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_full_size.py"
RTAMD_GROUP_BELOW=2000000000 timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all_group.log 2>&1; rc=$?
tail -2 $OUT/tests_all_group.log
[ $rc -eq 0 ] || exit $rc
RTAMD_GROUP_BELOW=2000000000 RTAMD_FORCE_EXACT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_forced_exact.log 2>&1; rc=$?
tail -1 $OUT/tests_forced_exact.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 900 python tools/ab.py 5 default@RTAMD_GROUP_BELOW=0 default default@RTAMD_GROUP_BELOW=8192 default@RTAMD_GROUP_BELOW=131072 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 2 default@RTAMD_GROUP_BELOW=0 default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
echo done
