# Round 3: order-free trace (trace_free_kernel + reference-order re-trace): every GPU test, the
# re-trace path forced, then an interleaved A/B against the reference-order trace
export TMPDIR=/tmp
OUT=gpurun_out/r3_free1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
RTAMD_FORCE_RETRACE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace_rays.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_forced.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests_forced.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_EXACT_TRACE=1 default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 400 python tools/ab.py 2 default@RTAMD_EXACT_TRACE=1 default > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
echo done
