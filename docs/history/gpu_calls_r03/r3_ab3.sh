# Round 3: predicated leaf/node step A/B + parity (GPU box)
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab3
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/pred1/librtamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_scenes.py tests/test_gpu_trace_rays.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_pred1.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests_pred1.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 4 default pred1 pred2 rcp pred1rcp > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 400 python tools/ab.py 3 default pred1 rcp pred1rcp > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 400 python tools/ab.py 3 default pred1 rcp pred1rcp > $OUT/ab_lamp.txt 2>&1; tail -6 $OUT/ab_lamp.txt
