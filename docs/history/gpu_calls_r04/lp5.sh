# Round 4: parallel leaves only from bounce k on (RTAMD_LEAFPAR_FROM): the tail's chains — interleaved A/B, 20 steps and the full frame
export TMPDIR=/tmp
OUT=gpurun_out/r4_lp5
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/lpo12w7/librtamd.so RTAMD_LEAFPAR_FROM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 900 python tools/ab.py 3 default lpo12w7@RTAMD_LEAFPAR_FROM=2 lpo12w7@RTAMD_LEAFPAR_FROM=3 lpo12w7@RTAMD_LEAFPAR_FROM=5 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
timeout -k 10 900 python tools/ab.py 2 default lpo12w7@RTAMD_LEAFPAR_FROM=2 lpo12w7@RTAMD_LEAFPAR_FROM=3 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -5 $OUT/ab_frame.txt
echo done
