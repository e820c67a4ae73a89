# Round 4: parallel leaves with the cheap trigger, and the min-7-waves later-bounce kernel — GPU suite on lp16w7, interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_lp2
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/lp16w7/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_lp16w7.log 2>&1 || { tail -30 $OUT/gpu_tests_lp16w7.log; exit 1; }
tail -1 $OUT/gpu_tests_lp16w7.log
timeout -k 10 900 python tools/ab.py 3 default w7 lp16w7 lp12w7 lp24w7 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -7 $OUT/ab_steps20.txt
echo done
