# Round 4: parallel-leaf trace (RT_LEAFPAR) — GPU suite on the lp48 build, then an interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_lp1
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/lp48/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_lp48.log 2>&1 || { tail -30 $OUT/gpu_tests_lp48.log; exit 1; }
tail -1 $OUT/gpu_tests_lp48.log
timeout -k 10 900 python tools/ab.py 3 default lp48 lp32 lp48r16 lp64 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -7 $OUT/ab_steps20.txt
echo done
