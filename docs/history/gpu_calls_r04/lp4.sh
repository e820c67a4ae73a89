# Round 4: parallel leaves with the triangle loads in flight beside the node records (lpo*) — GPU suite on lpo12w7, interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_lp4
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/lpo12w7/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_lpo12w7.log 2>&1 || { tail -30 $OUT/gpu_tests_lpo12w7.log; exit 1; }
tail -1 $OUT/gpu_tests_lpo12w7.log
timeout -k 10 900 python tools/ab.py 3 default lp12w7old lpo12w7 lpo16w7 lpo12 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -7 $OUT/ab_steps20.txt
echo done
