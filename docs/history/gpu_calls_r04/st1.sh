# Round 4: nontemporal hints on every streaming access -- st: stores of hits, ray state, buckets, reorder
# outputs; ld: loads of the same (and accumulation's reads); stld: both -- on top of the default
# (nontemporal acc stores): GPU suite on stld, interleaved A/B at 20 steps, then full frame
export TMPDIR=/tmp
OUT=gpurun_out/r4_st1
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/stld/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_stld.log 2>&1 || { tail -30 $OUT/gpu_tests_stld.log; exit 1; }
tail -1 $OUT/gpu_tests_stld.log
timeout -k 10 700 python tools/ab.py 4 default st ld stld -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -5 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 2 default st ld stld > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -5 $OUT/ab_frame.txt
echo done
