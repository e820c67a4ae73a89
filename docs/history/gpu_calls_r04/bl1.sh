# Round 4: trace records through one buffer resource with 32-bit offsets (bl1; bl2 with a branchless
# offset select), node records and triangles in one allocation (also the default build now):
# GPU suite on the default and bl2, interleaved A/B at 20 steps, full frame, lamp
export TMPDIR=/tmp
OUT=gpurun_out/r4_bl1
mkdir -p $OUT
for v in default bl2; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$v.log 2>&1 || { tail -30 $OUT/gpu_tests_$v.log; exit 1; }
  tail -1 $OUT/gpu_tests_$v.log
done
timeout -k 10 600 python tools/ab.py 4 default bl1 bl2 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -4 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default bl1 bl2 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 default bl1 bl2 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -4 $OUT/ab_lamp.txt
echo done
