# Round 4: material table staged in LDS per block in shade and the fused scatter-shade (RT_MAT_LDS,
# build_var/mlds): GPU suite, one pass alone under the kernel trace, interleaved A/B (20 steps, frame, lamp)
export TMPDIR=/tmp
OUT=gpurun_out/r4_mlds
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/mlds/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_mlds.log 2>&1 || { tail -30 $OUT/gpu_tests_mlds.log; exit 1; }
tail -1 $OUT/gpu_tests_mlds.log
for v in default mlds; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-extras > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
done
timeout -k 10 600 python tools/ab.py 5 default mlds -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -3 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default mlds > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default mlds -- --steps 20 --warmup 5 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -3 $OUT/ab_lamp.txt
echo done
