# Round 4: the later-bounce shade's memory round trips -- kernel traces of one teapot pass alone for the
# base (HEAD before the shade change), two diagnostic timing builds (wrong images on purpose: dg1 no acc store, dg2 no environment
# lookup) and sh1 (ray id with the state loads; material index + surface record in one trip; whole-record
# loads) sh2 (sh1 + the shade kernel's next round prefetched), ss2 (sh1 + the fused scatter-shade's next round prefetched), then their parity and an interleaved A/B po (sh1 + the primary ray PCG increment opaque: no bounce-0 trace spills)
export TMPDIR=/tmp
OUT=gpurun_out/r4_sh1
mkdir -p $OUT
for v in base dg1 dg2 sh1 sh2 ss2 po; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-extras > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  echo "$v ok"
done
for v in sh1; do
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$v.log 2>&1 || { tail -30 $OUT/gpu_tests_$v.log; exit 1; }
tail -1 $OUT/gpu_tests_$v.log
done
timeout -k 10 600 python tools/ab.py 3 base sh1 sh2 ss2 po -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
