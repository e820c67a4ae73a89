# Round 4: where the later-bounce shade's time goes -- diagnostic timing builds (wrong images on purpose:
# dg1 no acc store, dg2 no environment lookup, dg3 no triangle-normal load) against the default, one
# teapot pass alone on the chip under the kernel trace
export TMPDIR=/tmp
OUT=gpurun_out/r4_dg1
mkdir -p $OUT
for v in default dg1 dg2 dg3; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-extras > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  echo "$v ok"
done
echo done
