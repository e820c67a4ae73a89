# Round 4: the later-bounce shade's scattered acc stores (44 % of its exclusive time by the dg1 timing build,
# gpurun_out/r4_sh1) as nontemporal stores (nt), the shade and scatter-shade prefetch (pf) and both (ntpf),
# against the default (sh1 + opaque PCG increment): GPU suite on the default and ntpf, kernel traces of one
# pass alone, interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_nt1
mkdir -p $OUT
for v in default ntpf; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$v.log 2>&1 || { tail -30 $OUT/gpu_tests_$v.log; exit 1; }
  tail -1 $OUT/gpu_tests_$v.log
done
for v in default nt ntpf; do
  LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so
  [ $v = default ] && LIB=$PWD/cuda-raytracer_amd/build/librtamd.so
  RTAMD_LIB=$LIB timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-extras > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  echo "$v ok"
done
timeout -k 10 700 python tools/ab.py 4 default nt pf ntpf -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -5 $OUT/ab_steps20.txt
echo done
