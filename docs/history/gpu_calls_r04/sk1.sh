# Round 4: step-kind turns (RT_STEPKIND) and leaf lanes without the child-ref load (RT_KIDS_MASK): parity on two variants, the async ABI tests, then an interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_sk1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -v --timeout 120 --timeout-method thread > $OUT/gpu_async.log 2>&1 || { tail -30 $OUT/gpu_async.log; exit 1; }
tail -1 $OUT/gpu_async.log
for v in sk11 sk11all km1 km2; do
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { tail -30 $OUT/parity_$v.log; exit 1; }
tail -1 $OUT/parity_$v.log
done
timeout -k 10 900 python tools/ab.py 3 default sk11 sk21 sk12 sk11all km1 km2 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -9 $OUT/ab_steps20.txt
echo done
