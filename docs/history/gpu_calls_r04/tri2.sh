# Round 4: two triangles per leaf step in the later-bounce trace (t2; t2w7 with a 7-wave minimum):
# parity of t2, interleaved A/B at 20 steps, full frame and lamp
export TMPDIR=/tmp
OUT=gpurun_out/r4_tri2
mkdir -p $OUT
for v in t2 t2w7; do
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { tail -30 $OUT/parity_$v.log; exit 1; }
tail -1 $OUT/parity_$v.log
done
timeout -k 10 600 python tools/ab.py 4 default t2 t2w7 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -4 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default t2 t2w7 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 default t2 t2w7 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -4 $OUT/ab_lamp.txt
echo done
