# Round 4: nontemporal environment texel loads (envnt), and re-tuning after the cheaper shade: 16 passes
# in flight, shade grid 4 / 16 blocks per CU (default 8); parity of envnt, interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_env1
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/envnt/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity_envnt.log 2>&1 || { tail -30 $OUT/parity_envnt.log; exit 1; }
tail -1 $OUT/parity_envnt.log
timeout -k 10 800 python tools/ab.py 4 default envnt default@RTAMD_INFLIGHT=16 bpc4 bpc16 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
