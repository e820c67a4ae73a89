# Round 4: nontemporal hints on the trace kernel's own streams (hit stores, ray loads: trnt) and on
# accumulation's reads (acnt) against the default; parity of trnt, interleaved A/B at 20 steps and full frame
export TMPDIR=/tmp
OUT=gpurun_out/r4_nt2
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/trnt/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity_trnt.log 2>&1 || { tail -30 $OUT/parity_trnt.log; exit 1; }
tail -1 $OUT/parity_trnt.log
timeout -k 10 600 python tools/ab.py 4 default trnt acnt -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -4 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 2 default trnt acnt > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -4 $OUT/ab_frame.txt
echo done
