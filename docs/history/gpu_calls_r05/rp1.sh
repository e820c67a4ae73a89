#!/bin/bash
# r05: the fused replay (sort_scatter_shade_kernel, bounce 0 of big scenes, every bounce of small ones) at 7 / 8 waves
export TMPDIR=/tmp
OUT=gpurun_out/r5_rp1; mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/rp8/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 900 python tools/ab.py 4 default rp7 rp8 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -4 $OUT/ab20.txt
timeout -k 10 900 python tools/ab.py 2 default rp7 rp8 -- > $OUT/abfull.txt 2>&1 || { tail $OUT/abfull.txt; exit 1; }
tail -4 $OUT/abfull.txt
timeout -k 10 900 python tools/ab.py 2 default rp7 rp8 -- --scene cornell_plus > $OUT/abcp.txt 2>&1 || { tail $OUT/abcp.txt; exit 1; }
tail -4 $OUT/abcp.txt
timeout -k 10 900 python tools/ab.py 2 default rp7 rp8 -- --scene spheres --steps 20 --warmup 3 > $OUT/absp.txt 2>&1 || { tail $OUT/absp.txt; exit 1; }
tail -4 $OUT/absp.txt
