#!/bin/bash
# r05: LLVM AMDGPU machine-scheduler strategies for the whole library (max-ilp, max-memory-clause, iterative-ilp)
export TMPDIR=/tmp
OUT=gpurun_out/r5_ss1; mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/smem/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity_smem.log 2>&1 || { tail -30 $OUT/parity_smem.log; exit 1; }
tail -1 $OUT/parity_smem.log
timeout -k 10 600 python tools/launch_ab.py 3 default silp smem sitil > $OUT/launch.txt 2>&1 || { tail $OUT/launch.txt; exit 1; }
tail -5 $OUT/launch.txt
timeout -k 10 1000 python tools/ab.py 3 default silp smem sitil -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -5 $OUT/ab20.txt
