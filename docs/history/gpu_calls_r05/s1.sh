#!/bin/bash
# r05: scalar-load path for uniform trace records: parity, exclusive launch A/B, 20-step A/B.
export TMPDIR=/tmp
OUT=gpurun_out/r5_s1; mkdir -p $OUT
echo "== parity $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
echo "== launch ab $(date +%T)"
timeout -k 10 600 python tools/launch_ab.py 3 sr0 dup0 default sr2 > $OUT/launch_ab.txt 2>&1 || { tail $OUT/launch_ab.txt; exit 1; }
tail -5 $OUT/launch_ab.txt
echo "== ab20 $(date +%T)"
timeout -k 10 900 python tools/ab.py 3 sr0 dup0 default sr2 -- --steps 20 --warmup 5 > $OUT/ab20.txt 2>&1 || { tail $OUT/ab20.txt; exit 1; }
tail -5 $OUT/ab20.txt
