# Round 4: overlapped slice exchange — RCCL dist tests, parity, then the 13-pass rank share through the dist path, overlap off/on (A/B)
export TMPDIR=/tmp
OUT=gpurun_out/r4_xo1
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_rccl.py tests/test_gpu_parity.py tests/test_gpu_bench_contract.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 900 python tools/ab.py 4 default@RTAMD_XCHG_OVERLAP=0 default -- --dist --steps 13 --warmup 3 > $OUT/ab_share13.txt 2>&1 || { tail -20 $OUT/ab_share13.txt; exit 1; }
tail -3 $OUT/ab_share13.txt
echo done
