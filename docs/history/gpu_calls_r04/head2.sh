# Round 4: last check at HEAD (host-side timeline diagnostic added after the closing measurement; kernels
# unchanged): GPU suite, smoke, the driver-style bench line
export TMPDIR=/tmp
OUT=gpurun_out/r4_head2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err || { tail -20 $OUT/bench_steps20.err; exit 1; }
cut -c1-300 $OUT/bench_steps20.json
echo done
