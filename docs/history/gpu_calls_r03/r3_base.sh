export TMPDIR=/tmp
OUT=gpurun_out/r3_base
mkdir -p $OUT
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > $OUT/host.txt
nproc >> $OUT/host.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail $OUT/bench_driver.err; exit 1; }
cat $OUT/bench_driver.json
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
cat $OUT/bench_teapot.json
