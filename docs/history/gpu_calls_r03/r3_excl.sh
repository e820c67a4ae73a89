# Round 3: the new trace-rays case (rays leaving the scene), then the exclusive trace launch of pass 0
# measured three times in separate processes (the closing line's 0.747 ms vs the profiler's 0.641)
export TMPDIR=/tmp
OUT=gpurun_out/r3_excl
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace_rays.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/trace_rays.log 2>&1 || { tail -20 $OUT/trace_rays.log; exit 1; }
tail -1 $OUT/trace_rays.log
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { tail $OUT/bench_$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$k.json'));r=d['roofline'];print('$k',d['value'],d['ms_per_step'],r['ms_per_launch'],r['exclusive_pass_kernel_ms'],r['pmc_run']['ms_per_launch'])"
done
echo done
