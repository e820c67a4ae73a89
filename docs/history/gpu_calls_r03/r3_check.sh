# Round 3: quick GPU check of the latest changes (tiles tests incl. the one-rank RCCL exchange, a bench line)
export TMPDIR=/tmp
OUT=gpurun_out/r3_check
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tiles_tests.log 2>&1; rc=$?
tail -3 $OUT/tiles_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_teapot.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['ms_per_launch'],r['exclusive_pass_kernel_ms'],r['frac'],r['traffic_frac'],r['pmc_run']['frac'])"
