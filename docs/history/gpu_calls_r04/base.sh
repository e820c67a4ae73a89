# Round 4 baseline at HEAD: GPU suite, then the driver's bench command
export TMPDIR=/tmp
OUT=gpurun_out/r4_base
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_driver_style.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['bit_exact_vs_oracle'],r['ms_per_launch'])"
echo done
