#!/bin/bash
# r05 baseline at HEAD: GPU tests, driver-style bench, 13-pass share through dist path.
export TMPDIR=/tmp
OUT=gpurun_out/r5_base; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b20_$i.json 2> $OUT/b20_$i.err || { tail $OUT/b20_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b20_$i.json'));print('b20',d['ms_per_step'],d['value'])"
timeout -k 10 300 python bench.py --steps 13 --dist --no-extras > $OUT/s13_$i.json 2> $OUT/s13_$i.err || { tail $OUT/s13_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/s13_$i.json'));print('s13',d['ms_per_step'],d['value'])"
done
