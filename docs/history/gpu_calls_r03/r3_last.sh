# Round 3 last check at HEAD (clean build): smoke, then the driver's own bench command
export TMPDIR=/tmp
OUT=gpurun_out/r3_last
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_driver_style.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['bit_exact_vs_oracle'],r['ms_per_launch'],r['pmc_run']['ms_per_launch'])"
echo done
