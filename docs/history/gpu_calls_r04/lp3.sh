# Round 4: PMC issue/lane-utilisation of the default and parallel-leaf (lp12w7) builds; the refactored bench end to end
export TMPDIR=/tmp
OUT=gpurun_out/r4_lp3
mkdir -p $OUT
bash tools/pmc.sh r4_def_is tools/pmc_groups/issue.txt > $OUT/pmc_def.log 2>&1 || { cat $OUT/pmc_def.log; exit 1; }
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/lp12w7/librtamd.so bash tools/pmc.sh r4_lp12_is tools/pmc_groups/issue.txt > $OUT/pmc_lp12.log 2>&1 || { cat $OUT/pmc_lp12.log; exit 1; }
python3 tools/pmc_summary.py r4_def_is > $OUT/issue_def.txt && python3 tools/pmc_summary.py r4_lp12_is > $OUT/issue_lp12.txt || exit 1
grep trace_kernel $OUT/issue_def.txt $OUT/issue_lp12.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_steps20.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['bit_exact_vs_oracle'],r['ms_per_launch'],r.get('heavy'),r.get('tail'))"
timeout -k 10 300 python bench.py --dist --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_dist.json 2> $OUT/bench_dist.err || { tail $OUT/bench_dist.err; exit 1; }
cut -c1-400 $OUT/bench_dist.json
echo done
