# Round 3 measurement at HEAD (GPU box): part A of tools/round_measure.sh + the end-of-batch ramp trace
TAG=$1
export TMPDIR=/tmp
bash tools/round_measure.sh $TAG A || exit 1
OUT=gpurun_out/$TAG
echo "== ramp trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_ramp13 -o run --output-format csv -- python3 bench.py --steps 13 --dist --no-extras > $OUT/prof_ramp13.log 2>&1 || { tail $OUT/prof_ramp13.log; exit 1; }
timeout -k 10 300 python bench.py --steps 13 --dist --no-extras > $OUT/ramp13.json 2> $OUT/ramp13.err || { tail $OUT/ramp13.err; exit 1; }
cut -c1-200 $OUT/ramp13.json
echo done-all
