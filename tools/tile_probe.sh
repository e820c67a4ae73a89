export TMPDIR=/tmp
O=gpurun_out/tiles1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "--no-sort" "--no-sort --shard tiles" "--no-sort --dist --shard tiles" "--no-sort --steps 13" "--no-sort --tile-share 8" "--scene lamp --no-sort --steps 26" "--scene lamp --no-sort --tile-share 8"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 300 python bench.py --no-cpu-baseline --no-counters $a > $O/b_$n.json 2> $O/b_$n.err || { tail $O/b_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$n.json'));print('$a', d['ms_per_step'], d['value'], d['config']['render_wall_ms'])"
done
