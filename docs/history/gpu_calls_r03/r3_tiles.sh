# Round 3: pixel tiles with the reorder on (GPU box)
export TMPDIR=/tmp
OUT=gpurun_out/r3_tiles
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tiles_tests.log 2>&1; rc=$?
tail -30 $OUT/tiles_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/rccl_same_gpu_probe.py 2 > $OUT/rccl_same_gpu.log 2>&1; echo "rccl probe rc=$?"; tail -20 $OUT/rccl_same_gpu.log
timeout -k 10 300 python bench.py --tile-share 8 --no-cpu-baseline > $OUT/tile_share8_sorton.json 2> $OUT/tile_share8_sorton.err || { tail $OUT/tile_share8_sorton.err; exit 1; }
cat $OUT/tile_share8_sorton.json
timeout -k 10 300 python bench.py --tile-share 8 --no-sort --no-cpu-baseline > $OUT/tile_share8_sortoff.json 2> $OUT/tile_share8_sortoff.err || { tail $OUT/tile_share8_sortoff.err; exit 1; }
cat $OUT/tile_share8_sortoff.json
RTAMD_TSTAGGER=0 timeout -k 10 300 python bench.py --tile-share 8 --no-cpu-baseline --no-counters > $OUT/tile_share8_sorton_nostagger.json 2> $OUT/tile_share8_sorton_nostagger.err || { tail $OUT/tile_share8_sorton_nostagger.err; exit 1; }
cat $OUT/tile_share8_sorton_nostagger.json
echo "== A/B mtflat"
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 default mtflat popflat popmt > $OUT/ab_mtflat.txt 2>&1; tail -6 $OUT/ab_mtflat.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 600 python tools/ab.py 3 default mtflat popflat popmt > $OUT/ab_mtflat20.txt 2>&1; tail -6 $OUT/ab_mtflat20.txt
