# Round 3: coherence-ordered trace A/B + parity (GPU box)
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab2
mkdir -p $OUT
RTAMD_COHERENT=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_coherent.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests_coherent.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 700 python tools/ab.py 4 default default@RTAMD_COHERENT=1 coh16k coh32k recmad > $OUT/ab_frame.txt 2>&1; tail -7 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default default@RTAMD_COHERENT=1 coh16k > $OUT/ab_lamp.txt 2>&1; tail -5 $OUT/ab_lamp.txt
timeout -k 10 300 python bench.py --tile-share 8 --no-cpu-baseline --no-counters > $OUT/tile_share8_sorton.json 2> $OUT/tile_share8_sorton.err || { tail $OUT/tile_share8_sorton.err; exit 1; }
cat $OUT/tile_share8_sorton.json | cut -c1-400
