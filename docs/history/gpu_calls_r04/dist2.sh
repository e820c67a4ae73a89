# Round 4: passes in flight on the torch.distributed path at N = 1: 12 / 14 / 16 (default) / 18 / 19 --
# interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_dist2
mkdir -p $OUT
AB_ARGS="--no-extras --dist" timeout -k 10 900 python tools/ab.py 3 default@RTAMD_INFLIGHT=12 default@RTAMD_INFLIGHT=14 default default@RTAMD_INFLIGHT=18 default@RTAMD_INFLIGHT=19 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
echo done
