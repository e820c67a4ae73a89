# Round 3: passes in flight on the torch.distributed path with the shaped stagger (20-pass rank share)
export TMPDIR=/tmp
OUT=gpurun_out/r3_distq
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5 --dist" timeout -k 10 900 python tools/ab.py 5 default default@RTAMD_INFLIGHT=20 default@RTAMD_INFLIGHT=18 > $OUT/ab_20dist.txt 2>&1; tail -4 $OUT/ab_20dist.txt
echo done
