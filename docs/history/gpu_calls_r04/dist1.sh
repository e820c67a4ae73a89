# Round 4: the torch.distributed path at N = 1 (what every rank of the driver's multi-GPU runs uses):
# passes in flight 16 (default there) / 20, hardware queues 28 (default) / 32, overlapped exchange off --
# interleaved A/B at 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_dist1
mkdir -p $OUT
AB_ARGS="--no-extras --dist" timeout -k 10 900 python tools/ab.py 4 default default@RTAMD_INFLIGHT=20 default@GPU_MAX_HW_QUEUES=32 default@RTAMD_INFLIGHT=20,GPU_MAX_HW_QUEUES=32 default@RTAMD_XCHG_OVERLAP=0 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras > $OUT/nodist.json 2>&1 && tail -1 $OUT/nodist.json | cut -c1-200
echo done
