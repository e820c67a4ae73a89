# Round 3: staggered start on the torch.distributed path (16 in flight): 20-pass and 13-pass rank shares
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger4
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5 --dist" timeout -k 10 800 python tools/ab.py 5 default@RTAMD_STAGGER_US=0 default default@RTAMD_STAGGER_US=1000 > $OUT/ab_20dist.txt 2>&1; tail -4 $OUT/ab_20dist.txt
AB_ARGS="--no-extras --steps 13 --dist" timeout -k 10 800 python tools/ab.py 5 default@RTAMD_STAGGER_US=0 default default@RTAMD_STAGGER_US=1000 > $OUT/ab_13dist.txt 2>&1; tail -4 $OUT/ab_13dist.txt
echo done
