# Round 3: trace grid share with the shaped stagger (10 / 15 / 20 % of the resident workgroups per pass)
export TMPDIR=/tmp
OUT=gpurun_out/r3_occ
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 900 python tools/ab.py 5 default occ10 occ20 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 default occ10 occ20 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
echo done
