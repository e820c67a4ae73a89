# Round 3: shade grid (blocks per CU) with the histogram counted in the shade kernel
export TMPDIR=/tmp
OUT=gpurun_out/r3_bpc
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 800 python tools/ab.py 4 default bpc4 bpc16 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 default bpc4 bpc16 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
echo done
