# Round 3: the staggered start on the other configs (short frames), against no stagger and admission (H=4, B=0)
export TMPDIR=/tmp
OUT=gpurun_out/r3_cfgstag
mkdir -p $OUT
for sc in cornell_plus spheres lamp; do
AB_ARGS="--no-extras --scene $sc" timeout -k 10 600 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default default@RTAMD_ADMIT_H=4 > $OUT/ab_$sc.txt 2>&1; tail -4 $OUT/ab_$sc.txt
done
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default default@RTAMD_ADMIT_H=4 > $OUT/ab_teapot.txt 2>&1; tail -4 $OUT/ab_teapot.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 600 python tools/ab.py 4 default default@RTAMD_ADMIT_H=4 default@RTAMD_ADMIT_H=6 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
echo done
