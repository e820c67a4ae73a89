# Round 3: admission control of heavy bounces (pass k starts after pass k-H finished bounce B) vs the shaped stagger
export TMPDIR=/tmp
OUT=gpurun_out/r3_admit
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1100 python tools/ab.py 5 default default@RTAMD_ADMIT_H=4,RTAMD_ADMIT_B=1 default@RTAMD_ADMIT_H=6,RTAMD_ADMIT_B=1 default@RTAMD_ADMIT_H=4,RTAMD_ADMIT_B=0 default@RTAMD_ADMIT_H=8,RTAMD_ADMIT_B=0 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 2 default default@RTAMD_ADMIT_H=6,RTAMD_ADMIT_B=1 default@RTAMD_ADMIT_H=8,RTAMD_ADMIT_B=0 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
echo done
