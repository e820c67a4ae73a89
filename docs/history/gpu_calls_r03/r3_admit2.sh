# Round 3: admission control in the full frame's steady state (after the staggered first wave)
export TMPDIR=/tmp
OUT=gpurun_out/r3_admit2
mkdir -p $OUT
AB_ARGS="--no-extras" timeout -k 10 1100 python tools/ab.py 4 default default@RTAMD_ADMIT_H=6,RTAMD_ADMIT_B=1 default@RTAMD_ADMIT_H=10,RTAMD_ADMIT_B=1 default@RTAMD_ADMIT_H=10,RTAMD_ADMIT_B=1,RTAMD_ADMIT_STEADY=1 default@RTAMD_ADMIT_H=14,RTAMD_ADMIT_B=1,RTAMD_ADMIT_STEADY=1 > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
echo done
