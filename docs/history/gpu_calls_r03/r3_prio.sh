# Round 3: stream priority for the later contexts of a batch (experiment)
export TMPDIR=/tmp
OUT=gpurun_out/r3_prio
mkdir -p $OUT
python3 -c "import ctypes; h=ctypes.CDLL('libamdhip64.so'); lo=ctypes.c_int(); hi=ctypes.c_int(); print('priority range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), lo.value, hi.value)"
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 900 python tools/ab.py 5 default default@RTAMD_PRIO_FROM=10 default@RTAMD_PRIO_FROM=15 default@RTAMD_PRIO_FROM=0 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
echo done
