# Round 4: GPU suite after moving the multi-device abort protocol into mgpu_protocol.h
export TMPDIR=/tmp
OUT=gpurun_out/r4_proto
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo done
