#!/bin/bash
# r05: is the 20-in-flight cliff torch's bundled HIP runtime (the dist path runs on it)?
export TMPDIR=/tmp
OUT=gpurun_out/r5_q3; mkdir -p $OUT
run() { name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name',d['ms_per_step'])"
}
run plain20 RTAMD_INFLIGHT=20
run torch20 RTAMD_INFLIGHT=20 RTAMD_TORCH_FIRST=1
run torch19 RTAMD_INFLIGHT=19 RTAMD_TORCH_FIRST=1
run torch20_q32 RTAMD_INFLIGHT=20 RTAMD_TORCH_FIRST=1 RTAMD_HW_QUEUES=32
run torch20_q8 RTAMD_INFLIGHT=20 RTAMD_TORCH_FIRST=1 RTAMD_HW_QUEUES=8
python3 -c "import torch;print(torch.__version__, torch.version.hip)"
