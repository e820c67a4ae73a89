#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
for q in 4 8 24; do
  echo "== GPU_MAX_HW_QUEUES=$q" >> $O/launch_chain_q.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 tools/experiments/launch_chain >> $O/launch_chain_q.txt 2>&1 || { cat $O/launch_chain_q.txt; exit 1; }
done
cat $O/launch_chain_q.txt
