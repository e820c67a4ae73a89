#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
GPU_MAX_HW_QUEUES=24 timeout -k 10 120 tools/experiments/launch_chain > $O/launch_chain.txt 2>&1 || { cat $O/launch_chain.txt; exit 1; }
cat $O/launch_chain.txt
