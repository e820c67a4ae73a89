#!/bin/bash
# Round 6, call C: the C++ ABI host (one-shot renders, then a persistent renderer's runs), and the PMC stall
# split of the dropped two-level trace (build_var/trace2, every bounce from 1) beside the default kernel.
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
env -u GPU_MAX_HW_QUEUES timeout -k 10 300 tests/native/build/abi_host assets/teapot.scene assets 1920 1080 2048 16 20 2 /tmp/p0.bin > $O/abi_host.txt 2>&1 || { cat $O/abi_host.txt; exit 1; }
cat $O/abi_host.txt
bash tools/pmc.sh r06c_st0 tools/pmc_groups/stall.txt > $O/pmc_st0.log 2>&1 || { cat $O/pmc_st0.log; exit 1; }
python3 tools/stall_summary.py r06c_st0 > $O/pmc_stall_default.txt || exit 1
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/trace2/librtamd.so RTAMD_TRACE2=1 bash tools/pmc.sh r06c_st2 tools/pmc_groups/stall.txt > $O/pmc_st2.log 2>&1 || { cat $O/pmc_st2.log; exit 1; }
python3 tools/stall_summary.py r06c_st2 > $O/pmc_stall_trace2.txt || exit 1
head -20 $O/pmc_stall_default.txt; head -20 $O/pmc_stall_trace2.txt
