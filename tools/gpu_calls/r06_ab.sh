#!/bin/bash
# Round 6, call AB: PMC records of the timed regime itself (the driver's 20 concurrent passes, --steps 20 --warmup 0),
# wave time / instruction counts and fabric traffic, one rocprofv3 --pmc run per counter group.
export TMPDIR=/tmp
O=gpurun_out/r06ab; mkdir -p $O
bash tools/pmc.sh r06t20_st tools/pmc_groups/stall.txt --steps 20 > $O/stall.log 2>&1 || { tail $O/stall.log; exit 1; }
bash tools/pmc.sh r06t20_tf tools/pmc_groups/traffic.txt --steps 20 > $O/traffic.log 2>&1 || { tail $O/traffic.log; exit 1; }
cat $O/stall.log $O/traffic.log
