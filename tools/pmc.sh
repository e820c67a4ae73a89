#!/bin/bash
# PMC counter passes over a short bench run (run on the GPU box).  One rocprofv3 invocation per
# counter group (no tracing domains mixed in).  Stops at the first crash/timeout exit status.
# usage: tools/pmc.sh TAG [extra bench args]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-counters $*"
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $GROUP -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $BENCH > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc: $GROUP"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
GRBM_GUI_ACTIVE
GROUPS
