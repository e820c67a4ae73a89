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
  timeout -k 10 240 rocprofv3 --pmc $GROUP -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $BENCH > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc: $GROUP"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE GRBM_TA_BUSY
GROUPS
