#!/bin/bash
# r05 closing measurement, part B: PMC records of the other configs, then their bench lines, the strong-scaling
# probes (torch.distributed path and the in-library path) and REPORT.pdf Table 1.   usage: fin_b.sh TAG
export TMPDIR=/tmp
TAG=${1:-r5fin}
bash tools/pmc_configs.sh $TAG > gpurun_out/${TAG}_pmc_configs.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_configs.log; exit 1; }
tail -2 gpurun_out/${TAG}_pmc_configs.log
bash tools/round_measure.sh $TAG B || exit 1
timeout -k 10 600 python tools/share_probe.py 13 26 > gpurun_out/$TAG/share_probe.txt 2>&1 || { tail gpurun_out/$TAG/share_probe.txt; exit 1; }
cat gpurun_out/$TAG/share_probe.txt
