#!/bin/bash
# Round 6, call AA: does instruction fetch stall the trace kernel?  I-cache counters with one pass alone and with the
# driver's 20 concurrent passes (each pass a single rocprofv3 --pmc run; no tracing domains).
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST_ANY\|SQ_INSTS_[A-Z]*" $O/avail.txt | sort -u > $O/avail_icache.txt || true
cat $O/avail_icache.txt
C=SQC_ICACHE_HITS,SQC_ICACHE_MISSES,SQ_IFETCH,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES
timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/pmc_r06aa1_1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-extras > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_r06aa20_1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 0 --no-extras > $O/p20.log 2>&1 || { tail -5 $O/p20.log; exit 1; }
python3 tools/icache_summary.py r06aa1 r06aa20 | tee $O/icache.txt | head -30
