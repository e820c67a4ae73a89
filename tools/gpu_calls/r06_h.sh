#!/bin/bash
# Round 6, call H: device-clock pass timelines (RTAMD_TIMELINE, the bench's event-timed leg) of a 13-pass share
# through torch.distributed and of the 20-pass driver batch.
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
RTAMD_TIMELINE=1 timeout -k 10 300 python bench.py --steps 13 --warmup 2 --dist --no-cpu-baseline --no-counters > $O/b13.json 2> $O/b13.err || { tail $O/b13.err; exit 1; }
python3 tools/pass_timeline.py $O/b13.err 13 | tee $O/timeline13.txt
RTAMD_TIMELINE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $O/b20.json 2> $O/b20.err || { tail $O/b20.err; exit 1; }
python3 tools/pass_timeline.py $O/b20.err 20 | tee $O/timeline20.txt
