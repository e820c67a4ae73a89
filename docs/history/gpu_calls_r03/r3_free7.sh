# Round 3: kernel trace of the whole lamp frame with the order-free kernel
export TMPDIR=/tmp
OUT=gpurun_out/r3_free7
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-extras --scene lamp > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/free_launches.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'trace_free' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows]
print(len(rows), 'launches; total', sum(d))
for i in range(0, len(rows), max(1, len(rows) // 60)):
    r = rows[i]
    print(i, round((int(r['Start_Timestamp']) - t0) / 1e6, 1), r['Stream_Id'], round(d[i], 3), r['Kernel_Name'][:45])
big = sorted(range(len(d)), key=lambda i: -d[i])[:15]
print('longest:', [(i, round(d[i], 2)) for i in big])
PY
head -3 $OUT/free_launches.txt
echo done
