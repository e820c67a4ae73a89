"""Summary of the device-clock pass timeline that librtamd prints with RTAMD_TIMELINE=1 (one line per
pass of an event-timed run: "timeline pass k: <bounce-0 start> <bounce-1 start> <bounce-2 start> | <end>",
ms from the run's first trace start).  Takes the last run of BATCH passes in the file.

    python tools/pass_timeline.py bench.err [BATCH=20]

Prints each pass's heavy phase (bounce 0 start -> bounce 2 start) and tail phase (bounce 2 start -> end),
and the batch's tail-only phase: from the last pass's bounce-2 start (no heavy bounce left to run) to the
end of the batch."""
import re
import sys


def main():
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    runs, cur = [], []
    for line in open(sys.argv[1]):
        m = re.match(r"timeline pass (\d+): ([\d.]+) ([\d.]+) ([\d.]+) \| ([\d.]+)", line)
        if not m:
            continue
        k = int(m.group(1))
        if k == 0 and cur:
            runs.append(cur)
            cur = []
        cur.append(tuple(float(m.group(i)) for i in range(2, 6)))
    if cur:
        runs.append(cur)
    runs = [r for r in runs if len(r) == batch]
    if not runs:
        sys.exit("no run of %d passes" % batch)
    r = runs[-1]
    end = max(p[3] for p in r)
    last_heavy = max(p[2] for p in r)
    print("%4s %8s %8s %8s %8s %8s %8s" % ("pass", "start", "b1", "b2", "end", "heavy", "tail"))
    for k, (b0, b1, b2, e) in enumerate(r):
        print("%4d %8.2f %8.2f %8.2f %8.2f %8.2f %8.2f" % (k, b0, b1, b2, e, b2 - b0, e - b2))
    print("batch %.2f ms; heavy bounces of every pass done by %.2f ms; tail-only phase %.2f ms (%.1f %%); "
          "mean tail phase %.2f ms" % (end, last_heavy, end - last_heavy, 100 * (end - last_heavy) / end,
                                        sum(p[3] - p[2] for p in r) / len(r)))


if __name__ == "__main__":
    main()
