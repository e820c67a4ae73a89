"""Interleaved A/B of librtamd.so variants (run on the GPU box after tools/variants.sh here).

    python tools/ab.py ROUNDS name1 name2 ... [-- extra bench args]      (name: variant[@VAR=v,...])
Each round runs bench.py once per variant (RTAMD_LIB points at build_var/<name>), in order, so
device/clock drift hits every variant alike; prints median/min ms_per_step and process ms."""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    rounds, names = int(args[0]), args[1:]
    res = {n: [] for n in names}
    for r in range(rounds):
        for n in names:
            # "name@VAR=v,VAR2=w": library variant `name` (or "default") with extra environment
            base, _, extra_env = n.partition("@")
            lib = os.path.join(REPO, "cuda-raytracer_amd", "build_var", base, "librtamd.so")
            if base == "default":
                lib = os.path.join(REPO, "cuda-raytracer_amd", "build", "librtamd.so")
            env = dict(os.environ, RTAMD_LIB=lib)
            for kv in filter(None, extra_env.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            base_args = os.environ.get("AB_ARGS", "--no-extras").split()
            out = subprocess.run([sys.executable, "bench.py"] + base_args + extra,
                                 cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print("variant %s failed rc=%d: %s" % (n, out.returncode, out.stderr[-2000:]), flush=True)
                sys.exit(1)
            rec = json.loads(out.stdout.strip().splitlines()[-1])
            spans = rec["config"].get("summed_concurrent_spans_per_pass", {})
            res[n].append((rec["ms_per_step"], spans.get("process_ms", 0.0), rec["value"]))
            print("round %d %-12s ms/step %.3f process %.3f Mrays/s %.1f trace/step %s sort/step %s" % (
                r, n, *res[n][-1], spans.get("trace_ms"), spans.get("sort_ms")), flush=True)
    print("summary (median / min ms_per_step, median process ms, median Mrays/s):")
    for n in names:
        ms = [x[0] for x in res[n]]
        pr = [x[1] for x in res[n]]
        va = [x[2] for x in res[n]]
        print("%-12s %.3f / %.3f   %.3f   %.1f" % (n, statistics.median(ms), min(ms), statistics.median(pr),
                                                  statistics.median(va)))


if __name__ == "__main__":
    main()
