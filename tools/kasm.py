"""Extract one kernel's instruction stream from a hipcc -S dump (labels renumbered) for codegen diffs.
usage: python tools/kasm.py dump.s NAME_SUBSTRING > out.txt"""
import re
import sys

s = open(sys.argv[1]).read().splitlines()
key = sys.argv[2]
start = next(i for i, l in enumerate(s) if re.match(r"^\S+:\s*;\s*@", l) and key in l.split(":")[0])
out = []
for l in s[start + 1:]:
    if l.startswith(".Lfunc_end"):
        break
    l = l.split(";")[0].rstrip()
    if not l.strip() or l.strip().startswith("."):
        continue
    out.append(re.sub(r"\.LBB\d+_", ".LBB_", l))
print("\n".join(out))
