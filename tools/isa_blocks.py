"""Per-basic-block instruction counts of a kernel in a hipcc -S listing: the
largest blocks of a microbenchmark kernel are its loop bodies.
usage: isa_blocks.py file.s <kernel-substring> [min_instructions]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split("\n")
want, floor = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 50
inside, blk, cur = False, None, collections.Counter()
out = []
for line in txt:
    if re.match(r"^_Z\S*:", line):
        if inside and blk is not None:
            out.append((blk, cur))
        inside = want in line.split(":")[0]
        blk, cur = "entry", collections.Counter()
        continue
    if not inside:
        continue
    m = re.match(r"^(\.LBB\S+):", line)
    if m:
        out.append((blk, cur))
        blk, cur = m.group(1), collections.Counter()
        continue
    t = line.strip()
    if not t or t.startswith((".", ";")):
        continue
    op = t.split()[0]
    cur[op] += 1
    if op == "s_endpgm":  # the function may go on (loops placed after an early exit)
        out.append((blk, cur))
        blk, cur = blk + "+", collections.Counter()
if inside:
    out.append((blk, cur))
for name, c in out:
    v = sum(n for o, n in c.items() if o.startswith("v_"))
    if v >= floor:
        top = ", ".join("%s %d" % oc for oc in c.most_common(6))
        print("%-12s VALU %5d  total %5d  | %s" % (name, v, sum(c.values()), top))
