"""Count VALU instructions per kernel in an llvm-objdump listing (tools/microbench/ec_isa_count.hip)."""
import re, sys, collections
txt = open(sys.argv[1]).read()
funcs = re.split(r"\n(?=[0-9a-f]+ <)", txt)
for f in funcs:
    m = re.match(r"[0-9a-f]+ <(\S+)>:", f)
    if not m or not any(k in m.group(1) for k in sys.argv[2:]): continue
    ops = collections.Counter()
    for line in f.split("\n")[1:]:
        t = line.strip().split()
        if not t or t[0].startswith("s_") : 
            if t: ops["SALU/"+t[0]] += 1
            continue
        ops[t[0]] += 1
    v = sum(c for o, c in ops.items() if o.startswith("v_"))
    print(m.group(1)[:40], "VALU", v, "total", sum(ops.values()))
    if len(sys.argv) > 2 and "-v" in sys.argv: print(ops.most_common(25))
