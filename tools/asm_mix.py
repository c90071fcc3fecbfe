"""Instruction mix per basic block of one kernel in a device .s file (blocks with > 20 instructions)."""
import sys

path, name = sys.argv[1], sys.argv[2]
s = open(path).read()
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
blocks, cur = [], None
for line in s[a:b].split("\n"):
    t = line.split(";")[0].strip()
    if t.endswith(":"):
        cur = [t, []]
        blocks.append(cur)
    elif cur is not None and t and not t.startswith("."):
        cur[1].append(t.split()[0])
for nm, ins in blocks:
    c = {}
    for i in ins:
        k = ("mfma" if "mfma" in i else "ds" if i.startswith("ds_") else "vmem" if i.startswith(("buffer", "global"))
             else "waitcnt" if i.startswith("s_waitcnt") else "valu" if i.startswith("v_") else "salu" if i.startswith("s_")
             else "other")
        c[k] = c.get(k, 0) + 1
    if len(ins) > 20:
        print(nm, len(ins), c)
