"""Per-kernel device time of the non-root switch round (tools/nr_probe.py under
rocprofv3 --kernel-trace), split by the up batch (children's frames) and the
down batch (the parent's results): python tools/nr_prof_split.py <results.db>"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, grid_x from kernels where name like '%k_nr%' "
                 "or name like '%k_egress<2, true, true>%' order by start")
d = defaultdict(list)
cur = None
for name, s, e, g in rows:
    short = name.split("::")[1].split("(")[0]
    if "k_nr_claim" in name:
        cur = "up" if g >= 131072 else "down"
    d[(cur, short)].append((e - s) / 1000)
for k, v in sorted(d.items()):
    print(f"{k[0]:5s} {k[1]:26s} {len(v):3d} launches  {sum(v) / len(v):7.2f} us")
