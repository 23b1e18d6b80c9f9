"""Per-kernel mean of every counter in rocprofv3 --pmc CSV files (one or more
passes), kernel names shortened.  FETCH_SIZE is reported as measured; on gfx950
double it for wide streaming reads (MI355X_MICROARCH.md)."""
import collections
import csv
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            name = k.split("::")[1].split("(")[0] if "::" in k else k.split("(")[0]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, d in sorted(agg.items()):
        print(name, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})


if __name__ == "__main__":
    main(sys.argv[1:])
