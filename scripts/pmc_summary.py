"""Average per-dispatch PMC counters per kernel from gpu_pmc*.sh outputs."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/counters_p*.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void gvdb::(anonymous namespace)::", "")[:40]
        d[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, cs in d.items():
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        per, dur = collections.defaultdict(float), {}
        for di, val, du in v:
            per[di] += val
            dur[di] = du
        vals = list(per.values())
        print(f"   {c:32s} {sum(vals) / len(vals):14.4g}  n={len(vals)} dur_us={sum(dur.values()) / len(dur) / 1e3:.1f}")
