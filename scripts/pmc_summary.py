"""Average per-dispatch PMC counters per kernel from scripts/gpu.sh pmc:* outputs.

--first NAME=N[,NAME=N...]: keep only the first N dispatches (in dispatch order,
per counter pass) of kernels whose short name contains NAME -- e.g. the
warmup + timed launches of bench.py, before its smaller-N legs run."""
import collections
import csv
import glob
import sys

first = {}
if "--first" in sys.argv:
    for kv in sys.argv[sys.argv.index("--first") + 1].split(","):
        name, n = kv.split("=")
        first[name] = int(n)

d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/counters_p*.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void gvdb::(anonymous namespace)::", "").removeprefix("void ")[:40]
        d[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, cs in d.items():
    lim = next((n for name, n in first.items() if name in k), None)
    if lim is None:
        continue
    for c, v in cs.items():
        keep = sorted({di for di, _, _ in v})[:lim]
        cs[c] = [x for x in v if x[0] in set(keep)]
for k, cs in d.items():
    if len(sys.argv) > 2 and not sys.argv[2].startswith("--") and sys.argv[2] not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        per, dur = collections.defaultdict(float), {}
        for di, val, du in v:
            per[di] += val
            dur[di] = du
        vals = list(per.values())
        print(f"   {c:32s} {sum(vals) / len(vals):14.4g}  n={len(vals)} dur_us={sum(dur.values()) / len(dur) / 1e3:.1f}")

# --json <path>: the per-kernel averages in the profiles/ JSON layout used by bench.py's pmc_traffic
if "--json" in sys.argv:
    import json

    outp = sys.argv[sys.argv.index("--json") + 1]
    res = {"source": f"scripts/pmc_summary.py over {sys.argv[1]} (rocprofv3 --pmc, one counter set per run)"
                     + (f"; first dispatches only: {first}" if first else ""),
           "fetch_size_unit": "KiB; gfx950 FETCH_SIZE counts half of the bytes of a 16-B/lane streaming read "
                              "(MI355X_MICROARCH.md, HBM) -> hbm_read_bytes = 2 * 1024 * FETCH_SIZE",
           "kernels": {}}
    for k, cs in d.items():
        e = {}
        for c, v in cs.items():
            per = collections.defaultdict(float)
            for di, val, du in v:
                per[di] += val
            e[c] = sum(per.values()) / len(per)
            e["dispatches"] = len(per)
            e["avg_dur_us"] = sum(du for _, _, du in v) / len(v) / 1e3
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes_per_launch"] = 2 * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes_per_launch"] = 1024 * e["WRITE_SIZE"]
        res["kernels"][k] = e
    with open(outp, "w") as f:
        json.dump(res, f, indent=1)
