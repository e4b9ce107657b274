"""Per-kernel mean of every counter in rocprofv3 --pmc csv files (summed over a dispatch's
instances), for the culled-walk kernels and the other ompl_amd kernels.
usage: python tools/pmc_csv_summary.py <dir with *counter_collection.csv> <out.json> [note]"""
import csv
import glob
import json
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
note = sys.argv[3] if len(sys.argv) > 3 else ""
acc = {}
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "ompl_amd" not in n:
            continue
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = n[: n.find("(")] if "(" in n else n
        key = (n, r.get("Dispatch_Id", r.get("Correlation_Id", "")), r["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (n, _, c), v in per.items():
        acc.setdefault(n, {}).setdefault(c, []).append(v)
summ = {k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} for k, d in acc.items()}
json.dump({"units": "per dispatch, summed over the dispatch's instances (rocprofv3 --pmc)", "note": note,
           "per_kernel_mean": summ}, open(dst, "w"), indent=1)
print(json.dumps(summ, indent=1))
