"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE csv passes per kernel (KB per dispatch).
usage: python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<dir>/pmc_summary.json"""
import csv
import json
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
out = {}
for f, c in ((f"{src}/pmc_fetch_counter_collection.csv", "FETCH_SIZE"), (f"{src}/pmc_write_counter_collection.csv", "WRITE_SIZE")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "ompl_amd" not in n:
            continue
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = n[: n.find("(")] if "(" in n else n
        out.setdefault(n, {}).setdefault(c, []).append(float(r["Counter_Value"]))
summ = {k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} for k, d in out.items()}
json.dump({"units": "KB per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE, separate --pmc passes); on gfx950 "
           "FETCH_SIZE reads 1/2 of wide coalesced streaming bytes (MI355X_MICROARCH.md, HBM): double it for bytes",
           "per_kernel_mean": summ}, open(dst, "w"), indent=1)
print(json.dumps(summ, indent=1))
