"""Summarise a rocprofv3 --pmc SQ-counter pass (tools/sq_counters.sh) per kernel (mean per dispatch).
usage: python tools/sq_summary.py gpurun_out/<dir>/pmc_sq_counter_collection.csv profiles/<dir>/sq_summary.json"""
import csv
import json
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
acc = {}
for r in csv.DictReader(open(src)):
    n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    n = n[: n.find("(")] if "(" in n else n
    key = (n, r.get("Dispatch_Id", ""))
    acc.setdefault(n, {}).setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
    acc[n][r["Counter_Name"]][key] += float(r["Counter_Value"])  # summed over SQ instances
summ = {k: {c: round(sum(v.values()) / len(v), 1) for c, v in sorted(d.items())} for k, d in acc.items()}
json.dump({"units": "per dispatch, summed over the dispatch's SQ instances (rocprofv3 --pmc, one pass: "
           "tools/sq_counters.sh)", "per_kernel_mean": summ}, open(dst, "w"), indent=1)
for k, v in summ.items():
    if "group" in k:
        print(k, json.dumps(v))
        if v.get("SQ_WAVE_CYCLES"):
            print("issue-busy", v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"], "wait", v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"])
