"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv: name, calls, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    print(f"{float(r['AverageNs']) / 1e3:10.1f} us  x{r['Calls']:>4}  {r['Name'][:110]}")
