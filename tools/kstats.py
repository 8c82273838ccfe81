"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python tools/kstats.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{len(rows)} kernels, {tot / 1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f}us "
          f"{float(r['Percentage']):5.1f}% {r['Name'][:100]}")
