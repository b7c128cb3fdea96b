"""Print the rocprofv3 kernel stats table (and optionally the last step's kernel timeline)."""
import csv
import sys

d = sys.argv[1]
for r in list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:8.1f}us {float(r['Percentage']):6.2f}%")
if len(sys.argv) > 3:
    rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[3])
    t0 = int(rows[-n]["Start_Timestamp"])
    for r in rows[-n:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {r['Kernel_Name'][:90]}")
