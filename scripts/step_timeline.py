"""Timeline of one graph-replayed step from a rocprofv3 kernel trace: the kernels between the
k-th last and the (k-1)-th last k_fc launch (a step starts with the policy), start offsets and
durations in us, the queue each ran on, so concurrent branches show as overlapping intervals.
usage: python scripts/step_timeline.py <prof_dir> [k=2]"""
import csv
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fc<" in r["Kernel_Name"]]
i0, i1 = starts[-k], starts[-k + 1] if k > 1 else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
end = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("spai::", "").split("(")[0][:60]
    q = r.get("Queue_Id", r.get("Stream_Id", ""))
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3s}  {name}")
print(f"step span {(end - t0) / 1e3:.1f} us")
