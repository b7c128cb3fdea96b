"""One A/B summary line from a bench JSON line on stdin: ms/step, the main phases and the
per-kernel HIP-event times (libraries with the kernel timers).  usage: ... | python ab_line.py <name>"""
import json
import sys

d = json.loads(sys.stdin.read())
ph = {k: round(v, 4) for k, v in d["phases_ms"].items()
      if k in ("policy", "rollout_select", "rollout_sort", "rollout_finish", "fill_residual")}
km = {k: round(v * 1e3, 1) for k, v in d.get("kernel_ms", {}).items()}
print(sys.argv[1], round(d["ms_per_step"], 4), ph, km, flush=True)
