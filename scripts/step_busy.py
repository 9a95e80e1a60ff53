"""GPU-busy vs wall time of the last optimizer-delimited steps in a rocprofv3 kernel trace
(launch-bound check), and the top kernels per step.  usage: step_busy.py trace.csv [opt_substr]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "clip_finalize"   # one launch per optimizer step (AdamW or SGD)
opt = [r for r in rows if key in r["Kernel_Name"]]
n = min(3, len(opt) - 1)
a, b = int(opt[-1 - n]["End_Timestamp"]), int(opt[-1]["End_Timestamp"])
win = [r for r in rows if a < int(r["Start_Timestamp"]) <= b]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
print(f"{n} steps: wall {(b - a) / 1e6 / n:.2f} ms/step, kernel busy {busy / 1e6 / n:.2f} ms/step, "
      f"{len(win) / n:.0f} kernels/step")
c = collections.Counter()
for r in win:
    c[r["Kernel_Name"][:70]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in c.most_common(14):
    print(f"  {v / n / 1e3:8.1f} us/step  {k}")
