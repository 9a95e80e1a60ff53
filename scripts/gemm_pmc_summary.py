"""Summarise scripts/gpu/r06_gemm_pmc.sh passes: per kernel family, mean counters per dispatch,
effective clock (GRBM_GUI_ACTIVE / 8 / wall) and derived ratios."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        fam = "edl8" if "gemm_nt8" in name else ("hipblaslt" if "Cijk" in name else None)
        if fam is None:
            continue
        key = (r.get("Dispatch_Id"), r.get("Counter_Name"))
        agg[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur = float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
        if dur > 0:
            agg[fam]["_wall_ns"].append(dur)
for fam, cs in agg.items():
    mean = {k: sum(v) / len(v) for k, v in cs.items()}
    line = [fam]
    for k in sorted(mean):
        line.append(f"{k}={mean[k]:.4g}")
    print(" ".join(line))
    w = mean.get("_wall_ns")
    if w and "GRBM_GUI_ACTIVE" in mean:
        print(f"  clock_GHz={mean['GRBM_GUI_ACTIVE'] / 8 / w:.3f}")
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS"):
            if k in mean:
                print(f"  {k}/WAVE_CYCLES={mean[k] / wc:.3f}")
