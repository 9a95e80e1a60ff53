"""Summarise the rocprofv3 --pmc passes of scripts/gpu/pmc.sh into one row per (kernel, grid).

Passes: p1 SQ instruction / busy counters, p2 SQ stall counters, p3 FETCH_SIZE, p4 WRITE_SIZE (each
with GRBM_GUI_ACTIVE where it fits).  Per row: calls, ms per call, HBM read / write GB per call and
GB/s, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA-busy share of the busy cycles,
instructions per wave (MFMA, VALU, LDS), LDS bank conflicts per LDS instruction, and the share of
wave cycles spent waiting (any / on LDS) and issuing VALU / MFMA (SQ quad-cycle counters,
MI355X_MICROARCH.md 'Per-instruction cycle constants').
usage: pmc_summarize.py <dir with p1/ .. p4/> [kernel-name substring]"""
import collections
import csv
import os
import sys


def load(path):
    per = collections.defaultdict(dict)   # dispatch id -> {counter: value, ...}
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        d = per[r["Dispatch_Id"]]
        nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        d["name"] = nm.split("(")[0][:70]
        d["ours"] = "(anonymous namespace)::" in r["Kernel_Name"]
        d["grid"] = r["Grid_Size"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def _csv(root, p):
    d = os.path.join(root, p)
    for dirpath, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(dirpath, f)
    return os.path.join(d, "k_counter_collection.csv")


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else None
    passes = [load(_csv(root, p)) for p in ("p1", "p2", "p3", "p4")]
    keyed = [collections.defaultdict(list) for _ in passes]
    for i, per in enumerate(passes):
        for d in per.values():
            keyed[i][(d["name"], d["grid"])].append(d)

    def tot(i, key, c):
        return sum(d.get(c, 0) for d in keyed[i].get(key, []))

    def n(i, key):
        return max(1, len(keyed[i].get(key, [])))

    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "calls", "ms_per_call", "read_GB", "write_GB", "GB_per_s", "clock_GHz",
                "mfma_busy_share", "mfma_per_wave", "valu_per_wave", "lds_per_wave", "lds_conflict_per_inst",
                "wait_any_share", "wait_lds_share", "valu_active_share", "mfma_active_share"])
    for key, fl in keyed[0].items():
        if filt is None and not fl[0]["ours"]:
            continue
        if filt is not None and filt not in key[0]:
            continue
        calls = len(fl)
        ns = sum(d["ns"] for d in fl) / calls
        rd = tot(2, key, "FETCH_SIZE") / n(2, key) * 1024 / 1e9
        wr = tot(3, key, "WRITE_SIZE") / n(3, key) * 1024 / 1e9
        grbm = tot(2, key, "GRBM_GUI_ACTIVE") / n(2, key)
        p3ns = sum(d["ns"] for d in keyed[2].get(key, [])) / n(2, key)
        busy, mf = tot(0, key, "SQ_BUSY_CYCLES"), tot(0, key, "SQ_VALU_MFMA_BUSY_CYCLES")
        waves = tot(0, key, "SQ_WAVES") or 1
        lds, bc = tot(0, key, "SQ_INSTS_LDS"), tot(0, key, "SQ_LDS_BANK_CONFLICT")
        wc = tot(1, key, "SQ_WAVE_CYCLES") or 1
        w.writerow([key[0], key[1], calls, round(ns / 1e6, 4), round(rd, 3), round(wr, 3),
                    round((rd + wr) / (ns / 1e9)) if ns else "", round(grbm / 8 / p3ns, 3) if p3ns else "",
                    round(mf / busy, 3) if busy else "", round(tot(0, key, "SQ_INSTS_MFMA") / waves, 1),
                    round(tot(1, key, "SQ_INSTS_VALU") / waves, 1), round(lds / waves, 1),
                    round(bc / lds, 3) if lds else "", round(tot(1, key, "SQ_WAIT_ANY") / wc, 3),
                    round(tot(0, key, "SQ_WAIT_INST_LDS") / wc, 3) if tot(1, key, "SQ_WAVE_CYCLES") else "",
                    round(tot(1, key, "SQ_ACTIVE_INST_VALU") / wc, 3),
                    round(tot(1, key, "SQ_ACTIVE_INST_MFMA") / wc, 3)])


if __name__ == "__main__":
    main()
