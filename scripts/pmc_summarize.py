"""Summarise rocprofv3 --pmc passes (p1: SQ counters, p2: FETCH_SIZE, p3: WRITE_SIZE) of a
PMC driver run into one row per (kernel, grid): calls, ms per call (from the FETCH_SIZE
pass), HBM read/write GB per call, achieved GB/s, MFMA-busy share and LDS bank conflicts.
usage: pmc_summarize.py <dir with p1/ p2/ p3/> [name-substring-filter]"""
import collections
import csv
import os
import sys


def load(path):
    per = collections.defaultdict(dict)   # dispatch id -> {counter: value, ...}
    for r in csv.DictReader(open(path)):
        d = per[r["Dispatch_Id"]]
        nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        d["name"] = nm.split("(")[0][:70]
        d["ours"] = "(anonymous namespace)::" in r["Kernel_Name"]
        d["grid"] = r["Grid_Size"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else "anonymous namespace"
    passes = [load(os.path.join(root, p, "k_counter_collection.csv")) for p in ("p1", "p2", "p3")]
    keyed = [collections.defaultdict(list) for _ in passes]
    for i, per in enumerate(passes):
        for d in per.values():
            keyed[i][(d["name"], d["grid"])].append(d)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "calls", "ms_per_call", "read_GB", "write_GB", "GB_per_s", "mfma_busy_per_busy_cycle",
                "lds_bank_conflict_per_inst"])
    for key, fl in keyed[1].items():
        if not (fl[0]["ours"] if filt == "anonymous namespace" else filt in key[0]):
            continue
        calls = len(fl)
        ns = sum(d["ns"] for d in fl) / calls
        rd = sum(d.get("FETCH_SIZE", 0) for d in fl) / calls * 1024 / 1e9
        wl = keyed[2].get(key, [])
        wr = sum(d.get("WRITE_SIZE", 0) for d in wl) / max(1, len(wl)) * 1024 / 1e9
        sl = keyed[0].get(key, [])
        busy = sum(d.get("SQ_BUSY_CYCLES", 0) for d in sl)
        mf = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in sl)
        lds = sum(d.get("SQ_INSTS_LDS", 0) for d in sl)
        bc = sum(d.get("SQ_LDS_BANK_CONFLICT", 0) for d in sl)
        w.writerow([key[0], key[1], calls, round(ns / 1e6, 4), round(rd, 3), round(wr, 3),
                    round((rd + wr) / (ns / 1e9)), round(mf / busy, 3) if busy else "",
                    round(bc / lds, 3) if lds else ""])


if __name__ == "__main__":
    main()
