"""Summarise tools/pmc.sh output: per-kernel counter totals and derived ratios."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "screen"
agg = collections.defaultdict(float)
dur = 0.0
launches = 0
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for f in sorted(glob.glob(os.path.join(d, "p1", "run_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            dur += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
            launches += 1
print({k: "%.4g" % v for k, v in sorted(agg.items())})
g = agg.get("GRBM_GUI_ACTIVE", 0) / 8
if g:
    print("kernel s %.4f, clock GHz %.3f" % (dur, g / dur / 1e9 if dur else 0))
    print("MFMA busy (per SIMD) %.3f" % (agg["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / g))
w = agg.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        print("%s / WAVE_CYCLES %.3f" % (k, agg[k] / w))
m = agg.get("SQ_INSTS_MFMA", 0)
if m:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
        if k in agg:
            print("%s per MFMA %.2f" % (k, agg[k] / m))
if "TCC_HIT_sum" in agg:
    print("L2 hit %.3f" % (agg["TCC_HIT_sum"] / (agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"])))
if "FETCH_SIZE" in agg:
    print("FETCH_SIZE (KB, x2 gfx950 correction) %.4g -> %.4g GB" % (agg["FETCH_SIZE"], 2 * agg["FETCH_SIZE"] * 1024 / 1e9))

if len(sys.argv) > 3 and "FETCH_SIZE" in agg:
    import json
    fetch = 2 * agg["FETCH_SIZE"] * 1024  # KB, gfx950 wide-read correction (MI355X_MICROARCH.md:298)
    write = agg.get("WRITE_SIZE", 0.0) * 1024
    level = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # bench.py screen_level this was measured at
    rec = {"kernel": key, "screen_level": level, "launches": launches, "kernel_s": dur,
           "fetch_bytes": fetch, "write_bytes": write,
           "hbm_bytes_per_launch": (fetch + write) / max(launches, 1),
           "source": os.path.relpath(d), "counters": {k: v for k, v in sorted(agg.items())}}
    json.dump(rec, open(sys.argv[3], "w"), indent=1)
    print("wrote", sys.argv[3], "bytes/launch %.4g" % rec["hbm_bytes_per_launch"])
