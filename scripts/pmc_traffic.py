"""Per-dispatch PMC summary of one kernel from rocprofv3 --pmc passes (p*/run_counter_collection.csv).

    python scripts/pmc_traffic.py <pmc_dir> [kernel_substring (default corr_batch_kernel)]

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced streaming reads → read bytes = 2 × FETCH_SIZE × 1024; WRITE_SIZE
is exact for 16-B stores.  8-B/lane loads (the correlators' CF32 samples) are an access width the
guide leaves uncalibrated, so the read figure is the guide's correction applied as prescribed (an
upper estimate if 8-B requests are tallied at full size).  Every other counter is reported as its
per-dispatch median (SQ_INSTS_VALU → valu_insts_per_launch)."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "corr_batch_kernel"
last_only = len(sys.argv) > 3 and sys.argv[3] == "last"  # only each pass's last dispatch of the kernel (the timed launch)
vals = {}
for f in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")) + glob.glob(os.path.join(root, "p*", "*", "*counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if kname in r["Kernel_Name"]]
    if last_only and rows:
        key = lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)  # noqa: E731
        top = max(key(r) for r in rows)
        rows = [r for r in rows if key(r) == top]
    for row in rows:
        disp = (f, row.get("Dispatch_Id") or row.get("Correlation_Id") or "")
        vals.setdefault(row["Counter_Name"], {}).setdefault(disp, 0.0)
        vals[row["Counter_Name"]][disp] += float(row["Counter_Value"])
med = lambda v: sorted(v)[len(v) // 2] if v else None  # noqa: E731
out = {"kernel": kname, "dispatches": {c: len(v) for c, v in vals.items()}}
f_kib = med(list(vals.get("FETCH_SIZE", {}).values()))
w_kib = med(list(vals.get("WRITE_SIZE", {}).values()))
out["fetch_size_kib_median"], out["write_size_kib_median"] = f_kib, w_kib
out["hbm_read_bytes_corrected"] = 2 * f_kib * 1024 if f_kib is not None else None
out["hbm_write_bytes"] = w_kib * 1024 if w_kib is not None else None
if f_kib is not None and w_kib is not None:
    out["hbm_bytes_per_launch"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
for c, v in vals.items():
    if c in ("FETCH_SIZE", "WRITE_SIZE"):
        continue
    out[c + "_median"] = med(list(v.values()))
if "SQ_INSTS_VALU" in vals:
    out["valu_insts_per_launch"] = out["SQ_INSTS_VALU_median"]
print(json.dumps(out, indent=1))
