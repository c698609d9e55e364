"""Per-dispatch HBM bytes of corr_batch_kernel from the FETCH_SIZE / WRITE_SIZE passes.

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced streaming reads → read bytes = 2 × FETCH_SIZE × 1024; WRITE_SIZE
is exact for 16-B stores.  The correlator's IF loads are 8 B/lane (CF32) — an access width the
guide leaves uncalibrated — so the read figure is the guide's correction applied as prescribed
(an upper estimate if 8-B requests are tallied at full size)."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
vals = {}
for f in glob.glob(os.path.join(root, "p*", "run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if "corr_batch_kernel" not in name:
            continue
        key = (row.get("Dispatch_Id") or row.get("Correlation_Id") or "", row["Counter_Name"])
        vals.setdefault(row["Counter_Name"], {}).setdefault(key[0], 0.0)
        vals[row["Counter_Name"]][key[0]] += float(row["Counter_Value"])
fetch = sorted(vals.get("FETCH_SIZE", {}).values())
write = sorted(vals.get("WRITE_SIZE", {}).values())
med = lambda v: v[len(v) // 2] if v else None  # noqa: E731
f_kib, w_kib = med(fetch), med(write)
out = {"kernel": "corr_batch_kernel", "dispatches": [len(fetch), len(write)], "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib,
       "hbm_read_bytes_corrected": 2 * f_kib * 1024 if f_kib is not None else None,
       "hbm_write_bytes": w_kib * 1024 if w_kib is not None else None}
if f_kib is not None and w_kib is not None:
    out["hbm_bytes_per_launch"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
print(json.dumps(out, indent=1))
