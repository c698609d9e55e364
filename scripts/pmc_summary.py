"""Summarise rocprofv3 PMC passes (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel:
mean counter value per dispatch.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming
reads, so hbm_read_bytes = 2 × FETCH_SIZE × 1024 (an upper estimate for narrower accesses)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, d in vals.items():
    if "rocclr" in k:
        continue
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
    if "FETCH_SIZE" in out[k]:
        out[k]["hbm_read_bytes_corrected"] = 2 * out[k]["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in out[k]:
        out[k]["hbm_write_bytes"] = out[k]["WRITE_SIZE"] * 1024
print(json.dumps(out, indent=1))
