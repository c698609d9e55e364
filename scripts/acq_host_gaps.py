"""Host-side gaps of repeated acquisition sweeps from a rocprofv3 --hip-trace --kernel-trace run:
per gnsship_acq_run call, hipGraphLaunch entry -> first kernel start, last kernel end ->
hipStreamSynchronize return, and the call's whole span.
    python scripts/acq_host_gaps.py <dir with run_hip_api_trace.csv and run_kernel_trace.csv> [kernel name part]
(with a name part, only the calls whose kernels include one so named)"""
import csv
import glob
import os
import sys

import numpy as np

d = sys.argv[1]
api = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
ker = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
ker = sorted(((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in ker if "rocclr" not in k["Kernel_Name"]))
launches = sorted(int(a["Start_Timestamp"]) for a in api if a["Function"] == "hipGraphLaunch")
syncs = sorted(int(a["End_Timestamp"]) for a in api if a["Function"] == "hipStreamSynchronize")
rows = []
for i, t in enumerate(launches):
    nxt = launches[i + 1] if i + 1 < len(launches) else 1 << 62
    ks = [k for k in ker if t <= k[0] < nxt]
    if not ks or (len(sys.argv) > 2 and not any(sys.argv[2] in k[2] for k in ks)):
        continue
    kend = max(k[1] for k in ks)
    s = [x for x in syncs if x >= kend and x < nxt]
    if not s:
        continue
    rows.append(((ks[0][0] - t) / 1e3, (kend - ks[0][0]) / 1e3, (s[0] - kend) / 1e3, (s[0] - t) / 1e3))
r = np.array(rows[2:])
print(f"{len(r)} sweeps: launch->first kernel {np.median(r[:, 0]):.1f} us, kernels {np.median(r[:, 1]):.1f} us, "
      f"last kernel->sync return {np.median(r[:, 2]):.1f} us, launch->sync return {np.median(r[:, 3]):.1f} us")
