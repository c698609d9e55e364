"""Timeline of the last acquisition sweep in a rocprofv3 kernel trace (run_kernel_trace.csv): each
dispatch's start and end relative to the sweep's first kernel, and the sweep's span.  The sweep starts
at the last launch whose name contains FIRST (default: the E1 huge layout's forward column kernel).
    python scripts/acq_timeline.py gpurun_out/.../run_kernel_trace.csv [FIRST]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rocclr" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last sweep: from the last forward column launch of the huge layout to the decision after it
first_pat = sys.argv[2] if len(sys.argv) > 2 else "acq_huge_cols_fwd"
idx = [i for i, r in enumerate(rows) if first_pat in r["Kernel_Name"]]
if not idx:
    raise SystemExit("no huge sweep in the trace")
first = idx[-1]
last = next(i for i in range(first, len(rows)) if "acq_decide" in rows[i]["Kernel_Name"])
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:last + 1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gnsship::", "")
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  q{r['Queue_Id']}  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}  {name}")
print(f"sweep span {(int(rows[last]['End_Timestamp']) - t0) / 1e3:.1f} us")
