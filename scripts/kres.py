"""Per-kernel register/LDS/occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.
   python scripts/kres.py [extra hipcc flags...]   (corr_kernel.hip)"""
import re, subprocess, sys
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Iinclude",
       "-Ignss_sim_receiver_amd/csrc", "-Rpass-analysis=kernel-resource-usage", "-c", __import__("os").environ.get("KRES_SRC", "gnss_sim_receiver_amd/csrc/corr_kernel.hip"),
       "-o", "/tmp/kres.o"] + sys.argv[1:]
txt = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in txt.splitlines():
    m = re.search(r"remark: +(.*?) \[-Rpass", line)
    if not m:
        continue
    kv = m.group(1)
    if kv.startswith("Function Name:"):
        name = kv.split(":", 1)[1].strip()
        t = re.search(r"corr_batch_kernelILi(\d)ELi(\d)ELb(\d)", name)
        cur = {"k": f"corr fmt{t.group(1)} nt{t.group(2)} m{t.group(3)}" if t else name[:40]}
        rows.append(cur)
    elif cur is not None and ":" in kv:
        k, v = kv.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r['k']:28s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} sgpr {r.get('TotalSGPRs','?'):>4} "
          f"spill v{r.get('VGPRs Spill','?')} s{r.get('SGPRs Spill','?')} occ {r.get('Occupancy [waves/SIMD]','?')} lds {r.get('LDS Size [bytes/block]','?')}")
