"""Static instruction mix of one corr_batch_kernel instance (default: CF32, 3 taps, in-margin).
   python scripts/isa_count.py [fmt nt margin]"""
import collections, subprocess, sys
fmt, nt, m = (sys.argv[1:4] if len(sys.argv) > 3 else ("0", "3", "1"))
src = __import__("os").environ.get("KRES_SRC", "gnss_sim_receiver_amd/csrc/corr_kernel.hip")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-Iinclude",
                "-Ignss_sim_receiver_amd/csrc", "--cuda-device-only", "-S", src, "-o", "/tmp/isa.s"], check=True, capture_output=True)
s = open("/tmp/isa.s").read()
key = f"_ZN7gnsship17corr_batch_kernelILi{fmt}ELi{nt}ELb{m}E"
a = s.index(key)
a = s.index(":\n", a)
b = s.index(".Lfunc_end", a)
ins = [l.strip() for l in s[a:b].splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(i.split()[0] for i in ins)
cls = collections.Counter()
for k, v in c.items():
    cls["valu" if k.startswith("v_") else "salu" if k.startswith("s_") and not k.startswith(("s_load", "s_buffer", "s_waitcnt", "s_nop", "s_cbranch", "s_branch")) else
        "lds" if k.startswith("ds_") else "vmem" if k.startswith(("global_", "flat_", "buffer_", "scratch_")) else "smem" if k.startswith(("s_load", "s_buffer")) else "other"] += v
print(len(ins), dict(cls))
open("/tmp/isa_kernel.s", "w").write(s[a:b])
if "-v" in sys.argv:
    for k, v in c.most_common(40):
        print(k, v)
