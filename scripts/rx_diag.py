"""Diagnostic: the C1 receiver test's run of tools/gnsship_rx (tests/test_gpu_receiver.py) with its
events and records kept under gpurun_out/rxdiag/ for an offline comparison with oracle/receiver.py.
    python scripts/rx_diag.py [extra gnsship_rx args]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gnss_sim_receiver_amd import signals as S  # noqa: E402

FS = 4000000
out = os.path.join(ROOT, "gpurun_out", "rxdiag")
os.makedirs(out, exist_ok=True)
sats = S.c1_sky(extra=((3, -2400.0, 3001.0),))
x = S.generate_if(FS, int(0.5 * FS), sats, seed=0x6E550001)
path = os.path.join(out, "c1.dat")
x.tofile(path)
cmd = [os.path.join(ROOT, "tools", "gnsship_rx"), "--file", path, "--item", "gr_complex", "--fs", str(FS), "--channels", "3",
       "--in-acquisition", "1", "--rotator", "avx", "--block-ms", "100", "--acq-piece", "8192", "--events", os.path.join(out, "events.csv"),
       "--records", os.path.join(out, "records.bin"), "--dump", os.path.join(out, "trk_ch_"), *sys.argv[1:]]
r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
print(r.stdout[-2000:], r.stderr[-2000:])
os.remove(path)
sys.exit(r.returncode)
