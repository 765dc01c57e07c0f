"""CLI ingest at P = 1, 2, 3 on the K22 text (configs[1] written as a SNAP file): the
`parallel_johnson` phases (PJ_PHASES=1: load = read + parse + CSR / partition build) and the
wall time, with P > 1 ranks sharing this GPU (PJ_GPUS, host transport). Since round 5 the
partitioned load parses the file once on rank 0's GPU and scatters each rank its entries
(pj_part_load_snap_group); before, every rank parsed the whole file.
Usage: python tools/probe_cli_ingest.py [scale=22] [reps=2]"""
import os
import re
import subprocess
import sys
import tempfile
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
with tempfile.TemporaryDirectory() as td:
    path = os.path.join(td, f"k{scale}.txt")
    with pj.Context(0) as ctx:
        ctx.kronecker_write_snap(path, scale, 16, 1)
    print(f"text {os.path.getsize(path) / 1e9:.2f} GB", flush=True)
    for rep in range(reps):
        for P in (1, 2, 3):
            out = os.path.join(td, f"sol{P}.txt")
            env = dict(os.environ, PJ_GPUS=str(P), PJ_PHASES="1")
            t = time.perf_counter()
            r = subprocess.run([pj.cli_path(), path, "1", out], capture_output=True, text=True, timeout=600, env=env)
            wall = time.perf_counter() - t
            if r.returncode != 0:
                raise SystemExit(f"P={P} failed: {r.stderr[-800:]}")
            ph = {m.group(1): float(m.group(2)) for m in (re.match(r"phase (.+): ([0-9.e+-]+) s", ln)
                                                          for ln in r.stderr.splitlines()) if m}
            print(f"rep {rep} P={P}: wall {wall:.3f} s, phases {ph}, {r.stdout.strip()}", flush=True)
        same = [open(os.path.join(td, f"sol{P}.txt"), "rb").read() for P in (1, 2, 3)]
        print(f"rep {rep}: sol_files identical across P: {same[0] == same[1] == same[2]}", flush=True)
