"""Ingestion phases of the CLI on SNAP text (the reference's read_webgraph + coord2csr
path, :66-159): writes the web-Google-shaped synthetic and a Kronecker text file
(generation order) to a scratch dir, then times `parallel_johnson` end to end with
PJ_PHASES=1 and prints one JSON line per input.
Usage: python tools/ingest_probe.py [kron_scale ...] [--keep]   (default 22)"""
import json
import os
import subprocess
import sys
import tempfile
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import paralleljohnson_amd as pj  # noqa: E402
from helpers import csr_to_text  # noqa: E402

keep = "--keep" in sys.argv  # leave the text files (and print their paths) for a profiler run
scales = [int(a) for a in sys.argv[1:] if a.isdigit()] or [22]
td = tempfile.mkdtemp(dir=os.environ.get("PJ_SCRATCH", "/tmp"))
ctx = pj.Context(0)
inputs = []
g = ctx.generate_webgraph(seed=1)
row, col, _ = g.get_csr()
g.close()
p = os.path.join(td, "wg.txt")
with open(p, "wb") as f:
    f.write(csr_to_text(row, col.view("uint32")))
inputs.append(("wg", p, 0))
for sc in scales:
    p = os.path.join(td, f"k{sc}.txt")
    t = time.perf_counter()
    ctx.kronecker_write_snap(p, sc, 16, 1)
    print(f"# wrote {p} ({os.path.getsize(p) / 1e9:.2f} GB) in {time.perf_counter() - t:.1f} s", flush=True)
    inputs.append((f"k{sc}", p, 1))
ctx.close()
for name, path, src in inputs:
    out = os.path.join(td, "sol.txt")
    t = time.perf_counter()
    r = subprocess.run([pj.cli_path(), path, str(src), out], capture_output=True, text=True,
                       env=dict(os.environ, PJ_PHASES="1"), timeout=600)
    wall = time.perf_counter() - t
    phases = [ln for ln in r.stderr.splitlines() if ln.startswith("phase ")]
    print(json.dumps({"input": name, "text_bytes": os.path.getsize(path), "rc": r.returncode,
                      "time_to_solution_s": round(wall, 3), "time_line": r.stdout.strip(), "phases": phases}),
          flush=True)
    os.remove(out)
    if keep:
        print(f"# kept {path}", flush=True)
    else:
        os.remove(path)
