"""configs[4] through the drop-in: the web-Google-shaped text, the 1024 smallest ids with
out-degree >= 1 in PJ_SOURCES, `parallel_johnson` writing one sol_file per source; times
the process end to end and spot-checks files against single-source runs.
Usage: python tools/ms_cli_probe.py [n_sources] [gpus]"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import paralleljohnson_amd as pj  # noqa: E402
from helpers import csr_to_text  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
gpus = int(sys.argv[2]) if len(sys.argv) > 2 else 1
td = tempfile.mkdtemp(dir=os.environ.get("PJ_SCRATCH", "/tmp"))
ctx = pj.Context(0)
g = ctx.generate_webgraph(seed=1)
row, col, _ = g.get_csr()
g.close()
ctx.close()
path = os.path.join(td, "wg.txt")
with open(path, "wb") as f:
    f.write(csr_to_text(row, col.view(np.uint32)))
srcs = np.nonzero(np.diff(row) >= 1)[0][:k]
lst = os.path.join(td, "sources.txt")
with open(lst, "w") as f:
    f.write("\n".join(map(str, srcs)) + "\n")
out_dir = os.path.join(td, "out")
os.makedirs(out_dir)
env = dict(os.environ, PJ_SOURCES="@" + lst, PJ_GPUS=str(gpus), PJ_PHASES="1")
t = time.perf_counter()
r = subprocess.run([pj.cli_path(), path, "0", os.path.join(out_dir, "sol_{s}.txt")], env=env, capture_output=True,
                   text=True, timeout=900)
wall = time.perf_counter() - t
assert r.returncode == 0, r.stderr[-2000:]
files = os.listdir(out_dir)
total = sum(os.path.getsize(os.path.join(out_dir, x)) for x in files)
ok = True
for s in (srcs[0], srcs[len(srcs) // 2], srcs[-1]):  # spot check vs single-source runs
    single = os.path.join(td, "single.txt")
    subprocess.run([pj.cli_path(), path, str(s), single], check=True, capture_output=True)
    ok &= open(single, "rb").read() == open(os.path.join(out_dir, f"sol_{s}.txt"), "rb").read()
print(json.dumps({"sources": int(len(srcs)), "gpus": gpus, "files": len(files), "bytes_written": total,
                  "time_to_solution_s": round(wall, 3), "time_line": r.stdout.strip(),
                  "phases": [ln for ln in r.stderr.splitlines() if ln.startswith("phase")],
                  "spot_check_identical_to_single_runs": bool(ok)}), flush=True)
shutil.rmtree(td)
