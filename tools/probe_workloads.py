"""Quick timings of the secondary workloads (not the driver's bench line)."""
import os, subprocess, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import paralleljohnson_amd as pj
from helpers import csr_to_text

ctx = pj.Context(0)
res = {}
# configs[0]: web-Google-shaped, source 0
t = time.perf_counter(); g = ctx.generate_webgraph(); res["wg_gen_s"] = time.perf_counter() - t
for _ in range(3): g.sssp(0, copy=False)
ts = []
for _ in range(10):
    g.sssp(0, copy=False); ts.append(g.stats())
st = g.reach_stats()
res["wg_solve_ms"] = float(np.median([x["kernel_ms"] for x in ts])); res["wg_levels"] = ts[-1]["levels"]
res["wg_td_bu"] = (ts[-1]["td_levels"], ts[-1]["bu_levels"]); res["wg_reached"] = st["reached"]; res["wg_m_r"] = st["reached_edges"]
row, col, _ = g.get_csr()
text = csr_to_text(row, col.astype(np.uint32)); path = "/tmp/wg.txt"; open(path, "wb").write(text)
res["wg_text_mb"] = len(text) / 1e6
t = time.perf_counter()
r = subprocess.run([pj.cli_path(), path, "0", "/tmp/wg_sol.txt"], capture_output=True, text=True)
res["wg_cli_time_to_solution_s"] = time.perf_counter() - t; res["wg_cli_stdout"] = r.stdout.strip()
# MS1024 on WG
src = [int(x) for x in np.nonzero(np.diff(row) > 0)[0][:1024]]
g.sssp_batch(src[:64], copy=False)
t = time.perf_counter(); g.sssp_batch(src, copy=False); el = time.perf_counter() - t
res["ms1024_wall_s"] = el; res["ms1024_kernel_ms"] = g.stats()["kernel_ms"]; res["ms1024_levels_max"] = g.stats()["levels"]
g.close()
# weighted delta-stepping
for scale in (20, 22, 24):
    t = time.perf_counter(); gw = ctx.generate_kronecker(scale, 16, 1, weighted=True); gen = time.perf_counter() - t
    roots = gw.sample_roots(2, 4)
    gw.sssp(int(roots[0]), copy=False)
    ks = []
    for r in roots:
        gw.sssp(int(r), copy=False); s = gw.stats(); rs = gw.reach_stats(); ks.append((s["kernel_ms"], s["levels"], s["relax_rounds"], rs["reached_edges"]))
    res[f"k{scale}w"] = {"gen_build_s": gen, "solves": ks, "gteps": float(np.mean([k[3] / k[0] / 1e6 for k in ks]))}
    gw.close()
print(json.dumps(res, indent=1))
