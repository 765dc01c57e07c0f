"""Fixed SSSP workload for the per-kernel table of a round cycle (tools/cycle.sh `wtable`):
the kernel trace and the rocprofv3 --pmc passes run this same command, so time, PMC bytes
and the device work counters describe the same solves. Runs SOLVES solves of the bench's
roots (sample_roots seed 2 = bench.py's args.seed + 1) on a Kronecker graph, after one
untimed solve that builds the solver workspace, and writes per solve its pj_stats (work
counters, kernel_ms) plus pj_build_id() to --json.
Usage: python tools/traffic_probe.py [scale] [solves] [weighted 0/1] [--json PATH]"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out_path = None
if "--json" in sys.argv:
    out_path = sys.argv[sys.argv.index("--json") + 1]
    args = [a for a in args if a != out_path]
scale = int(args[0]) if len(args) > 0 else 22
solves = int(args[1]) if len(args) > 1 else 8
weighted = bool(int(args[2])) if len(args) > 2 else False
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=weighted)
roots = [int(r) for r in g.sample_roots(2, solves)]
per = []
for r in [roots[0]] + roots:  # (the first solve also prepares the solver: its kernels are excluded by name)
    g.sssp(r, copy=False)
    st = g.stats()
    rs = g.reach_stats()  # (the gather to input ids and the reach pass: not solve kernels, excluded by name)
    st.update(root=r, reached=rs["reached"], reached_edges=rs["reached_edges"])
    per.append(st)
res = {"build_id": pj.build_id(), "scale": scale, "weighted": weighted, "n": g.n, "nnz": g.nnz, "roots": roots,
       "solves": per,
       "note": "solves[0] repeats roots[0] and carries the solver preparation; every solve's v2_init_k starts it"}
if out_path:
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
print(f"traffic_probe scale {scale} weighted {weighted} solves {len(per)} build {pj.build_id()} "
      f"roots {roots}", flush=True)
