"""Fixed SSSP workload for rocprofv3 --pmc passes (HBM traffic per solve).
Runs SOLVES solves on a Kronecker graph; every solve kernel (sel_*, d_relax_k, unlabel_k,
d_source_k / bfs_*) belongs to one of them.
Usage: python tools/traffic_probe.py [scale] [solves] [weighted 0/1]"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
solves = int(sys.argv[2]) if len(sys.argv) > 2 else 8
weighted = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=weighted)
roots = g.sample_roots(2, solves)
for r in roots:
    g.sssp(int(r), copy=False)
print(f"traffic_probe scale {scale} weighted {weighted} solves {len(roots)} roots {list(map(int, roots))}", flush=True)
