"""One weighted Kronecker solve with options: python tools/probe_one.py SCALE [key=value ...]"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_kronecker(int(sys.argv[1]), 16, 1, weighted=True)
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    g.set_option(k, float(v))
r = int(g.sample_roots(2, 1)[0])
g.sssp(r, copy=False)
print("solve", r, g.stats(), flush=True)
