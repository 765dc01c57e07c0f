"""web-Google-shaped synthetic (configs[0]): a few unit-weight solves from source 0 (for kernel traces)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
for kv in sys.argv[1:]:
    k, v = kv.split("="); g.set_option(k, float(v))
for _ in range(5):
    g.sssp(0, copy=False)
    print(g.stats(), flush=True)
