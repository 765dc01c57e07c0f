import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj
ctx = pj.Context(0)
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
roots = g.sample_roots(2, 3)
for d in ([0] + [float(x) for x in sys.argv[2:]]):
    g.set_option("delta", d)
    for r in roots:
        g.sssp(int(r), copy=False); s = g.stats()
        print(f"delta {d} root {r}: {s['kernel_ms']:.2f} ms levels {s['levels']} rounds {s['relax_rounds']}", flush=True)
