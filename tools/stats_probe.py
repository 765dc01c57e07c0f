"""Solves of the k26w bench graph under libpj options, for the PJ_V2_STATS build's per-round
counters (stderr) and per-solve kernel times: python tools/stats_probe.py scale solves key=val ..."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj

scale, solves = int(sys.argv[1]), int(sys.argv[2])
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
for kv in sys.argv[3:]:
    k, v = kv.split("=")
    g.set_option(k, float(v))
roots = [int(r) for r in g.sample_roots(2, solves)]
for r in roots:
    g.sssp(r, copy=False)
    st = g.stats()
    print(f"root {r} kernel_ms {st['kernel_ms']:.3f} bands {st['levels']} rounds {st['relax_rounds']}", flush=True)
    print(f"== solve root {r} done", file=sys.stderr, flush=True)
