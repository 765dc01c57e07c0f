"""k26w light rounds, launch by launch: configs[2]'s graph (Kronecker s26, weights 1..255), the bench's
roots (sample_roots seed 2), one untimed solve for the workspace, then ROOTS solves with the round_log
option (libpj prints one stderr line per v2_pull_round_k launch: kind, band lo, frontier, its light
edges) and a "== solve root" line after each. Run under a kernel trace; tools/round_kinds.py joins the
two. Usage: python tools/k26w_rounds.py [roots=4] [opt=value ...]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

nroots = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ctx = pj.Context(0)
g = ctx.generate_kronecker(26, 16, 1, weighted=True)
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    g.set_option(k, float(v))
roots = [int(r) for r in g.sample_roots(2, nroots)]
g.sssp(roots[0], copy=False)  # (workspace; unlogged)
g.set_option("round_log", 1)
for r in roots:
    g.sssp(r, copy=False)
    st = g.stats()
    print(f"== solve root {r} kernel_ms {st['kernel_ms']:.4f} bands {st['levels']} rounds {st['relax_rounds']} "
          f"scanned {st['scanned_edges']} probes {st['probes']}", file=sys.stderr, flush=True)
g.set_option("round_log", 0)
