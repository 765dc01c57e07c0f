"""Per-level profile of the unit-weight BFS on configs[1] (Graph500 Kronecker s22, the bench's
roots: sample_roots seed 2 = bench.py's args.seed + 1). One untimed solve builds the workspace,
then ROOTS solves run with the level_log option: libpj prints one stderr line per level launch
(level, push / pull, where the frontier came from, its vertices and out-edges, and the in-edge
probes the previous launch scanned). tools/cycle.sh `klevels` runs this under the kernel trace
and --pmc passes; tools/k22_level_table.py joins them launch by launch.
Usage: python tools/k22_levels.py [roots=4] [graph=wg|kNN] [rootlist=a/b/...] [opt=value ...]  (graph=wg:
configs[0]'s web-Google-shaped graph, source 0 and sampled roots; kNN: Kronecker scale NN; rootlist: these
roots instead of the sampled ones)"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

nroots = int(sys.argv[1]) if len(sys.argv) > 1 else 4
opts = dict(kv.split("=") for kv in sys.argv[2:])
ctx = pj.Context(0)
gname = opts.pop("graph", "k22")
rootlist = opts.pop("rootlist", "")
wg = gname == "wg"
g = ctx.generate_webgraph() if wg else ctx.generate_kronecker(int(gname[1:]), 16, 1)
for k, v in opts.items():
    g.set_option(k, float(v))
roots = ([0] + [int(r) for r in g.sample_roots(2, nroots - 1)]) if wg else [int(r) for r in g.sample_roots(2, nroots)]
if rootlist:
    roots = [int(x) for x in rootlist.split("/")]
g.sssp(roots[0], copy=False)  # (workspace; unlogged)
g.set_option("level_log", 1)
for r in roots:
    print(f"solve root {r}", file=sys.stderr, flush=True)
    g.sssp(r, copy=False)
    st = g.stats()
    rs = g.reach_stats()
    print(f"solve_done root {r} kernel_ms {st['kernel_ms']:.4f} levels {st['levels']} push {st['td_levels']} "
          f"pull {st['bu_levels']} scanned_edges {st['scanned_edges']} reached {rs['reached']} "
          f"reached_edges {rs['reached_edges']}", file=sys.stderr, flush=True)
g.set_option("level_log", 0)
