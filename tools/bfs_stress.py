"""Repeat unit-weight solves under each direction policy and bfs_small setting and count results that
differ from the first solve of the same root (a race shows up as an occasional mismatch).
Usage: python tools/bfs_stress.py [graph=k22|wg] [reps=10] [key=value ...]"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

args = dict(kv.split("=") for kv in sys.argv[1:])
name = args.pop("graph", "k22")
reps = int(args.pop("reps", 10))
ctx = pj.Context(0)
if name == "wg":
    g = ctx.generate_webgraph()
    roots = [0] + [int(r) for r in g.sample_roots(7, 7)]
else:
    g = ctx.generate_kronecker(int(name[1:]), 16, 1)
    roots = [int(r) for r in g.sample_roots(7, 8)]
for k, v in args.items():
    g.set_option(k, float(v))
ref = {}
for r in roots:
    g.set_option("direction", 0)
    g.set_option("bfs_small", 0)
    ref[r] = g.sssp(r)
bad = 0
for mode in (0, 1, 2):
    g.set_option("direction", mode)
    for small in (0, 1):
        g.set_option("bfs_small", small)
        nbad = 0
        for rep in range(reps):
            for r in roots:
                d = g.sssp(r)
                if not np.array_equal(d, ref[r]):
                    nbad += 1
                    diff = np.nonzero(d != ref[r])[0]
                    print(f"MISMATCH direction={mode} small={small} rep={rep} root={r} ndiff={diff.size} "
                          f"first={diff[:5].tolist()} got={d[diff[:5]].tolist()} ref={ref[r][diff[:5]].tolist()} "
                          f"stats={g.stats()}", flush=True)
        bad += nbad
        print(f"{name} direction={mode} small={small}: {nbad} of {reps * len(roots)} differ", flush=True)
print("bfs_stress: total mismatches", bad, flush=True)
sys.exit(1 if bad else 0)
