"""Repeat weighted (delta-stepping) solves and weighted batches and count results that differ from
the first solve of the same root (final distances are unique, so a race shows up as a mismatch).
Single solves repeat `reps` times per root; batches run the same roots under batch_streams 1, 2, 3.
Usage: python tools/delta_stress.py [scale=22] [reps=10] [key=value ...]"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

args = dict(kv.split("=") for kv in sys.argv[1:])
scale = int(args.pop("scale", 22))
reps = int(args.pop("reps", 10))
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
for k, v in args.items():
    g.set_option(k, float(v))
roots = [int(r) for r in g.sample_roots(7, 8)]
ref = {r: g.sssp(r) for r in roots}


def report(tag, rep, r, d):
    diff = np.nonzero(d != ref[r])[0]
    print(f"MISMATCH {tag} rep={rep} root={r} ndiff={diff.size} first={diff[:5].tolist()} "
          f"got={d[diff[:5]].tolist()} ref={ref[r][diff[:5]].tolist()}", flush=True)


bad = 0
nbad = 0
for rep in range(reps):
    for r in roots:
        d = g.sssp(r)
        if not np.array_equal(d, ref[r]):
            nbad += 1
            report("single", rep, r, d)
print(f"k{scale}w single: {nbad} of {reps * len(roots)} differ", flush=True)
bad += nbad
for streams in (1, 2, 3):
    g.set_option("batch_streams", streams)
    nbad = 0
    for rep in range(max(1, reps // 2)):
        rows = g.sssp_batch(roots)
        for i, r in enumerate(roots):
            if not np.array_equal(rows[i], ref[r]):
                nbad += 1
                report(f"batch_streams={streams}", rep, r, rows[i])
    print(f"k{scale}w batch_streams={streams}: {nbad} of {max(1, reps // 2) * len(roots)} differ", flush=True)
    bad += nbad
print("delta_stress: total mismatches", bad, flush=True)
sys.exit(1 if bad else 0)
