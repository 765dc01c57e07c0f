"""Weighted delta-stepping timings across Kronecker scales (progress printed per solve).
Usage: python tools/probe_weighted_scales.py 22 24 26"""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj

ctx = pj.Context(0)
out = {}
for scale in [int(x) for x in sys.argv[1:]] or [22]:
    t = time.perf_counter()
    g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
    gen = time.perf_counter() - t
    print(f"s{scale}w: n={g.n} nnz={g.nnz} gen+build {gen:.2f} s", flush=True)
    roots = g.sample_roots(2, 4)
    g.sssp(int(roots[0]), copy=False)
    rows = []
    for r in roots:
        g.sssp(int(r), copy=False)
        s = g.stats()
        rs = g.reach_stats()
        rows.append(dict(root=int(r), ms=s["kernel_ms"], wall_ms=s["wall_ms"], bands=s["levels"],
                         rounds=s["relax_rounds"], m_r=rs["reached_edges"], n_r=rs["reached"]))
        print(f"  root {r}: {s['kernel_ms']:.2f} ms bands {s['levels']} rounds {s['relax_rounds']} "
              f"m_r {rs['reached_edges']} -> {rs['reached_edges'] / s['kernel_ms'] / 1e6:.1f} GTEPS", flush=True)
    out[f"k{scale}w"] = dict(gen_build_s=gen, solves=rows,
                            gteps=float(np.mean([x["m_r"] / x["ms"] / 1e6 for x in rows])))
    g.close()
print(json.dumps(out))
