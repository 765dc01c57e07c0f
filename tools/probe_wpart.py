"""Weighted partitioned solve (wpart.hip + engine.cpp) on Kronecker s{scale} weights 1..255 at
world 1 (no transport) and world 2 (both ranks on this GPU, host transport): per-solve time
with the tail switch, the heavy pull and the light pull rounds at their defaults and off, or under the
given (tail_frac, pull_factor, light_pull[, tail_light_pull = 3[, tail_mult = 64[, delta = 0 (auto)]]])
sets, each timed on 3 roots after one untimed warm-up solve.
Usage: python tools/probe_wpart.py [scale=26] ["tf,pf,lp[,tlp[,tm[,delta]]];..."] (";" or "/") [worlds=12]"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
from paralleljohnson_amd.partition import Comm, delta_group, load_weighted_kronecker

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
worlds = [int(c) for c in (sys.argv[3] if len(sys.argv) > 3 else "12")]
for world in worlds:
    ctxs = [pj.Context(0) for _ in range(world)]
    comms = Comm.group(ctxs, "host") if world > 1 else [Comm.for_rank(ctxs[0], 1, 0)]
    g = ctxs[0].generate_kronecker(scale, 16, 1, weighted=True)  # (the roots)
    roots = [int(x) for x in g.sample_roots(2, 3)]
    g.close()
    # each rank generates only its block's rows (pj_wpart_generate_kronecker)
    parts = [load_weighted_kronecker(ctxs[r], scale, 16, 1, r, world) for r in range(world)]
    sets = ((0.1, 4, 0), (0.1, 4, 0))
    if len(sys.argv) > 2:
        sets = [tuple(float(x) for x in t.split(",")) for t in sys.argv[2].replace("/", ";").split(";")]
    for st4 in sets:
        tf, pf, lp = st4[:3]
        tlp = st4[3] if len(st4) > 3 else 3.0
        tm = st4[4] if len(st4) > 4 else 64.0
        dl = int(st4[5]) if len(st4) > 5 else 0
        for p in parts:
            p.set_option("tail_frac", tf)
            p.set_option("pull_factor", pf)
            p.set_option("light_pull", lp)
            p.set_option("tail_light_pull", tlp)
            p.set_option("tail_mult", tm)
        delta_group(parts, comms, roots[0], dl)  # (warm-up: buffers of this option set)
        ms = []
        for r in roots:
            st = delta_group(parts, comms, r, dl)
            ms.append(max(s["solve_ms"] for s in st))
        print(f"world {world} s{scale}w tail_frac {tf} pull_factor {pf} light_pull {lp} tail_light_pull {tlp} "
              f"tail_mult {tm} delta {dl or st[0]['delta']}: mean {np.mean(ms):.2f} solve ms "
              f"{[round(x, 2) for x in ms]} bands {st[0]['bands']} rounds {st[0]['rounds']} heavy pulls "
              f"{st[0]['heavy_pulls']} light pulls {st[0]['bu_levels']} "
              f"sent {[s['sent'] for s in st]}", flush=True)
    for p in parts:
        p.close()
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
