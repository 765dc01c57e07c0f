"""Interleaved A/B of libpj BFS options on the web-Google-shaped synthetic (configs[0]: source 0
and 7 sampled roots) and Kronecker s22 (configs[1]): median kernel ms per option set, every
variant's distances checked bit-exact against the first set's. Option sets are ';'-separated
lists of key=value (default: "bfs_mid=0;bfs_mid=1").
Usage: python tools/bfs_mid_ab.py [graphs=wg,k22] [sets="bfs_mid=0;bfs_mid=1"] [reps=6]"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

opts = dict(kv.split("=", 1) for kv in sys.argv[1:])
graphs = opts.get("graphs", "wg,k22").split(",")
sets = [dict(kv.split("=") for kv in s.split(",") if kv) for s in opts.get("sets", "bfs_mid=0;bfs_mid=1").split(";")]
reps = int(opts.get("reps", "6"))
ctx = pj.Context(0)
for name in graphs:
    if name == "wg":
        g = ctx.generate_webgraph()
        roots = [0] + [int(r) for r in g.sample_roots(7, 3)]
    else:
        g = ctx.generate_kronecker(22, 16, 1)
        roots = [int(r) for r in g.sample_roots(7, 8)]
    ref = {r: g.sssp(r) for r in roots}
    times = [[] for _ in sets]
    levels = [None] * len(sets)
    for rep in range(reps):
        for i, st in enumerate(sets):
            for k, v in st.items():
                g.set_option(k, float(v))
            lv = []
            for r in roots:
                d = g.sssp(r, copy=(rep == 0))
                if rep == 0:
                    assert np.array_equal(d, ref[r]), (name, st, r)
                s = g.stats()
                times[i].append(s["kernel_ms"])
                lv.append((s["levels"], s["td_levels"], s["bu_levels"]))
            levels[i] = lv
    for i, st in enumerate(sets):
        print(f"{name} {st}: median kernel_ms {np.median(times[i]):.4f} min {np.min(times[i]):.4f} "
              f"levels(td,bu) root0 {levels[i][0]}", flush=True)
    g.close()
print("bfs_mid_ab: all variants bit-identical")
