"""configs[2]'s graph as bench.py's k26w_partitioned_host_w2: the weighted partition at world 2, both ranks
in this process on one GPU over the host transport, 3 roots (sample_roots seed 2); ms per SSSP under
wpart option sets, interleaved. Usage: python tools/k26w_part_w2.py [scale=26] [passes=2]
[sets=default+grid_per_cu=4]  (a set: k=v/k=v..., "default" = none)"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402
from paralleljohnson_amd.partition import Comm, delta_group, load_weighted_kronecker  # noqa: E402

opts = dict(kv.split("=", 1) for kv in sys.argv[1:])
scale = int(opts.get("scale", "26"))
passes = int(opts.get("passes", "2"))
sets = [{} if x == "default" else dict(kv.split("=") for kv in x.split("/"))
        for x in opts.get("sets", "default+grid_per_cu=4").split("+")]
ctxs = [pj.Context(0) for _ in range(2)]
comms = Comm.group(ctxs, "host")
g = ctxs[0].generate_kronecker(scale, 16, 1, weighted=True)
roots = [int(x) for x in g.sample_roots(2, 3)]
g.close()
parts = [load_weighted_kronecker(ctxs[r], scale, 16, 1, r, 2) for r in range(2)]
base = {"grid_per_cu": 8}
for ps in range(passes):
    for o in sets:
        for p in parts:
            for k, v in {**base, **o}.items():
                p.set_option(k, float(v))
        delta_group(parts, comms, roots[0])  # (warm)
        t = time.perf_counter()
        for r in roots:
            delta_group(parts, comms, r)
        ms = 1e3 * (time.perf_counter() - t) / len(roots)
        print(f"pass {ps} {o or 'default'} ms per SSSP {ms:.3f}", flush=True)
for p in parts:
    p.close()
for c in comms:
    c.close()
