"""MS1024 on the web-Google-shaped graph: batch wall time (median of 7) and kernel time under
libpj option sets, interleaved. Usage: python tools/probe_ms.py "k=v,k=v" "k=v" ...  ("" = defaults)"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
row, _, _ = g.get_csr()
src = [int(x) for x in np.nonzero(np.diff(row) > 0)[0][:1024]]
sets = sys.argv[1:] or [""]
DEFAULTS = {"ms_width": 0, "ms_alpha": 16}
for rep in range(2):
    for o in sets:
        opts = dict(DEFAULTS)
        for kv in filter(None, o.split(",")):
            k, v = kv.split("=")
            opts[k] = float(v)
        for k, v in opts.items():
            g.set_option(k, v)
        g.sssp_batch(src[:64], copy=False)
        g.sssp_batch(src, copy=False)
        ts, ks = [], []
        for _ in range(7):
            t = time.perf_counter(); g.sssp_batch(src, copy=False); ts.append(time.perf_counter() - t)
            ks.append(g.stats()["kernel_ms"])
        print(f"[{o}] pass {rep + 1}: batch {1e3 * np.median(ts):.2f} ms (min {1e3 * min(ts):.2f}) kernel "
              f"{np.median(ks):.2f} ms levels {g.stats()['levels']}", flush=True)
