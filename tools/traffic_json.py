"""HBM traffic per solve from the FETCH_SIZE / WRITE_SIZE passes of tools/cycle.sh (pmc step)
(rocprofv3 --pmc over tools/traffic_probe.py): sum of the solve kernels' counters (KB)
per solve, 2 x FETCH_SIZE + WRITE_SIZE in bytes (MI355X_MICROARCH.md HBM section).
Usage: python tools/traffic_json.py gpurun_out/TAG > profiles/traffic_k26w.json"""
import csv, glob, json, os, sys
from collections import defaultdict

PATTERNS = ["v2_", "unlabel_k"]
EXCLUDED = ["v2_interleave", "v2_light_csr", "v2_long", "v2_wmax", "v2_haslight", "v2_w8"]
root = sys.argv[1]
out = {}
disp = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    tot, solves, n = 0.0, 0, 0
    per = defaultdict(float)
    for p in glob.glob(os.path.join(root, f"pmc_{c}", "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if "v2_init_k" in k or "v2_source_k" in k:  # one per solve
                solves += 1
            if any(s in k for s in PATTERNS) and not any(s in k for s in EXCLUDED):
                tot += float(r["Counter_Value"])
                n += 1
    out[c] = tot / max(solves, 1)
    disp[c] = n / max(solves, 1)
out["dispatches_per_solve"] = disp
out["patterns"], out["excluded"] = PATTERNS, EXCLUDED
out["hbm_bytes_per_sssp"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
out["hbm_bytes_per_sssp_uncorrected"] = (out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
print(json.dumps(out, indent=1))
