"""FETCH_SIZE calibration from tools/cycle.sh's `calib` step (tools/calib/gather_calib.hip under
rocprofv3 --pmc, one pass per counter group): for each calibration kernel the requested bytes
(known: every 16-byte piece of the table once, random whole 128-byte lines, or random 4-byte
words) against the L2's memory-side read requests (TCC_EA0_RDREQ, of which 32-byte ones
TCC_EA0_RDREQ_32B, TCC_BUBBLE, TCC_EA0_RDREQ_DRAM), FETCH_SIZE and WRITE_SIZE, per launch.
Gives the bytes one non-32-byte request moves (from the random-lines kernel, where no byte
of a request is wasted), hence DRAM-side bytes = (RDREQ - RDREQ_32B) x that + RDREQ_32B x 32,
the correction pmc_solve_table.py applies to the solve's kernels, and the random-gather rate
that bounds a probe-bound kernel.
Usage: python tools/calib_table.py gpurun_out/TAG > profiles/r06/gather_calib.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
runs = [json.loads(ln) for ln in open(os.path.join(root, "calib.log")) if ln.startswith("{")]
by_name = {r["kernel"]: r for r in runs}
# dispatch order of the program: warm-up + reps launches per kernel, in the order printed
order = []
for r in runs:
    order += [r["kernel"]] * r["launches"]


def short(k):
    if "cal_stream_k" in k:
        return "stream"
    if "cal_lines_k" in k:
        return "lines"
    if "cal_dwords_k<0>" in k:
        return "dwords"
    if "cal_dwords_k<1>" in k:
        return "dwords_small"
    return None


names = {"stream": "cal_stream_k", "lines": "cal_lines_k", "dwords": "cal_dwords_k", "dwords_small": "cal_dwords_small_k"}
ctr = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
for p in glob.glob(os.path.join(root, "calpmc_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        if k:
            ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"program": "tools/calib/gather_calib.hip", "kernels": {}}
for k, full in names.items():
    if full not in by_name:
        continue
    t = by_name[full]
    c = {n: sum(v) / len(v) for n, v in ctr[k].items() if v}
    e = {"table_bytes": t["table_bytes"], "bytes_requested": t["bytes_requested_per_launch"],
         "gathers": t["gathers_per_launch"], "ms": t["ms_per_launch"], "GBps_requested": t["GBps_requested"],
         "Ggathers_per_s": t["Ggathers_per_s"], "counters_per_launch": c}
    if "FETCH_SIZE" in c:
        e["fetch_size_bytes"] = c["FETCH_SIZE"] * 1024
        e["requested_over_fetch_size"] = t["bytes_requested_per_launch"] / (c["FETCH_SIZE"] * 1024)
    out["kernels"][k] = e
L = out["kernels"].get("lines", {}).get("counters_per_launch", {})
if "TCC_EA0_RDREQ_sum" in L:
    big = L["TCC_EA0_RDREQ_sum"] - L.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    out["bytes_per_request"] = out["kernels"]["lines"]["bytes_requested"] / big
    out["rule"] = ("DRAM-side read bytes = (TCC_EA0_RDREQ_sum - TCC_EA0_RDREQ_32B_sum) x bytes_per_request + "
                   "TCC_EA0_RDREQ_32B_sum x 32 (requests served by the Infinity Cache included: an upper bound)")
    for k, e in out["kernels"].items():
        c = e["counters_per_launch"]
        if "TCC_EA0_RDREQ_sum" in c:
            rb = (c["TCC_EA0_RDREQ_sum"] - c.get("TCC_EA0_RDREQ_32B_sum", 0.0)) * out["bytes_per_request"] + \
                c.get("TCC_EA0_RDREQ_32B_sum", 0.0) * 32
            e["read_bytes_calibrated"] = rb
            if e["gathers"]:
                e["read_bytes_per_gather"] = rb / e["gathers"]
            if "FETCH_SIZE" in c:
                e["calibrated_over_fetch_size"] = rb / (c["FETCH_SIZE"] * 1024)
D = out["kernels"].get("dwords", {})
if D:
    out["random_dword_gathers_per_s"] = D["Ggathers_per_s"] * 1e9
json.dump(out, sys.stdout, indent=1)
print()
