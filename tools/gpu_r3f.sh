#!/bin/bash
# atomics experiment: A/B of the default build against orpre / noatom (timing-only) variants
set -o pipefail
PASSES=2 bash tools/ab_variants.sh r3f "bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 16 --warmup 2" default orpre noatom noatom_orpre || exit 1
for v in default orpre noatom noatom_orpre; do python3 -c "
import json,sys
for p in (1,2):
    l=[x for x in open('gpurun_out/r3f/$v.%d.log'%p) if x.startswith('{')][-1]; d=json.loads(l); print('$v',p,d['value'],d['kernel_ms_mean'])"; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/noatom/libpj.so
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3f/kt -o run -- python3 tools/stats_probe.py 26 2 round_log=1 > gpurun_out/r3f/rlog.out 2> gpurun_out/r3f/rlog.err || exit 1
grep -v amdgpu gpurun_out/r3f/rlog.err | grep -v rocprof | head -20
python3 tools/trace_solve.py gpurun_out/r3f/kt/run_kernel_trace.csv 0 v2_init_k | head -30
