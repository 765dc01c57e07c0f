#!/bin/bash
# weighted parity tests (light CSR build), per-round atomics counts (stats build), MS1024 profile at the
# default pass width, prep kernel stats of one k26w solve
set -o pipefail
OUT=gpurun_out/r3g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "weighted" > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stats/libpj.so timeout -k 10 200 python3 -u tools/stats_probe.py 26 2 > $OUT/stats.out 2> $OUT/stats.err || { echo stats failed; tail -5 $OUT/stats.err; exit 1; }
grep -v amdgpu $OUT/stats.err
bash tools/ms_profile.sh r3g_ms > $OUT/ms.log 2>&1 || { echo ms failed; tail $OUT/ms.log; exit 1; }
cat $OUT/ms.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/traffic_probe.py 26 1 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
head -30 $OUT/kt/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)//' 
