#!/bin/bash
# round 3: SWAR line parsing, edge-tiled light CSR build; ms tile removed, defer_heavy off:
# every -m gpu test, the ingest profile, the k26w kernel trace (prep kernels), MS1024 timing
set -o pipefail
OUT=gpurun_out/r3n; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/ingest_profile.sh r3n_ing > $OUT/ing.log 2>&1 || { echo ingest failed; tail $OUT/ing.log; exit 1; }
grep -E "parse_lines|parse_count|phase load|time_to_solution" $OUT/ing.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
tail -1 $OUT/kt.log
python3 tools/kt_summary.py $OUT/kt/run_kernel_stats.csv 1 30
timeout -k 10 300 python -u tools/probe_ms.py "" "ms_width=4" > $OUT/probe.log 2>&1 || { echo probe failed; tail $OUT/probe.log; exit 1; }
grep pass $OUT/probe.log
