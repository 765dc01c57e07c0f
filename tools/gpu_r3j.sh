#!/bin/bash
# round 3: every -m gpu test, smoke, the default bench line, then the profiles of the parse
# (per-block max ids), relabel (edge tiles: variants) and MS-BFS (sharded counter, no distance
# fill) changes, and the k26w kernel trace + FETCH/WRITE passes
set -o pipefail
OUT=gpurun_out/r3j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
bash tools/ingest_profile.sh r3j_ing > $OUT/ing.log 2>&1 || { echo ingest failed; tail $OUT/ing.log; exit 1; }
tail -30 $OUT/ing.log
bash tools/kt_variants.sh r3j_rl "tools/stats_probe.py 26 2" default rl0 rl2 rl4 > $OUT/rl.log 2>&1 || { echo rl failed; tail $OUT/rl.log; exit 1; }
grep -E "==|copy_" $OUT/rl.log
bash tools/ms_profile.sh r3j_ms > $OUT/ms.log 2>&1 || { echo ms failed; tail $OUT/ms.log; exit 1; }
tail -25 $OUT/ms.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 tools/traffic_probe.py 26 4 1 > $OUT/pmc_$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
echo r3j ok
