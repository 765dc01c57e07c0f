#!/bin/bash
# weighted + partition gpu tests, then the k26w profile set: bench kernel trace (timeline), the PMC
# traffic passes over tools/traffic_probe.py (per-kernel table + profiles/traffic_k26w.json input)
set -o pipefail
TAG=${1:-r3c}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py \
  tests/test_gpu_parity.py -k "weighted or part" > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bkt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/bkt.log 2>&1 || { echo bkt failed; exit 1; }
grep -v amdgpu $OUT/bkt.log | tail -1 | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/traffic_probe.py 26 4 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 tools/traffic_probe.py 26 4 1 > $OUT/pmc_$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
python3 tools/traffic_json.py $OUT > $OUT/traffic.json && python3 tools/pmc_kernel_table.py $OUT > $OUT/pmc_table.txt
cat $OUT/pmc_table.txt
python3 tools/trace_solve.py $OUT/bkt/run_kernel_trace.csv -2 v2_init_k > $OUT/timeline.txt; cat $OUT/timeline.txt
