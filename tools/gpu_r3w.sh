#!/bin/bash
# round 3: BFS level decision reads its state and counters in one round trip: BFS parity
# tests, web-Google level stamps (PJ_BFS_STAMPS build), bfs_time on wg, the bench's secondary legs
set -o pipefail
OUT=gpurun_out/r3w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_tree.py tests/test_multisource.py > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stamps/libpj.so timeout -k 10 120 python3 -u tools/probe_wg.py > $OUT/stamps1.out 2> $OUT/stamps1.err || { echo stamps failed; tail $OUT/stamps1.err; exit 1; }
grep stamps $OUT/stamps1.err | tail -9
timeout -k 10 200 python3 -u tools/bfs_time.py graphs=wg,k22 dirs=0 > $OUT/time.txt 2>&1 || { tail -5 $OUT/time.txt; exit 1; }
grep -v amdgpu $OUT/time.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-partitioned > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); s=d['secondary']; print(d['value'], d['ms_per_step'], d['time_to_solution_phases']['in_process_breakdown']['solver_prep_s'], s['wg']['ms_per_sssp'], s['wg']['kernel_ms_mean'], s['k22']['ms_per_sssp'], s['ms1024']['batch_ms'], s['wg_cli']['time_to_solution_s'])"
echo r3w ok
