#!/bin/bash
# round 3 (final checkpoint): the round cycle (every -m gpu test, the default bench line with the k26w world-2
# host-transport leg, its kernel trace, FETCH/WRITE passes), smoke, per-kernel PMC table
set -o pipefail
OUT=gpurun_out/r3ah; mkdir -p $OUT
bash tools/gpu_round.sh r3ah_round || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 gpurun_out/r3ah_round/pytest_gpu.log
python3 tools/pmc_solve_table.py gpurun_out/r3ah_round > $OUT/pmc_table.txt 2>&1
python3 tools/traffic_json.py gpurun_out/r3ah_round > $OUT/traffic_k26w.json 2>&1
python3 -c "import json; d=json.load(open('gpurun_out/r3ah_round/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['time_to_solution_s'], d['time_to_solution_phases']['in_process_breakdown'], d['secondary']['wg']['ms_per_sssp'], d['secondary']['ms1024']['batch_ms']); print(d['secondary'].get('k26w_partitioned_host_w2')); print(d['secondary'].get('k28_partitioned_host_w2'))"
