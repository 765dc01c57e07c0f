#!/bin/bash
# round 3: heavy head (first heavy edges of every row, vertex-major) -- weighted parity tests,
# A/B heavy_head 1/0, heavy-pull scan lengths (pstats debug build); then the round cycle: every
# -m gpu test, smoke, the default bench line, its kernel trace and FETCH/WRITE passes
set -o pipefail
OUT=gpurun_out/r3p; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "weighted or s26w" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PASSES=2 bash tools/ab_opts.sh r3p_ab "" "--opt heavy_head=0" || exit 1
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/pstats/libpj.so timeout -k 10 200 python3 -u tools/stats_probe.py 26 3 > $OUT/pstats.out 2> $OUT/pstats.err || { echo pstats failed; tail -5 $OUT/pstats.err; exit 1; }
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/pstats/libpj.so timeout -k 10 200 python3 -u tools/stats_probe.py 26 3 heavy_head=0 > $OUT/pstats0.out 2> $OUT/pstats0.err || { echo pstats failed; tail -5 $OUT/pstats0.err; exit 1; }
grep -h -E "heavy pulls" $OUT/pstats.err $OUT/pstats0.err
bash tools/gpu_round.sh r3p_round || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 gpurun_out/r3p_round/pytest_gpu.log
python3 -c "import json; d=json.load(open('gpurun_out/r3p_round/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['time_to_solution_s'], d['time_to_solution_phases']['in_process_breakdown'], d['secondary']['wg']['ms_per_sssp'], d['secondary']['ms1024']['batch_ms'])"
