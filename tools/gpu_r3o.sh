#!/bin/bash
# round 3: parse outputs staged through LDS (coalesced stores), fused weight sum/max: ingest and
# weighted tests, the ingest profile, the k26w line (solver_prep_s); MS-BFS build variants
# (lines per lane step MS_U, workgroups per CU) on MS1024
set -o pipefail
OUT=gpurun_out/r3o; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_ingest.py tests/test_multisource.py tests/test_csr_cache.py -k "appendix or parse or cli or csr or text or weighted or chain or cache or multi" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/ingest_profile.sh r3o_ing > $OUT/ing.log 2>&1 || { echo ingest failed; tail $OUT/ing.log; exit 1; }
grep -E "parse_lines|parse_count|time_to_solution" $OUT/ing.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 16 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['time_to_solution_s'], d['time_to_solution_phases']['in_process_breakdown'])"
PASSES=1 bash tools/ab_variants.sh r3o_ms "tools/probe_ms.py" default msu4 msu2 msg8 msu4g8 || exit 1
