#!/bin/bash
# round 3: relabel copy writes u8 weights and reduces sum / max (no wsummax / w8 passes);
# TTS process before the main leg. Every -m gpu test, the default bench line, a kernel +
# HIP API trace of two k26w solves (prep gaps)
set -o pipefail
OUT=gpurun_out/r3u; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['time_to_solution_s'], d['time_to_solution_phases']); print(d['secondary']['wg']['ms_per_sssp'], d['secondary']['ms1024']['batch_ms'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/ht -o run -- python3 tools/stats_probe.py 26 2 > $OUT/ht.log 2>&1 || { echo ht failed; tail $OUT/ht.log; exit 1; }
echo r3u ok
