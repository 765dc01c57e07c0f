#!/bin/bash
# round 3: relabel temporaries in one allocation + delta module loaded behind the copy:
# weighted tests, k26w line (solver_prep_s), kernel + HIP API trace of the preparation;
# web-Google level stamps (PJ_BFS_STAMPS build) with and without the one-workgroup levels
set -o pipefail
OUT=gpurun_out/r3v; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "weighted or s26w or kronecker" > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline --no-partitioned > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['time_to_solution_s'], d['time_to_solution_phases'])"
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stamps/libpj.so timeout -k 10 120 python3 -u tools/probe_wg.py > $OUT/stamps1.out 2> $OUT/stamps1.err || { echo stamps failed; tail $OUT/stamps1.err; exit 1; }
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stamps/libpj.so timeout -k 10 120 python3 -u tools/probe_wg.py bfs_small=0 > $OUT/stamps0.out 2> $OUT/stamps0.err || { echo stamps failed; tail $OUT/stamps0.err; exit 1; }
grep stamps $OUT/stamps1.err | tail -12
grep stamps $OUT/stamps0.err | tail -16
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/ht -o run -- python3 tools/stats_probe.py 26 2 > $OUT/ht.log 2>&1 || { echo ht failed; tail $OUT/ht.log; exit 1; }
echo r3v ok
