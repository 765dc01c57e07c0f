#!/bin/bash
# round 3: edge-tiled MS-BFS pulls (ms_tile), padded parse window (dword reads), deferred heavy
# edges (defer_heavy): their parity tests, then MS1024 timing ms_tile 1/0, the k26w A/B of
# defer_heavy, the CLI ingest profile and the MS1024 per-kernel profile
set -o pipefail
OUT=gpurun_out/r3m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_multisource.py tests/test_ingest.py -k "msbfs or multi or batch or ms1024 or weighted or appendix or parse or cli or csr or s26w" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/probe_ms.py "" "ms_tile=0" > $OUT/probe.log 2>&1 || { echo probe failed; tail $OUT/probe.log; exit 1; }
grep pass $OUT/probe.log
PASSES=2 bash tools/ab_opts.sh r3m_ab "" "--opt defer_heavy=0" || exit 1
bash tools/ingest_profile.sh r3m_ing > $OUT/ing.log 2>&1 || { echo ingest failed; tail $OUT/ing.log; exit 1; }
grep -E "parse_lines|parse_count|phase load" $OUT/ing.log
bash tools/ms_profile.sh r3m_ms > $OUT/ms.log 2>&1 || { echo ms failed; tail $OUT/ms.log; exit 1; }
tail -22 $OUT/ms.log
bash tools/kt_opts.sh r3m_kt "" || exit 1
python3 tools/trace_solve.py gpurun_out/r3m_kt_0/kt_kernel_trace.csv 3 v2_init_k > $OUT/tl.txt; tail -45 $OUT/tl.txt
