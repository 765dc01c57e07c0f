#!/bin/bash
# round 3: fold_hub (light rounds relax the previous round's hub tiles, no hub launch per round):
# weighted parity + multi-source tests, A/B against its own hub launches and light_pull neighbours,
# then one solve's timeline with the fold
set -o pipefail
OUT=gpurun_out/r3k; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_multisource.py -k "weighted or binned or band or tail or s26w or multisource or ms" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PASSES=2 bash tools/ab_opts.sh r3k_ab "" "--opt fold_hub=0" "--opt light_pull=2.5" "--opt light_pull=4" || exit 1
bash tools/kt_opts.sh r3k_kt "" || exit 1
python3 tools/trace_solve.py gpurun_out/r3k_kt_0/kt_kernel_trace.csv 3 v2_init_k > $OUT/tl.txt; cat $OUT/tl.txt
