#!/bin/bash
# round 3 first cycle: the new tests first, then every gpu test, then the default bench line
set -o pipefail
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  "tests/test_tree.py" "tests/test_gpu_parity.py::test_kronecker_csr_s20_exact" \
  "tests/test_gpu_parity.py::test_kronecker_csr_s26w_full_size_digest" \
  "tests/test_gpu_parity.py::test_partitioned_weighted_s22_world2" \
  "tests/test_gpu_parity.py::test_partitioned_bfs_s28_full_size" -m gpu > $OUT/new_tests.log 2>&1 || { echo new tests failed; tail -40 $OUT/new_tests.log; exit 1; }
tail -3 $OUT/new_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
