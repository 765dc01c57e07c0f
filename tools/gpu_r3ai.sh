#!/bin/bash
# round 3: weighted partition heavy pull with WP_HPU probes per lane step (default build 1;
# variants hpu2, hpu4): partition tests on hpu2, then probe_wpart s26w default / hpu2 / hpu4 twice
set -o pipefail
OUT=gpurun_out/r3ai; mkdir -p $OUT
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/hpu2/libpj.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_gpu_parity.py -k "wpart or weighted_s22" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for pass in 1 2; do
  for v in default hpu2 hpu4; do
    if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u tools/probe_wpart.py 26 "0.1,4,0" > $OUT/w26_${v}_$pass.log 2>&1 || { echo probe failed; tail $OUT/w26_${v}_$pass.log; exit 1; }
    echo "== $v pass $pass"; grep world $OUT/w26_${v}_$pass.log
  done
done
echo r3ai ok
