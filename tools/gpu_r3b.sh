#!/bin/bash
# round 3: parse / ingest / tree tests, per-round stats of k26w (default and tail_pull), A/B of tail_pull,
# CLI ingest profile (parse_lines_k), kernel trace of the k26w bench (copy_rows_k)
set -o pipefail
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ingest.py tests/test_tree.py \
  tests/test_gpu_parity.py -k "appendix or parse or cli or weighted or tail or chain" > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for o in "" "tail_pull=1"; do
  PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stats/libpj.so timeout -k 10 200 python3 -u tools/stats_probe.py 26 2 $o > $OUT/stats_$o.out 2> $OUT/stats_$o.err || { echo stats failed; tail -5 $OUT/stats_$o.err; exit 1; }
  cat $OUT/stats_$o.out
done
PASSES=2 bash tools/ab_opts.sh r3b_ab "" "--opt tail_pull=1" || exit 1
bash tools/ingest_profile.sh r3b_ing > $OUT/ing.log 2>&1 || { echo ingest failed; tail $OUT/ing.log; exit 1; }
tail -30 $OUT/ing.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
head -25 $OUT/kt/run_kernel_stats.csv
