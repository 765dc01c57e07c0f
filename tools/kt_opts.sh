#!/bin/bash
# Kernel traces of the k26w bench under several option sets:
# bash tools/kt_opts.sh TAG "opts1" "opts2" ...  -> gpurun_out/TAG_<i>/kt_kernel_trace.csv
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for o in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$i -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 4 --warmup 1 $o > gpurun_out/${TAG}_$i.log 2>&1 || { echo "[$o] failed"; tail -5 gpurun_out/${TAG}_$i.log; exit 1; }
  echo "[$o] -> ${TAG}_$i"
  i=$((i+1))
done
