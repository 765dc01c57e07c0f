#!/bin/bash
# Kernel-trace stats of one probe under several libpj builds:
# bash tools/kt_variants.sh TAG "probe.py args" v1 v2 ...   (v = default for the main build)
set -o pipefail
TAG=$1; shift; ARGS=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 -u $ARGS > $OUT/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v: $(grep -v amdgpu.ids $OUT/$v.log | tail -3 | tr '\n' ' ')"
  python3 tools/kt_summary.py $OUT/$v/run_kernel_stats.csv 1 10 || true
done
