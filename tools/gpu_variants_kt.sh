#!/bin/bash
# Kernel-trace each tuning variant: bash tools/gpu_variants_kt.sh TAG "probe args" v1 v2 ...
set -o pipefail
TAG=$1; shift; ARGS=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 $ARGS > $OUT/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v: $(grep -v amdgpu.ids $OUT/$v.log | grep -E 'mean|gteps' | tail -2)"
done
