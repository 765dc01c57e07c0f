#!/bin/bash
# Sweep tuning variants (paralleljohnson_amd/lib/variants/<v>/libpj.so) with a probe script.
# Usage: bash tools/gpu_variants.sh TAG "probe args" v1 v2 ...   (v = default for the main build)
set -o pipefail
TAG=$1; shift; ARGS=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  timeout -k 10 200 python -u $ARGS > $OUT/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v: $(grep -o '"gteps": [0-9.]*' $OUT/$v.log | tail -1)"
done
