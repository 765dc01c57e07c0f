#!/bin/bash
# A/B of libpj variants (paralleljohnson_amd/lib/variants/<v>/libpj.so; "default" = main build) on
# one probe: bash tools/ab_variants.sh TAG "script args" v1 v2 ...  (interleaved twice)
set -o pipefail
TAG=$1; shift; ARGS=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for pass in $(seq 1 ${PASSES:-2}); do
  for v in "$@"; do
    if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
    timeout -k 10 150 python3 -u $ARGS > $OUT/$v.$pass.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.$pass.log; exit 1; }
    echo "== $v pass $pass: $(grep -v Warn $OUT/$v.$pass.log | grep -v amdgpu.ids | tail -2 | tr '\n' ' ')"
  done
done
