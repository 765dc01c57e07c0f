#!/bin/bash
for v in "$@"; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  echo "== variant $v"
  timeout -k 10 120 python tools/debug_pull2.py 2>&1 | tail -3
done
