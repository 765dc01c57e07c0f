#!/bin/bash
set -o pipefail
TAG=${1:-w26}; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/probe_weighted_scales.py 26 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/probe_weighted_scales.py 26 > $OUT/p$i.log 2>&1 || { echo "pmc $i failed"; exit 1; }
  i=$((i+1))
done
echo w26 ok
