#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over one probe command.
# Usage: bash tools/pmc_probe.sh TAG "python3 tools/probe_one.py 26 light_pull=2"
TAG=$1; CMD=$2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 100 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -3 "$OUT/p$i.log"; exit 1; }
  i=$((i+1))
done
echo pmc done
