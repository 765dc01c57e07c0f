#!/bin/bash
# BFS parity subset, WG stress, direction-auto timing and a WG kernel trace
set -o pipefail
OUT=gpurun_out/${1:-bfs}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "random_graphs or s22_full or webgraph or kronecker" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/bfs_stress.py graph=wg reps=4 > $OUT/stress.txt 2>&1 || { grep -v amdgpu $OUT/stress.txt | cut -c1-300 | tail; exit 1; }
tail -n 1 $OUT/stress.txt
timeout -k 10 100 python3 -u tools/bfs_time.py dirs=0 > $OUT/time.txt 2>&1 || { tail -5 $OUT/time.txt; exit 1; }
grep -v amdgpu $OUT/time.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 tools/probe_wg.py > $OUT/kt.txt 2>&1 || exit 1
python3 tools/trace_levels.py $OUT/kt/kt_kernel_trace.csv 12 | tail -13
