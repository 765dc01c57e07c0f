#!/bin/bash
# round 3: hub-queue launch width (hub_gpc: workgroups per CU of v2_hub_k; ~17 of 24 hub
# launches per solve find the queue empty) -- interleaved A/B of the k26w line
set -o pipefail
PASSES=2 bash tools/ab_opts.sh r3z_ab "" "--opt hub_gpc=2" "--opt hub_gpc=1" "--opt hub_gpc=6" || exit 1
echo r3z ok
