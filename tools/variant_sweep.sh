#!/bin/bash
# Time the group-walk tuning variants (OMPL_GPU_GROUP_VARIANT) on the SE3 probe workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
    echo "variant $v"
    OMPL_GPU_GROUP_VARIANT=$v timeout -k 10 120 python tools/knn_probe.py --modes 0 --only cfg3_se3_1e6_k10 2>&1 | grep -v amdgpu.ids || exit $?
done
