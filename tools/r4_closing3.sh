#!/bin/bash
# Round-4 third closing call (chain cull at 4 queries per wave): tools/r4_final.sh (every GPU test,
# smoke, the default bench line, tree-mode N = 1 lines), then cfg4's trace + FETCH / WRITE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r4_final.sh || exit 1
bash tools/prof_workload.sh cfg4 r4_cfg4 || exit 1
echo closing-done
