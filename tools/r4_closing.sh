#!/bin/bash
# Round-4 closing call on the final build: tools/r4_final.sh (every GPU test, smoke, the default
# bench line, tree-mode N = 1 lines), then the profiles the G change touched (cfg3 with SQ and the
# walk probe, cfg2, extras, single query, build: tools/r4_prof.sh 1) and cfg5k's trace + FETCH / WRITE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r4_final.sh || exit 1
bash tools/r4_prof.sh 1 || exit 1
bash tools/prof_workload.sh cfg5 r4_cfg5k --bitstar-knn || exit 1
echo closing-done
