#!/bin/bash
# Round-end profiles of the bench line's three workloads (run on the GPU box):
# rocprofv3 kernel trace + FETCH_SIZE and WRITE_SIZE passes for C1 (tag <T>),
# C2 (<T>c2) and C3 (<T>c3), each its own bench process with --extra none so
# that one profile holds one workload. tools/profile_summary.py <tag> then
# writes profiles/<tag>_{kernel_stats.csv,pmc.json,summary.md}; bench.py's
# roofline.traffic reads the matching *_pmc.json.
# usage: bash tools/round_profiles.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r03}
bash tools/profile_round.sh $T --extra none --cpu-sample 0 || exit 1
bash tools/profile_round.sh ${T}c2 --config c2 --extra none --cpu-sample 0 || exit 1
bash tools/profile_round.sh ${T}c3 --config c3 --extra none --cpu-sample 0 || exit 1
echo "profiles done"
