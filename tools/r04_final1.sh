#!/bin/bash
# Round 4 final tree: full GPU suite, then bench + kernel trace (C4, C3) + PMC passes (tools/gpu_profile.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/gpu_tests.sh r04_final2_tests "" 600 || exit 1
bash tools/gpu_profile.sh r04_prof2 || exit 1
