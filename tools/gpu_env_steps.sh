#!/bin/bash
# tools/gpu_steps.sh with per-step environment: each argument is "<VAR=value,...>|<gpu_steps.sh step>"
# ("-|<step>" for none); the steps run in order under the same tag and stop at the first failure.
# usage: tools/gpu_env_steps.sh <tag> "<env>|<step>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
for st in "$@"; do
    envs=${st%%|*}; step=${st#*|}
    (
        if [ "$envs" != "-" ]; then
            IFS=',' read -ra kv <<< "$envs"
            for x in "${kv[@]}"; do export "$x"; done
        fi
        bash "$R/tools/gpu_steps.sh" "$TAG" "$step"
    ) || exit 1
done
echo "all env steps ok"
