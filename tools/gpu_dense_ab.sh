#!/bin/bash
# Dense MFMA Gram A/B on the GPU box: one process per arm (knobs are read once per process).
# usage: bash tools/gpu_dense_ab.sh OUT "ARM_ENV ..." n ...   (ARM_ENV: VAR=v,VAR2=w or "base")
set -o pipefail
out=$1; shift
arms=$1; shift
mkdir -p "$(dirname "$out")"
for arm in $arms; do
  envs=()
  if [ "$arm" != base ]; then IFS=, read -ra envs <<< "$arm"; fi
  env "${envs[@]}" timeout -k 10 300 python tools/dense_ab.py --label "$arm" "$@" >> "$out" 2>&1 || { echo "arm $arm failed rc=$?" >> "$out"; exit 1; }
done
