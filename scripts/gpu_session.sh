#!/bin/bash
# this session's GPU call (see scripts/gpu_check.sh for the step definitions)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_TAG=s20 AB_ARGS="--steps 20 --warmup 5" AB_REPS=3 timeout -k 10 600 bash scripts/ab_tpch.sh || exit $?
AB_TAG=s300 AB_ARGS="--steps 300 --warmup 50" AB_REPS=2 timeout -k 10 600 bash scripts/ab_tpch.sh
