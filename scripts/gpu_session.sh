#!/bin/bash
# this session's GPU call (see scripts/gpu_check.sh for the step definitions)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTEST_K="decima or persistent or device_collector or ppo"
bash scripts/gpu_check.sh pytestk bench_decima bench_ppo
