#!/bin/bash
# this session's GPU call (see scripts/gpu_check.sh for the step definitions)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh smoke pytestall bench_driver bench
