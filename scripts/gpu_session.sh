#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTEST_K="preempted_collection"
bash scripts/gpu_check.sh pytestk
