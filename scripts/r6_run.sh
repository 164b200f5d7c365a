#!/bin/bash
# Round-6 GPU session: a pytest selection (PYTEST_K) plus the listed gpu_check.sh steps; PMC passes per PMC_PASSES.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PMC_PASSES=${PMC_PASSES:-"fetch write"}
bash scripts/gpu_check.sh "$@"
