#!/bin/bash
# Register / scratch / LDS usage of every engine kernel of one translation unit (compiler remarks), e.g.
#   scripts/resource_usage.sh k_bench900.hip [extra hipcc flags]
set -euo pipefail
cd "$(dirname "$0")/.."
TU=${1:-k_bench900.hip}; shift || true
SCHED=""
case "$TU" in k_bench900.hip|k_bench.hip|k_lds.hip) SCHED="-mllvm -amdgpu-sched-strategy=iterative-ilp";; esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $SCHED "$@" -Iinclude -Igym-sparksched_amd/csrc \
  --offload-device-only -c -o /tmp/_ru.o "gym-sparksched_amd/csrc/$TU" -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|SGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs Spill|VGPRs Spill" | sed 's/^.*remark: //'
