#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 invocation; --pmc never combined with
# sys/runtime traces). Writes under gpurun_out/pmc/<pass>/. Stops at the first fault-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${PMC_MODE:-rollout}
# default: the driver's bench command (bench.py --steps 20 --warmup 5)
if [ "$MODE" = rollout ]; then ARGS=${PMC_ARGS:-"--steps 20 --warmup 5"}; else ARGS=${PMC_ARGS:-"--steps 100 --warmup 20"}; fi
OUT=gpurun_out/pmc_${PMC_TAG:-$MODE}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  echo "=== pmc $name ($(date +%T))"
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d "$PWD/$OUT/$name" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --mode "$MODE" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$name.log"; exit $rc; fi
}
PASSES=${PMC_PASSES:-waves icache fetch write}
want() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
want waves && run waves SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM
want icache && run icache SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVES
want fetch && run fetch FETCH_SIZE
want write && run write WRITE_SIZE
# mean latency per issued LDS / vector-memory / scalar-memory instruction = LEVEL / INSTS
want latency && run latency SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES
echo "=== pmc done"
