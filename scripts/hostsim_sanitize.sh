#!/bin/bash
# Host-side sanitizer run of the engine (tests/hostsim: the same engine.h compiled for the CPU with a one-lane wave):
# the diagnostic profile build (-DSSIM_PROFILE) and the product build, each under ASan + UBSan, through the
# CPU parity suite's lockstep / rollout / reset cases. Usage: scripts/hostsim_sanitize.sh [pytest -k expression]
set -euo pipefail
cd "$(dirname "$0")/.."
K="${1:-lockstep or rollout_replay or autoreset or sampled_reset or invalid}"
ASAN="$(gcc -print-file-name=libasan.so)"
UBSAN="$(gcc -print-file-name=libubsan.so)"
for variant in profile product; do
  so="/tmp/_hostsim_san_${variant}.so"
  flags="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
  [ "$variant" = profile ] && flags="$flags -DSSIM_PROFILE"
  rm -f "$so"
  echo "== hostsim $variant build under ASan/UBSan: $flags"
  HOSTSIM_SO="$so" HOSTSIM_FLAGS="$flags" LD_PRELOAD="$ASAN:$UBSAN" ASAN_OPTIONS=detect_leaks=0 \
    python -m pytest tests/test_hostsim_parity.py -x -q -p no:cacheprovider -k "$K"
done
