#!/bin/bash
# Round 6: the exec-score helper waves of the dr_lds50 unit (decima_policy.h dp_exec_tiles). The Decima rollout tests
# that run it (the device collector against the lockstep one, bit for bit), then the PPO iteration A/B of the HEAD
# build (build/ab/base.so) against this one (build/ab/help.so), then the lone-wave phase profile. Each step has its own
# time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${HELP_STEPS:-tests ab phase}
case " $S " in *" tests "*)
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_build_id.py tests/test_gpu_layout.py tests/test_decima_policy.py tests/test_trainers.py \
    tests/test_gpu_timed_paths.py \
    -k "build or lds_within_share or decima_fused or device_collector or rejected_action or preempted_collection or small_batch_replay or learner_matches" \
    > gpurun_out/help_tests.log 2>&1 || { tail -30 gpurun_out/help_tests.log; exit 1; }
  tail -3 gpurun_out/help_tests.log;;
esac
case " $S " in *" ab "*) AB_OUT=ab AB_REPS=${AB_REPS:-2} bash scripts/ab_ppo.sh || exit $?;; esac
case " $S " in *" abdec "*)
  mkdir -p gpurun_out/ab
  for rep in 1 2; do for n in ${ABDEC_LIBS:-base edge}; do
    SSIM_LIB=$PWD/gym-sparksched_amd/build/ab/$n.so timeout -k 10 300 python bench.py --workload decima --steps 40 \
      --warmup 5 --no-cpu-baseline > gpurun_out/ab/${n}_decima_$rep.log 2>&1 || exit $?
    echo "$n decima rep$rep $(grep '^{' gpurun_out/ab/${n}_decima_$rep.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["value"]))')"
  done; done;;
esac
case " $S " in *" phase "*)
  SSIM_PROF_LIB=$PWD/gym-sparksched_amd/build/libsparksched_prof_fine.so PROF_ENVS=16 PROF_STEPS=300 timeout -k 10 600 python scripts/phase_profile_decima.py > gpurun_out/phase_decima_fine16.txt 2>&1 || exit $?;;
esac
echo "=== r6_help done"
