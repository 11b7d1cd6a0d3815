#!/bin/bash
# One parameterised GPU batch for the box (run from the repo root; it replaces round 5's
# one-off tools/gpu_r05[a-m].sh).  Steps run in the order given, each under its own time limit,
# and the first failure ends the batch (no GPU step after a fault or a timeout):
#   bash tools/gpu_batch.sh STEP [STEP ...]
# steps:
#   tests:FILE[,FILE...]   pytest those files (-x, 120 s per test) -> gpurun_out/tests.log
#   suite                  the whole -m gpu suite -> gpurun_out/suite.log
#   smoke                  __graft_entry__.smoke()
#   prof:TAG[:PAT,...]     rocprofv3 --kernel-trace --stats of 3 bench steps -> gpurun_out/prof_TAG,
#                          then the kernels whose names contain a PAT (tools/db_kernels.py)
#   ab:VARIANT[:GREP]      same-box step A/B against abtest/VARIANT/libpcs.so (tools/ab_lib_step.sh)
#   bench[:ARG,...]        one bench.py line (commas stand for spaces) -> gpurun_out/bench.json
#   evidence:TAG           tools/evidence_round.sh TAG (suite, smoke, bf16 + fp8 rocprof / PMC passes)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  echo "== $step"
  case $kind in
    tests)
      timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${arg//,/ } \
        > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
      tail -1 gpurun_out/tests.log ;;
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread \
        > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
      tail -1 gpurun_out/suite.log ;;
    smoke)
      timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 ;;
    prof)
      tag=${arg%%:*}
      pats=${arg#*:}
      [ "$pats" = "$arg" ] && pats=""
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
      python3 tools/db_kernels.py gpurun_out/prof_$tag/run_results.db ${pats//,/ } ;;
    ab)
      var=${arg%%:*}
      grep_=${arg#*:}
      [ "$grep_" = "$arg" ] && grep_=""
      VAR=$var GREP="${grep_:-fwd:global_feat\|dgrad:global_feat}" bash tools/ab_lib_step.sh ;;
    bench)
      timeout -k 10 400 python -u bench.py ${arg//,/ } > gpurun_out/bench.json 2> gpurun_out/bench.err
      tail -1 gpurun_out/bench.json; grep -A16 per-kernel gpurun_out/bench.err || true ;;
    evidence)
      bash tools/evidence_round.sh $arg ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
