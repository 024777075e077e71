#!/bin/bash
# A/B driver for bench.py runs (replaces the round-1 one-off tools/_*.sh).
#
#   RUNS='label|ENV=1 ENV2=x|--workload 1080p_d128 --steps 20;label2||--workload 1080p_d192' \
#   REPS=2 tools/bench_ab.sh
#
# Each run is "label|environment assignments|bench.py arguments".  An
# alternative library build is selected with SVA_LIB_PATH=<path to .so> in the
# environment field (stereovisionarray_amd/__init__.py loads it); the in-tree
# product library is never overwritten.  Runs are interleaved REPS times so
# box-level drift hits every variant alike.  Output: one line per run with
# the bench value and per-kernel times; logs under gpurun_out/ab_<label>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
: "${RUNS:?set RUNS='label|env|bench args;...'}"
REPS=${REPS:-1}
IFS=';' read -ra SPECS <<< "$RUNS"
for ((r = 0; r < REPS; r++)); do
  for spec in "${SPECS[@]}"; do
    IFS='|' read -r label envs args <<< "$spec"
    log="gpurun_out/ab_${label}.log"
    # shellcheck disable=SC2086
    env $envs timeout -k 10 "${TIMEOUT:-300}" python bench.py --no-cpu-baseline $args > "$log" 2>&1
    rc=$?
    echo "$label rep=$r rc=$rc $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"kernels_ms": {[^}]*}' "$log")"
    if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
  done
done
