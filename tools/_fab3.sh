#!/bin/bash
# experiment: in-process A/B of fused path-kernel builds in ablibs/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_paths.py ${LIBS} --entry fused --iters 20 ${ABARGS:-}
