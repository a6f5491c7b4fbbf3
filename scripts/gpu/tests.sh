#!/bin/bash
# GPU parity suite on the box: pytest -m gpu (optionally a -k filter), log under gpurun_out/.
# usage: scripts/gpu/tests.sh [pytest -k expression] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
TAG=${2:-all}
ARGS=(tests -m gpu ${XFLAG--x} -v -s --timeout 600 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 1100 python -u -m pytest "${ARGS[@]}" > gpurun_out/tests_${TAG}.log 2>&1
rc=$?
tail -40 gpurun_out/tests_${TAG}.log
exit $rc
