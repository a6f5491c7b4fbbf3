#!/bin/bash
# Round-3 GPU check: the full -m gpu suite (no -x: every failure listed), then the default
# bench line (driver command).  A crash / timeout of the tests stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
K=${2:-}
XFLAG= bash scripts/gpu/tests.sh "$K" "$TAG"
rc=$?
[ $rc -le 1 ] || exit $rc
[ "${BENCH:-1}" = "1" ] || exit $rc
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
tail -12 gpurun_out/${TAG}_bench.err
exit $rc
