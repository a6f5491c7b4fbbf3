#!/bin/bash
# Round-3 artifacts on the final tree: the -m gpu suite, then kernel stats + PMC traffic of
# C2 / C3 / C3 B=8192 / C5 / C5 B=1024 (profiles/r03/<tag>_pmc.json, tagged with the source
# hash so the bench lines pick them up), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out profiles/r03
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  XFLAG= bash scripts/gpu/tests.sh "" final3; rc=$?; [ $rc -le 1 ] || exit $rc
fi
ROUND=r03 bash scripts/gpu/profile.sh c2 c2 --c1-reps 0 || exit 1
ROUND=r03 bash scripts/gpu/profile.sh c3 c3 --c1-reps 0 || exit 1
ROUND=r03 bash scripts/gpu/profile.sh c3 c3_b8192 --batch-size 8192 --c1-reps 0 || exit 1
ROUND=r03 bash scripts/gpu/profile.sh c5 c5 --c1-reps 0 || exit 1
ROUND=r03 bash scripts/gpu/profile.sh c5 c5_b1024 --batch-size 1024 --c1-reps 0 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/final3_bench.json 2> gpurun_out/final3_bench.err || { tail -30 gpurun_out/final3_bench.err; exit 1; }
cat gpurun_out/final3_bench.json
