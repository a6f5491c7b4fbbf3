#!/bin/bash
# rocprofv3 kernel trace (every dispatch, in order) of a short bench run -> gpurun_out/trace_TAG.csv
# usage: trace.sh TAG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
LEAN="--cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --tail-probe 0 --strong-batches 0 --c1-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_$TAG -o run --output-format csv -- \
  python3 bench.py $LEAN "$@" > gpurun_out/trace_$TAG.json 2> gpurun_out/trace_$TAG.err || { tail -20 gpurun_out/trace_$TAG.err; exit 1; }
f=$(find gpurun_out/tr_$TAG -name '*kernel_trace.csv' | head -1)
python3 - "$f" gpurun_out/trace_$TAG.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
with open(sys.argv[2], "w") as f:
    for r in rows:
        f.write(f'{r["Start_Timestamp"]},{r["End_Timestamp"]},{r["Kernel_Name"][:90]}\n')
print(len(rows), "dispatches")
PY
rm -rf gpurun_out/tr_$TAG
