#!/bin/bash
# One bench configuration on the box: rocprofv3 kernel stats, two PMC passes (FETCH_SIZE,
# WRITE_SIZE; parsed with the gfx950 correction by scripts/pmc_parse.py, tagged with the
# kernel-source hash), then the bench line itself.  Outputs under gpurun_out/<TAG>_*.
# usage: scripts/gpu/profile.sh CFG TAG [extra bench args...]
#   PMC=0 skips the counter passes; BENCH_ARGS_FULL overrides the final bench's args.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=$1; TAG=$2; shift 2
EXTRA="$*"
LEAN="--config $CFG --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --trainer-epochs 0 --tail-probe 0 --strong-batches 0 $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py $LEAN --steps 200 --warmup 20 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err \
  || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
cp "$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_kernel_stats.csv
rm -rf gpurun_out/prof_$TAG
python3 scripts/kstats.py gpurun_out/${TAG}_kernel_stats.csv
if [ "${PMC:-1}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- \
      python3 bench.py $LEAN --steps 100 --warmup 10 > gpurun_out/pmc_${TAG}_$C.json 2> gpurun_out/pmc_${TAG}_$C.err \
      || { tail -20 gpurun_out/pmc_${TAG}_$C.err; exit 1; }
  done
  python3 scripts/pmc_parse.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/${TAG}_pmc.json
  rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_pmc.json'));print('pmc per step', d.get('_per_step'))"
fi
# the bench line reads its PMC traffic from profiles/rNN/<name>_pmc.json of these sources
[ -f gpurun_out/${TAG}_pmc.json ] && mkdir -p profiles/${ROUND:-r02} && cp gpurun_out/${TAG}_pmc.json profiles/${ROUND:-r02}/${TAG}_pmc.json
timeout -k 10 600 python3 bench.py ${BENCH_ARGS_FULL:-$LEAN} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
