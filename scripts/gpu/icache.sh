#!/bin/bash
# Diagnostic: instruction-cache / wait counters of the C2 step kernels, and phase stamps
# with and without the chain sweep.  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--config c2 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0 --steps 50 --warmup 10"
GTR_CHAIN_SWEEP=0 GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so timeout -k 10 300 python3 scripts/phase_timing.py --steps 30 > gpurun_out/phases_c2_nosweep.txt 2>gpurun_out/phases_nosweep.err || exit 1
cat gpurun_out/phases_c2_nosweep.txt
for SW in 1 0; do
GTR_CHAIN_SWEEP=$SW timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU \
  --kernel-trace -d gpurun_out/pmc_ic$SW -o run --output-format csv -- python3 bench.py $LEAN > gpurun_out/pmc_ic$SW.json 2> gpurun_out/pmc_ic$SW.err || { tail -5 gpurun_out/pmc_ic$SW.err; exit 1; }
python3 - <<PY
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_ic$SW/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
print('sweep=$SW')
for k, d in acc.items():
    calls = max(n[(k, c)] for c in d) / 8 if False else None
    print(k, {c: round(v) for c, v in sorted(d.items())})
PY
done
