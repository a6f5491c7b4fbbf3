#!/bin/bash
# Instruction-cache counters of the C2 step kernels (one PMC pass), per kernel and dispatch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
LEAN="--config ${1:-c2} --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 0 --tail-probe 0 --steps 50 --warmup 10"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH \
  --kernel-trace -d gpurun_out/pmc_ic -o run --output-format csv -- python3 bench.py $LEAN > gpurun_out/pmc_ic.json 2> gpurun_out/pmc_ic.err \
  || { tail -5 gpurun_out/pmc_ic.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_ic/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    nm = r['Kernel_Name']
    k = (nm.split('::')[1] if '::' in nm else nm).split('(')[0][:40]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    disp[k].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
for k, d in acc.items():
    n = max(1, len(disp[k]))
    print(f"{k:40s} disp {n:4d} " + " ".join(f"{c}={v / n:.0f}" for c, v in sorted(d.items())))
PY
rm -rf gpurun_out/pmc_ic
