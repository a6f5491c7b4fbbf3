set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "${TESTK}" > gpurun_out/t_sub.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/t_sub.log | tail -20
tail -2 gpurun_out/t_sub.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --c1-reps 0 --strong-batches 0 > gpurun_out/b_tr.json 2> gpurun_out/b_tr.err || { tail -20 gpurun_out/b_tr.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_tr.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['ms_per_step']); print('trainer', d.get('trainer_epoch'))"
GTR_BB_ONE=0 timeout -k 10 400 python3 bench.py --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --c1-reps 0 --strong-batches 0 > gpurun_out/b_tr0.json 2> gpurun_out/b_tr0.err || { tail -20 gpurun_out/b_tr0.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_tr0.json').read().strip().splitlines()[-1]); print('BB_ONE=0 headline', d['value'], d['ms_per_step']); print('trainer', d.get('trainer_epoch'))"
