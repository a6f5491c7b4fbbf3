set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "trainer_graph or multi_step or dropin or sharded or test_abi or step_graph" > gpurun_out/t1.log 2>&1 || { tail -60 gpurun_out/t1.log; exit 1; }
tail -5 gpurun_out/t1.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-seconds 0 --gather-batch 0 --recall-steps 0 --e2e-steps 200 --c1-reps 0 --strong-batches 0 > gpurun_out/b1.json 2> gpurun_out/b1.err || { tail -30 gpurun_out/b1.err; exit 1; }
cat gpurun_out/b1.json
bash scripts/gpu/phases.sh "c3:8192 c4:1024" > gpurun_out/ph1.log 2>&1 || { tail -20 gpurun_out/ph1.log; exit 1; }
cat gpurun_out/ph1.log
