#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GTR_WGRAD=mfma XFLAG= bash scripts/gpu/tests.sh "large_batch or grads or fused_steps or c3_large" wgrad_mfma | tail -3 || exit 1
timeout -k 10 300 python3 scripts/wgrad_probe.py c3 8192 2> gpurun_out/wp.err || { tail -20 gpurun_out/wp.err; exit 1; }
timeout -k 10 300 python3 scripts/wgrad_probe.py c2 32 2> gpurun_out/wp2.err || { tail -20 gpurun_out/wp2.err; exit 1; }
