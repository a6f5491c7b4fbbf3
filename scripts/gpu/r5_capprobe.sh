#!/bin/bash
export PYTHONPATH=$PWD/gat-recommendation_amd:$PYTHONPATH
for m in inv; do
  echo "== $m"; timeout -k 10 90 python -u scripts/dbg/capture_probe.py $m 2>&1 | grep -vE "^\s*$" | tail -4; echo "rc ${PIPESTATUS[0]}"
done
