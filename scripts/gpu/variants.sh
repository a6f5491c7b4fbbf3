#!/bin/bash
# Build-time variants (EXTRA defines) for per-kernel A/B with scripts/dbg/kbench.py.
# Runs HERE (CPU): make BUILD=../build/<name> EXTRA="<defines>" for each name=defines pair.
cd "$(dirname "$0")/../../gat-recommendation_amd/csrc" || exit 1
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  make -s BUILD=../build/$name EXTRA="$defs" -j8 all || exit 1
done
