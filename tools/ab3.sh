#!/bin/bash
# Same-box A/B of kernel variants on the three BASELINE configs that run on one GPU (C2, C4, C5):
# "name:variant[:ENV=V,...]" specs as in tools/ab_env.sh, ROUNDS passes interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in C2 C4 C5; do
  BENCH_ARGS="--config $cfg" bash tools/ab_env.sh $(for s in "$@"; do n=${s%%:*}; echo "$cfg-$n:${s#*:}"; done) || exit $?
done
