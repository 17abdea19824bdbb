#!/bin/bash
# Same-box A/B of libgrr builds: alternating micro-kernel runs, R rounds.
#   bash scripts/ab_micro.sh KERNEL ROUNDS LIB...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=$1; R=$2; shift 2
for r in $(seq "$R"); do
  for L in "$@"; do
    echo "== $K $L $(GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel $K --iters 50 2>&1 | tail -1)" || exit 1
  done
done
