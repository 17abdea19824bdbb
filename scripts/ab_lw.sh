#!/bin/bash
# Same-box A/B of step-kernel builds (micro step kernel) + GPU parity of the candidates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in "$@"; do
  echo "== parity $L"
  GRR_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/parity_$(basename $L .so).log 2>&1 || { tail -30 gpurun_out/parity_$(basename $L .so).log; exit 1; }
  tail -1 gpurun_out/parity_$(basename $L .so).log
done
for r in 1 2; do
  for L in "$@"; do
    for K in step half; do
      echo "== micro $K $L"; GRR_LIB=$L timeout -k 10 120 python scripts/micro.py --kernel $K --iters 30 2>&1 | tail -1 || exit 1
    done
  done
done
