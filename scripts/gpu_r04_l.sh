#!/bin/bash
# Round 4: training lines + term-reverse PMC traffic (gpu_r04_i.sh), then the term reverse per shape (gpu_r04_k.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r04_i.sh || exit $?
bash scripts/gpu_r04_k.sh
