#!/bin/bash
# Same-box A/B of libgrr builds on the full bench (no CPU baseline / secondary), R rounds.
#   bash scripts/ab_bench.sh ROUNDS LIB...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
for r in $(seq "$R"); do
  for L in "$@"; do
    out=$(GRR_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary 2>/dev/null | grep '^{') || exit 1
    echo "$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; k=d["kernel_ms_per_step"]; print(d["value"], r["mean_launch_ms"], r["copy_gbps"], k["system_half"], k["gtv_rhs_full"], k["edge_weights"])')"
  done
done
