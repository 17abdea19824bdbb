#!/bin/bash
# GPU-box session: parity tests -> smoke -> bench (-> optional rocprofv3 kernel trace).
# Each GPU step has its own time limit; any fault / abort / segfault / timeout
# (exit status other than 0 or a plain pytest failure 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <limit-seconds> <allow-exit-1> cmd...
  local name=$1 lim=$2 allow1=$3; shift 3
  echo "=== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 30 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && ! { [ "$rc" -eq 1 ] && [ "$allow1" = 1 ]; }; then
    echo "stopping: $name exited $rc" | tee -a "$OUT/session.log"
    exit "$rc"
  fi
}

MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 1 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = smoke ]; then
  step smoke 300 0 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 900 0 python bench.py --steps 10 --warmup 3 --breakdown
fi
if [ "$MODE" = prof ]; then
  step rocprof 900 0 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
fi
if [ "$MODE" = traffic ]; then
  step pmc_fetch 600 0 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
  step pmc_write 600 0 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary
  python scripts/collect_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --out "$OUT/traffic_system_step.json"
fi
echo "session done"
