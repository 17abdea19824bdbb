#!/bin/bash
# Round-3 batch: each part is its own script with its own time limits; a part that fails ordinarily
# (tests failing, rc 1) lets the next run, one that ends in a fault / abort / time limit / kill
# (124, 134, 137, 139, negative) stops the batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for part in "$@"; do
  echo "=== $part"
  bash scripts/$part
  rc=$?
  echo "=== $part rc=$rc"
  case $rc in
    0|1) ;;
    *) echo "stopping the batch after rc=$rc"; exit $rc ;;
  esac
done
