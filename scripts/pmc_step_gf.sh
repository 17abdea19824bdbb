cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/mpmc
for gf in "32 3" "96 1"; do set -- $gf
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/mpmc/${1}_${2}_$ctr -o run -- python scripts/micro.py --kernel step --iters 3 --graphs $1 --fts $2 > gpurun_out/mpmc/${1}_${2}_$ctr.log 2>&1 || exit 1
  done
done
timeout 120 python scripts/micro.py --kernel step --iters 10 --graphs 32 --fts 3 > gpurun_out/mpmc/t32.log 2>&1
timeout 120 python scripts/micro.py --kernel step --iters 10 --graphs 96 --fts 1 > gpurun_out/mpmc/t96.log 2>&1
tail -2 gpurun_out/mpmc/t32.log gpurun_out/mpmc/t96.log
