# FETCH/WRITE of the step kernel alone, per graph-kernel variant (scripts/micro.py), one pass per counter
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/mpmc
for v in auto independent; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/mpmc/${v}_$ctr -o run -- python scripts/micro.py --kernel step --iters 3 --variant $v > gpurun_out/mpmc/${v}_$ctr.log 2>&1 || exit 1
  done
done
