#!/bin/bash
# A/B of the term reverse's x-gradient pass policy (ring kernel): inside at every width, only W <= 128, never
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${R05_OUT:-r05o}; mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in all w128 off; do
  case $v in all) env="" ; acc=1;; w128) env="GRR_TERM_ACC_MAXW=128"; acc=1;; off) env=""; acc=0;; esac
  for m in "msgf --batch 16 --steps 6 --warmup 2" "abstract --batch 8 --steps 5 --warmup 2" "abstract --size 512 --batch 32 --steps 2 --warmup 1"; do
    tag=$(echo $m | cut -d' ' -f1)$(echo $m | grep -o "size 512" | tr -d ' ')
    env $env timeout -k 10 400 python -u bench_train.py --model $m --term-acc $acc --no-cpu-baseline > $out/$v.$tag.$rep.json 2> $out/$v.$tag.$rep.err || { tail $out/$v.$tag.$rep.err; exit 1; }
    echo "$v $tag rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/$v.$tag.$rep.json)"
  done
done
done
