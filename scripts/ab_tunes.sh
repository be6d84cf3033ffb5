#!/bin/bash
# Same-box A/B of INTML_TUNE variants on the 1-GPU bench (no HPO): interleaved rounds,
#   bash scripts/ab_tunes.sh "" "wt=0" "head_generic=1"      (ROUNDS, STEPS, BENCH_ARGS)
cd $GRAFT_REPO_ROOT
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    r=$(INTML_TUNE="$v" timeout -k 10 120 python bench.py --steps ${STEPS:-800} --warmup 80 --no-hpo ${BENCH_ARGS} 2>/dev/null | tail -n 1) || exit 1
    echo "r$i [${v:-default}] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
