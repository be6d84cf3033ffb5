#!/bin/bash
# Same-box A/B of one env knob on the 1-GPU bench: interleaved runs, one JSON value per line.
#   KNOB=INTML_TUNE A=early_reduce=0 B=early_reduce=1 bash scripts/ab_bench.sh
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in $A $B; do
    r=$(env $KNOB=$v timeout -k 10 120 python bench.py --steps ${STEPS:-800} --warmup 80 ${BENCH_ARGS} 2>/dev/null | tail -n 1) || exit 1
    echo "$KNOB=$v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
