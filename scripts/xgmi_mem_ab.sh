#!/bin/bash
# xGMI fused all-reduce at N=1 (loopback): uncached vs fine-grained inbox/outbox memory, plus
# the 2-process protocol test with each memory type.
cd $GRAFT_REPO_ROOT
for mem in uncached finegrained; do
  INTML_XGMI_MEM=$mem timeout -k 10 200 python -u -m pytest tests/test_comm.py -q -m gpu -k "xgmi" --timeout 150 --timeout-method thread 2>&1 | tail -n 1 || exit 1
  for i in 1 2; do
    r=$(INTML_XGMI_MEM=$mem INTML_DP_FORCE=1 INTML_XGMI=1 timeout -k 10 120 python bench.py --steps 800 --warmup 80 2>/dev/null | tail -n 1) || exit 1
    echo "$mem $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("selfcheck",{}).get("exposed_comm_us_per_step"))')"
  done
done
