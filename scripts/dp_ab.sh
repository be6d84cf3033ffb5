cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for e in "X=1" "INTML_DP_FORCE=1" "INTML_DP_FORCE=1 INTML_XGMI=1"; do
    r=$(env $e timeout -k 10 120 python bench.py --steps 800 --warmup 80 2>/dev/null | tail -n 1) || exit 1
    echo "$e $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("selfcheck",{}).get("data_plane"), d.get("selfcheck",{}).get("exposed_comm_us_per_step"))')"
  done
done
