cd $GRAFT_REPO_ROOT
for cfg in "INTML_TWO_STREAMS=0 INTML_GRAPHS=1" "INTML_TWO_STREAMS=1 INTML_GRAPHS=1" "INTML_TWO_STREAMS=0 INTML_GRAPHS=0" "INTML_TWO_STREAMS=1 INTML_GRAPHS=0" "INTML_EARLY_OPTIM=1 INTML_GRAPHS=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/exp.log 2>&1 || { tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -n 1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
