# pass r5i: the exchange's fixed cost -- N = 1 DP (xGMI plane) with the single-GPU update in place
# (default) and with the exchange structure kept (xchg_p1=1, the fixed cost the N > 1 step pays),
# the looping-workgroup variant of the exchange launches, and the P = 2/4/8 one-GPU DP test
export TAG=r5i
export TESTS="tests/test_comm.py -k 'dp_step_xgmi'"
X="INTML_DP_FORCE=1 INTML_XGMI=xgmi"
export AB="|$X;|$X;xchg_p1=1|$X;xchg_p1=1,xchg_nx=128|$X;xchg_p1=1,xchg_nx=256,xchg_rfirst=0"
export AB_ROUNDS=2
bash scripts/gpu_pass.sh
