"""GPU worker for tests/test_comm.py::test_xgmi_*_processes_one_gpu: P processes on ONE
MI355X (RCCL refuses that, the xGMI path does not care whether the peer buffer is on this
GPU or another) run the fused all-reduce through real IPC-mapped peer memory.

mode "full" (P = 2, 4 or 8): the collective self-test, the fused Adam update of a whole
gradient against the closed form, three back-to-back launches (sequence counters), and a
bucket that is a sub-range [lo, hi) of a larger gradient (elements outside untouched).
mode "delay" (P = 2): rank 1 starts its launch after rank 0's wait has timed out: rank 0
reports the timeout, rank 1 the abort, both exit cleanly, and every later launch on both
ranks exits at once without touching the gradient (sticky abort).  Writes JSON per rank."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402


def allgather(obj):
    out = [None] * tdist.get_world_size()
    tdist.all_gather_object(out, obj)
    return out


def adam_args(K, p, g, m, v, st, n, P):
    a = K.OptimArgs()
    a.p, a.g, a.s0, a.s1, a.n, a.st = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, st.data_ptr()
    a.kind, a.grad_scale = 3, 1.0 / P
    return a


def full(r, P, dev, K, X, rep):
    n = 100003                                  # not a multiple of anything
    x = X.create(r, P, n, dev, allgather, shared=True)
    rep["created"] = x is not None
    if x is None:
        return
    rep["geometry"] = [x.chunk, x.sub, x.grid]
    stream = torch.cuda.current_stream().cuda_stream
    # fused Adam (step 1) on grad_r = (r+1) * pat: reduced mean = pat * (P+1)/2
    idx = torch.arange(n, device=dev, dtype=torch.float32)
    pat = (torch.remainder(idx, 13.0) - 6.0) * 0.125
    g = pat * float(r + 1)
    p = torch.linspace(-1, 1, n, device=dev)
    p0 = p.clone()
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    st = torch.zeros(K.STEP_STATE_BYTES, dtype=torch.uint8, device=dev)
    lr_t = 0.01 * (1 - 0.999) ** 0.5 / (1 - 0.9)
    st.view(torch.float32)[6] = lr_t              # StepState.s[0] (bias-corrected LR)
    x.launch(g.data_ptr(), stream, opt=adam_args(K, p, g, m, v, st, n, P))
    torch.cuda.synchronize()
    gm = pat * (P * (P + 1) / 2.0) / P
    m_ref = 0.1 * gm
    v_ref = 0.001 * gm * gm
    p_ref = p0 - lr_t * m_ref / (torch.sqrt(v_ref) + 1e-7)
    rep["err"] = int(x.err[0].item())
    rep["grad_sum_ok"] = bool(torch.equal(g, pat * float(P * (P + 1) / 2)))
    rep["adam_maxdiff"] = float((p - p_ref).abs().max())
    rep["p_digest"] = [float(p.double().sum()), float(p.double().abs().sum())]
    # three more sum-only launches back to back (flag sequence numbers advance per launch)
    ok = True
    for it in range(3):
        g2 = pat * float(r + 2 + it)
        x.launch(g2.data_ptr(), stream)
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(g2, pat * float(sum(q + 2 + it for q in range(P)))))
    rep["repeat_ok"] = ok and int(x.err[0].item()) == 0
    x.close()

    # a bucket [lo, hi) of a larger flat gradient (hybrid plane: the conv bucket)
    N, lo = 50021, 12345
    hi = N
    xb = X.create(r, P, hi - lo, dev, allgather, shared=True)
    rep["range_created"] = xb is not None
    if xb is None:
        return
    idx = torch.arange(N, device=dev, dtype=torch.float32)
    pat = (torch.remainder(idx, 7.0) - 3.0) * 0.25
    g = pat * float(r + 1)
    p = torch.linspace(-2, 2, N, device=dev)
    p0 = p.clone()
    m = torch.zeros(N, device=dev)
    v = torch.zeros(N, device=dev)
    a = X.offset_optim(adam_args(K, p, g, m, v, st, N, P), lo)
    xb.launch(g.data_ptr() + 4 * lo, stream, opt=a)
    torch.cuda.synchronize()
    gm = pat[lo:] * (P * (P + 1) / 2.0) / P
    p_ref = p0[lo:] - lr_t * (0.1 * gm) / (torch.sqrt(0.001 * gm * gm) + 1e-7)
    rep["range_err"] = int(xb.err[0].item())
    rep["range_sum_ok"] = bool(torch.equal(g[lo:], pat[lo:] * float(P * (P + 1) / 2)))
    rep["range_outside_untouched"] = bool(torch.equal(g[:lo], pat[:lo] * float(r + 1))
                                          and torch.equal(p[:lo], p0[:lo]) and not bool(m[:lo].any()))
    rep["range_adam_maxdiff"] = float((p[lo:] - p_ref).abs().max())
    rep["range_p_digest"] = [float(p.double().sum()), float(p.double().abs().sum())]
    xb.close()


def delay(r, P, dev, K, X, rep):
    n = 4099
    x = X.create(r, P, n, dev, allgather, timeout_s=2.0, shared=True)
    rep["created"] = x is not None
    if x is None:
        return
    stream = torch.cuda.current_stream().cuda_stream
    g = torch.full((n,), float(r + 1), device=dev)
    tdist.barrier()
    if r == 1:
        time.sleep(5.0)                          # longer than rank 0's 2 s wait
    t0 = time.time()
    x.launch(g.data_ptr(), stream)
    torch.cuda.synchronize()
    rep["first_launch_s"] = time.time() - t0
    rep["err1"] = int(x.err[0].item())
    # every later launch exits at once on both ranks and touches nothing
    g2 = torch.full((n,), 7.0, device=dev)
    t0 = time.time()
    x.launch(g2.data_ptr(), stream)
    torch.cuda.synchronize()
    rep["second_launch_s"] = time.time() - t0
    rep["err2"] = int(x.err[0].item())
    rep["second_untouched"] = bool((g2 == 7.0).all())
    try:
        x.check()
        rep["check_raised"] = False
    except RuntimeError as e:
        rep["check_raised"] = True
        rep["check_msg"] = str(e)
    tdist.barrier()
    x.close()


def main(out_dir, mode):
    tdist.init_process_group("gloo")
    r, P = tdist.get_rank(), tdist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from cori_intml_examples_amd.parallel import xgmi as X
    from cori_intml_examples_amd.ops.hip import kernels
    K = kernels()
    rep = {"rank": r, "size": P}
    (full if mode == "full" else delay)(r, P, dev, K, X, rep)
    with open(os.path.join(out_dir, "xgmi%d.json" % r), "w") as f:
        json.dump(rep, f)
    tdist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "full")
