"""GPU worker for tests/test_comm.py::test_xgmi_two_processes_one_gpu: two processes on ONE
MI355X (RCCL refuses that, the xGMI path does not care whether the peer buffer is on this
GPU or another) run the fused all-reduce through real IPC-mapped peer memory: the
collective self-test, then the fused Adam update against a closed form.  Writes JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402


def allgather(obj):
    out = [None] * tdist.get_world_size()
    tdist.all_gather_object(out, obj)
    return out


def main(out_dir):
    tdist.init_process_group("gloo")
    r, P = tdist.get_rank(), tdist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from cori_intml_examples_amd.parallel import xgmi as X
    from cori_intml_examples_amd.ops.hip import kernels
    K = kernels()
    rep = {"rank": r}
    n = 100003                                  # not a multiple of anything
    x = X.create(r, P, n, dev, allgather)
    rep["created"] = x is not None
    if x is not None:
        rep["geometry"] = [x.chunk, x.sub, x.grid]
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
        a = K.OptimArgs()
        a.p, a.g, a.s0, a.s1, a.n, a.st = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, st.data_ptr()
        a.kind, a.grad_scale = 3, 1.0 / P
        x.launch(g.data_ptr(), torch.cuda.current_stream().cuda_stream, opt=a)
        torch.cuda.synchronize()
        gm = pat * (P * (P + 1) / 2.0) / P
        m_ref = 0.1 * gm
        v_ref = 0.001 * gm * gm
        p_ref = p0 - lr_t * m_ref / (torch.sqrt(v_ref) + 1e-7)
        rep["err"] = int(x.err.item())
        rep["grad_sum_ok"] = bool(torch.equal(g, pat * float(P * (P + 1) / 2)))
        rep["adam_maxdiff"] = float((p - p_ref).abs().max())
        rep["p_digest"] = [float(p.double().sum()), float(p.double().abs().sum())]
        x.close()
    with open(os.path.join(out_dir, "xgmi%d.json" % r), "w") as f:
        json.dump(rep, f)
    tdist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
