"""CPU reference backend: executes a Plan with the fp32 PyTorch ops of
``ops/reference.py``.  This is the "MNIST 3-layer CNN single-process Keras fit() on
CPU (plumbing, no GPU)" configuration of BASELINE.json and the oracle for the
whole-model HIP tests.  Forward/backward are written out explicitly (no autograd
graph) in exactly the stage order the HIP executor uses.

``INTML_TUNE=ref_bf16=1`` makes it a bf16-FAITHFUL oracle: values are rounded to bf16 at
exactly the points where the HIP step stores them in bf16 (weight packs of the convs and
hidden denses, every stage output after its dropout, the hidden denses' dH and every pooled
dP after their masks), everything else in fp32 -- so the whole-step gradient test can use
the per-kernel tests' tight tolerances instead of the loose fp32-vs-bf16 bound.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..ops import reference as R
from ..ops.rng import dropout_keep
from ..utils.env import tune
from .executor_base import DeviceData, Executor, prepare_targets
from .plan import Plan


class RefExecutor(Executor):
    def __init__(self, plan: Plan, store, optimizer, seed: int):
        super().__init__(plan, store, optimizer, seed)
        self.device = torch.device("cpu")
        n_slots = getattr(optimizer, "n_slots", 0)
        self.slots: List[torch.Tensor] = [torch.zeros(store.capacity) for _ in range(n_slots)]
        self.m_schedule = 1.0
        self._acc = torch.zeros(3, dtype=torch.float64)
        self._last = (0.0, 0.0)
        self.emulate_bf16 = bool(tune("ref_bf16", False))

    # ------------------------------------------------------------------------------ data
    def upload(self, x, y):
        xt = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32))
        if xt.shape[1:] != tuple(self.plan.input_shape):
            raise ValueError("input shape %s != model input %s" % (tuple(xt.shape[1:]),
                                                                   self.plan.input_shape))
        yt = torch.as_tensor(prepare_targets(y, self.plan)) if y is not None else None
        return DeviceData(xt, yt, xt.shape[0])

    # ------------------------------------------------------------------------------ core
    def _mask(self, numel, rate, stream, step):
        keep = dropout_keep(numel, rate, self.seed, stream, step)
        return keep.to(torch.float32) / (1.0 - rate)

    def _q(self, t):
        """bf16 rounding at a HIP storage point (identity unless emulating bf16)."""
        return t.to(torch.bfloat16).to(torch.float32) if self.emulate_bf16 else t

    def _forward(self, x, training: bool, step: int):
        st = self.store
        saved = []
        a = x
        for cs in self.plan.convs:
            w = self._q(st.view(cs.conv, "kernel"))
            b = st.view(cs.conv, "bias") if cs.conv.use_bias else None
            z = R.conv2d(a, w, b, cs.stride, cs.conv.padding)
            r = torch.relu(z) if cs.relu else z
            code = None
            p = r
            if cs.pool is not None:
                p, code = R.maxpool2x2(r)
            mask = None
            if training and cs.rate > 0:
                mask = self._mask(p.numel(), cs.rate, cs.stream, step).view(p.shape)
                p = p * mask
            saved.append((a, r, code, mask))
            a = self._q(p)
        a = a.reshape(a.shape[0], -1)
        for ds in self.plan.denses:
            w = self._q(st.view(ds.dense, "kernel"))
            z = a @ w
            if ds.dense.use_bias:
                z = z + st.view(ds.dense, "bias")
            r = torch.relu(z) if ds.relu else z
            mask = None
            if training and ds.rate > 0:
                mask = self._mask(r.numel(), ds.rate, ds.stream, step).view(r.shape)
                r = r * mask
            saved.append((a, z, None, mask))
            a = self._q(r)
        hd = self.plan.head
        z = a @ st.view(hd.dense, "kernel")
        if hd.dense.use_bias:
            z = z + st.view(hd.dense, "bias")
        return z, a, saved

    def _head_loss(self, z, y):
        hd = self.plan.head
        if hd.activation == "softmax":
            return R.softmax_cce(z, y)
        if hd.activation == "sigmoid":
            loss, dz, corr = R.sigmoid_bce(z.reshape(-1), y.reshape(-1))
            return loss, dz.reshape(-1, 1), corr
        return R.mse(z, y)

    def _backward(self, dz, a_head, saved):
        st = self.store
        hd = self.plan.head
        st.view(hd.dense, "kernel", grad=True).copy_(a_head.t() @ dz)
        if hd.dense.use_bias:
            st.view(hd.dense, "bias", grad=True).copy_(dz.sum(0))
        da = dz @ st.view(hd.dense, "kernel").t()
        nconv = len(self.plan.convs)
        for i in reversed(range(len(self.plan.denses))):
            ds = self.plan.denses[i]
            a_in, z, _, mask = saved[nconv + i]
            if mask is not None:
                da = da * mask
            if ds.relu:
                da = da * (z > 0).to(da.dtype)
            da = self._q(da)                                   # the stored bf16 dH
            st.view(ds.dense, "kernel", grad=True).copy_(a_in.t() @ da)
            if ds.dense.use_bias:
                st.view(ds.dense, "bias", grad=True).copy_(da.sum(0))
            da = da @ self._q(st.view(ds.dense, "kernel")).t()
        if nconv:
            cs_last = self.plan.convs[-1]
            da = da.reshape((da.shape[0],) + tuple(cs_last.out_shape))
        for i in reversed(range(nconv)):
            cs = self.plan.convs[i]
            a_in, r, code, mask = saved[i]
            if mask is not None:
                da = da * mask
            if self.emulate_bf16:
                # the HIP step stores this gradient (masked by the dropout and the ReLU of
                # the stage output, at the stage's output resolution) as bf16 before routing it
                if cs.relu:
                    pooled = R.maxpool2x2(r)[0] if cs.pool is not None else r
                    da = da * (pooled > 0).to(da.dtype)
                da = self._q(da)
            if cs.pool is not None:
                da = R.maxpool2x2_backward(da, code, r.shape[1:3])
            if cs.relu:
                da = da * (r > 0).to(da.dtype)
            dx, dw, db = R.conv2d_backward(a_in, self._q(st.view(cs.conv, "kernel")), da, cs.stride,
                                           cs.conv.padding, need_dx=i > 0)
            st.view(cs.conv, "kernel", grad=True).copy_(dw)
            if cs.conv.use_bias:
                st.view(cs.conv, "bias", grad=True).copy_(db)
            da = dx

    def _apply_update(self):
        opt = self.optimizer
        base = getattr(opt, "_base_optimizer", opt)
        base.iterations += 1
        t = base.iterations
        lr = self.base_lr_for_step(t, float(base.lr))
        if base.initial_decay != 0:
            lr = lr / (1.0 + base.initial_decay * (t - 1))
        n = self.store.numel
        p, g = self.store.master[:n], self.store.grad[:n]
        k = base.kind
        if k == "adam":
            R.adam_update(p, g, self.slots[0][:n], self.slots[1][:n], t, lr, base.beta_1, base.beta_2,
                          base.epsilon)
        elif k == "adadelta":
            R.adadelta_update(p, g, self.slots[0][:n], self.slots[1][:n], lr, base.rho, base.epsilon)
        elif k == "nadam":
            self.m_schedule = R.nadam_update(p, g, self.slots[0][:n], self.slots[1][:n], t, lr,
                                             self.m_schedule, base.beta_1, base.beta_2, base.epsilon,
                                             base.schedule_decay)
            base.m_schedule = self.m_schedule
        elif k == "sgd":
            R.sgd_update(p, g, self.slots[0][:n] if self.slots else None, lr, base.momentum,
                         base.nesterov)
        elif k == "rmsprop":
            R.rmsprop_update(p, g, self.slots[0][:n], lr, base.rho, base.epsilon)
        else:
            raise NotImplementedError(k)

    # ------------------------------------------------------------------------------ steps
    def train_step(self, data: DeviceData, perm: torch.Tensor, pos: int, bs: int) -> None:
        idx = perm[pos:pos + bs]
        x, y = data.x[idx], data.y[idx]
        base = getattr(self.optimizer, "_base_optimizer", self.optimizer)
        step = base.iterations + 1
        with torch.no_grad():
            z, a_head, saved = self._forward(x, True, step)
            loss, dz, corr = self._head_loss(z, y)
            self._backward(dz / bs, a_head, saved)
            if self.reducer is not None:
                if not getattr(self, "_buckets_configured", False):
                    # same bucketing as the GPU executor: per-layer flat ranges in backward
                    # order (last layer first), merged up to the reducer's bucket size
                    ranges = sorted(self.store.layer_ranges().values(), key=lambda r: -r[0])
                    self.reducer.configure(ranges)
                    self._buckets_configured = True
                self.reducer.reduce_all(self.store.grad)
            self._apply_update()
        self._accumulate(loss, corr, bs)

    def _accumulate(self, loss, corr, bs):
        ls, cs = float(loss.sum()), float(corr.sum())
        self._acc += torch.tensor([ls, cs, bs], dtype=torch.float64)
        self._last = (ls / bs, cs / bs)

    def eval_step(self, data: DeviceData, pos: int, bs: int) -> None:
        x, y = data.x[pos:pos + bs], data.y[pos:pos + bs]
        with torch.no_grad():
            z, _, _ = self._forward(x, False, 0)
            loss, _, corr = self._head_loss(z, y)
        self._accumulate(loss, corr, bs)

    def predict_step(self, data: DeviceData, pos: int, bs: int) -> torch.Tensor:
        with torch.no_grad():
            z, _, _ = self._forward(data.x[pos:pos + bs], False, 0)
        act = self.plan.head.activation
        if act == "softmax":
            return torch.softmax(z, -1)
        if act == "sigmoid":
            return torch.sigmoid(z)
        return z

    def reset_metrics(self):
        self._acc.zero_()

    def read_metrics(self):
        ls, cs, n = self._acc.tolist()
        n = max(n, 1.0)
        return ls / n, cs / n, int(n)

    def last_batch_metrics(self):
        return self._last

    def m_schedule_value(self) -> float:
        return float(self.m_schedule)

    def set_m_schedule(self, v: float) -> None:
        self.m_schedule = float(v)

    def optimizer_state(self):
        return [s[:self.store.numel] for s in self.slots]

    def set_optimizer_state(self, iterations, slots):
        base = getattr(self.optimizer, "_base_optimizer", self.optimizer)
        base.iterations = int(iterations)
        for dst, src in zip(self.slots, slots):
            dst[:self.store.numel].copy_(torch.as_tensor(src).reshape(-1))
