"""Plain-PyTorch fp32 reference implementations of every fused op.

These serve two roles:
  * the oracle that the HIP-kernel numerics tests compare against, and
  * the CPU plumbing backend (BASELINE config "MNIST 3-layer CNN single-process
    Keras fit() on CPU").

Layouts follow Keras ``channels_last`` (``mnist.py:30``): activations NHWC,
conv kernels (KH, KW, Cin, Cout), dense kernels (in, out).  Semantics follow the
Keras 2.2 / TF 1.x ops the reference executes.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch
import torch.nn.functional as F

EPS = 1e-7  # keras.backend.epsilon()


# --------------------------------------------------------------------------- conv geometry
def conv_out_size(n: int, k: int, s: int, padding: str) -> int:
    if padding == "same":
        return -(-n // s)
    return (n - k) // s + 1


def same_pad(n: int, k: int, s: int) -> Tuple[int, int]:
    """TF 'same' padding split (extra row/col goes to the bottom/right)."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def conv_pads(h: int, w: int, kh: int, kw: int, s: int, padding: str):
    if padding == "same":
        pt, pb = same_pad(h, kh, s)
        pl, pr = same_pad(w, kw, s)
        return pt, pb, pl, pr
    return 0, 0, 0, 0


# --------------------------------------------------------------------------- conv
def conv2d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, stride: int = 1,
           padding: str = "valid") -> torch.Tensor:
    """x [B,H,W,C], w [KH,KW,C,Co] -> y [B,Ho,Wo,Co] (no activation)."""
    kh, kw = w.shape[0], w.shape[1]
    pt, pb, pl, pr = conv_pads(x.shape[1], x.shape[2], kh, kw, stride, padding)
    xn = x.permute(0, 3, 1, 2)
    if pt or pb or pl or pr:
        xn = F.pad(xn, (pl, pr, pt, pb))
    y = F.conv2d(xn, w.permute(3, 2, 0, 1), b, stride=stride)
    return y.permute(0, 2, 3, 1)


def conv2d_backward(x: torch.Tensor, w: torch.Tensor, dy: torch.Tensor, stride: int,
                    padding: str, need_dx: bool = True):
    """Returns (dx or None, dw [KH,KW,C,Co], db [Co])."""
    with torch.enable_grad():
        xr = x.detach().clone().requires_grad_(need_dx)
        wr = w.detach().clone().requires_grad_(True)
        y = conv2d(xr, wr, None, stride, padding)
        y.backward(dy)
    db = dy.sum(dim=(0, 1, 2))
    return (xr.grad if need_dx else None), wr.grad, db


# --------------------------------------------------------------------------- pool
def maxpool2x2(x: torch.Tensor):
    """2x2/2 valid max-pool on NHWC.  Returns (y, code) where code in {0..3} is the
    window position (dy*2+dx) of the FIRST maximum in row-major order."""
    B, H, W, C = x.shape
    Hp, Wp = H // 2, W // 2
    xw = x[:, :Hp * 2, :Wp * 2, :].reshape(B, Hp, 2, Wp, 2, C).permute(0, 1, 3, 2, 4, 5)
    xw = xw.reshape(B, Hp, Wp, 4, C)
    y, code = xw.max(dim=3)
    # torch.max returns *a* max index; enforce first-max tie-breaking explicitly
    eq = xw == y.unsqueeze(3)
    pos = torch.arange(4, device=x.device).view(1, 1, 1, 4, 1)
    code = torch.where(eq, pos, torch.full_like(pos, 4)).min(dim=3).values
    return y, code.to(torch.uint8)


def maxpool2x2_backward(dy: torch.Tensor, code: torch.Tensor, in_hw: Tuple[int, int]) -> torch.Tensor:
    B, Hp, Wp, C = dy.shape
    H, W = in_hw
    onehot = F.one_hot(code.long(), 4).permute(0, 1, 2, 4, 3).to(dy.dtype)  # B,Hp,Wp,4,C
    g = onehot * dy.unsqueeze(3)
    g = g.reshape(B, Hp, Wp, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(B, Hp * 2, Wp * 2, C)
    out = torch.zeros(B, H, W, C, dtype=dy.dtype, device=dy.device)
    out[:, :Hp * 2, :Wp * 2, :] = g
    return out


# --------------------------------------------------------------------------- losses
def softmax_cce(logits: torch.Tensor, y: torch.Tensor):
    """Keras categorical_crossentropy on a softmax output (TF backend semantics).

    Returns (loss_per_row, dlogits_per_row (not /B), correct_per_row)."""
    p = torch.softmax(logits, dim=-1)
    s = p.sum(dim=-1, keepdim=True)
    q = p / s
    inr = (q >= EPS) & (q <= 1.0 - EPS)
    qc = q.clamp(EPS, 1.0 - EPS)
    loss = -(y * torch.log(qc)).sum(dim=-1)
    g = torch.where(inr, -y / qc, torch.zeros_like(q))          # dL/dq
    gp = (g - (g * q).sum(-1, keepdim=True)) / s                 # dL/dp through normalisation
    dz = p * (gp - (p * gp).sum(-1, keepdim=True))               # softmax jacobian
    correct = (logits.argmax(-1) == y.argmax(-1)).to(torch.float32)
    return loss, dz, correct


def sigmoid_bce(z: torch.Tensor, y: torch.Tensor):
    """Keras binary_crossentropy on a sigmoid output: clip p to [eps, 1-eps], go back
    to logits, sigmoid-CE-with-logits.  z, y: [B] (or [B,1]).  Returns per-row
    (loss, dz, correct)."""
    p = torch.sigmoid(z)
    inr = (p >= EPS) & (p <= 1.0 - EPS)
    pc = p.clamp(EPS, 1.0 - EPS)
    lg = torch.log(pc / (1.0 - pc))
    loss = torch.clamp(lg, min=0) - lg * y + torch.log1p(torch.exp(-lg.abs()))
    dz = torch.where(inr, pc - y, torch.zeros_like(p))
    correct = (torch.round(p) == y).to(torch.float32)   # round-half-even like TF
    return loss, dz, correct


def mse(out: torch.Tensor, y: torch.Tensor):
    d = out - y
    loss = (d * d).mean(dim=-1)
    dz = 2.0 * d / out.shape[-1]
    return loss, dz, torch.zeros(out.shape[0], device=out.device)


# --------------------------------------------------------------------------- optimizers (Keras 2.2)
def adam_update(p, g, m, v, t: int, lr: float, beta_1=0.9, beta_2=0.999, eps=EPS):
    lr_t = lr * math.sqrt(1.0 - beta_2 ** t) / (1.0 - beta_1 ** t)
    m.mul_(beta_1).add_(g, alpha=1.0 - beta_1)
    v.mul_(beta_2).addcmul_(g, g, value=1.0 - beta_2)
    p.sub_(lr_t * m / (v.sqrt() + eps))


def adadelta_update(p, g, a, d, lr: float, rho=0.95, eps=EPS):
    a.mul_(rho).addcmul_(g, g, value=1.0 - rho)
    upd = g * torch.sqrt(d + eps) / torch.sqrt(a + eps)
    p.sub_(lr * upd)
    d.mul_(rho).addcmul_(upd, upd, value=1.0 - rho)


def nadam_schedule(t: int, m_schedule: float, beta_1=0.9, schedule_decay=0.004):
    mc_t = beta_1 * (1.0 - 0.5 * (0.96 ** (t * schedule_decay)))
    mc_t1 = beta_1 * (1.0 - 0.5 * (0.96 ** ((t + 1) * schedule_decay)))
    ms_new = m_schedule * mc_t
    ms_next = ms_new * mc_t1
    return mc_t, mc_t1, ms_new, ms_next


def nadam_update(p, g, m, v, t: int, lr: float, m_schedule: float, beta_1=0.9, beta_2=0.999,
                 eps=EPS, schedule_decay=0.004) -> float:
    """Returns the new m_schedule."""
    mc_t, mc_t1, ms_new, ms_next = nadam_schedule(t, m_schedule, beta_1, schedule_decay)
    g_prime = g / (1.0 - ms_new)
    m.mul_(beta_1).add_(g, alpha=1.0 - beta_1)
    v.mul_(beta_2).addcmul_(g, g, value=1.0 - beta_2)
    m_prime = m / (1.0 - ms_next)
    v_prime = v / (1.0 - beta_2 ** t)
    m_bar = (1.0 - mc_t) * g_prime + mc_t1 * m_prime
    p.sub_(lr * m_bar / (v_prime.sqrt() + eps))
    return ms_new


def sgd_update(p, g, mom, lr: float, momentum=0.0, nesterov=False):
    if momentum == 0.0:
        p.sub_(lr * g)
        return
    mom.mul_(momentum).sub_(lr * g)
    if nesterov:
        p.add_(momentum * mom - lr * g)
    else:
        p.add_(mom)


def rmsprop_update(p, g, a, lr: float, rho=0.9, eps=EPS):
    a.mul_(rho).addcmul_(g, g, value=1.0 - rho)
    p.sub_(lr * g / (a.sqrt() + eps))
