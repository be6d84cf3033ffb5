"""Keras-2.2 optimizers (hyper-parameters + state layout).

The update math runs in ONE fused multi-tensor HIP launch over the flat parameter
buffer (``csrc/kernels/optim.hip``) on GPU, or in ``ops/reference.py`` on CPU.
Name lookup by string mirrors ``getattr(optimizers, optimizer)(lr=lr)`` at
``rpv.py:62`` and ``model.compile(optimizer='Adadelta')`` at ``mnist.py:58``.
"""
from __future__ import annotations

from ..ops.reference import EPS


class KVariable:
    """Mutable scalar standing in for a Keras backend variable (``optimizer.lr``)."""

    def __init__(self, value: float, name: str = "var"):
        self._v = float(value)
        self.name = name

    def get(self) -> float:
        return self._v

    def set(self, v) -> None:
        self._v = float(v)

    def __float__(self):
        return self._v

    def __repr__(self):
        return "<KVariable %s=%g>" % (self.name, self._v)

    # arithmetic convenience (keeps user code like ``lr * 0.5`` working)
    def __mul__(self, o): return self._v * float(o)
    __rmul__ = __mul__
    def __truediv__(self, o): return self._v / float(o)
    def __add__(self, o): return self._v + float(o)
    __radd__ = __add__
    def __sub__(self, o): return self._v - float(o)
    def __lt__(self, o): return self._v < float(o)
    def __gt__(self, o): return self._v > float(o)
    def __le__(self, o): return self._v <= float(o)
    def __ge__(self, o): return self._v >= float(o)
    def __eq__(self, o):
        try:
            return self._v == float(o)
        except (TypeError, ValueError):
            return False
    __hash__ = object.__hash__


def get_value(x) -> float:
    return x.get() if isinstance(x, KVariable) else float(x)


def set_value(x, v) -> None:
    if not isinstance(x, KVariable):
        raise TypeError("set_value needs a KVariable")
    x.set(v)


class Optimizer:
    kind = "base"
    n_slots = 0          # number of flat fp32 state buffers
    default_lr = 0.01

    def __init__(self, lr=None, decay=0.0, learning_rate=None, **kw):
        if lr is None:
            lr = learning_rate if learning_rate is not None else self.default_lr
        self.lr = KVariable(lr, "lr")
        self.decay = float(decay)
        self.initial_decay = self.decay
        self.iterations = 0          # host mirror of the device step counter
        self.distributed = False
        self.compression = None
        self._extra = {}

    def current_lr(self) -> float:
        lr = self.lr.get()
        if self.initial_decay > 0:
            lr = lr / (1.0 + self.initial_decay * self.iterations)
        return lr

    def hparams(self) -> dict:
        return {}

    def get_config(self) -> dict:
        cfg = {"lr": self.lr.get(), "decay": self.decay}
        cfg.update(self.hparams())
        return cfg

    @classmethod
    def from_config(cls, cfg):
        return cls(**cfg)

    @property
    def class_name(self) -> str:
        return type(self).__name__


class SGD(Optimizer):
    kind = "sgd"
    default_lr = 0.01

    def __init__(self, lr=None, momentum=0.0, decay=0.0, nesterov=False, **kw):
        super().__init__(lr=lr, decay=decay, **kw)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        self.n_slots = 1 if self.momentum else 0

    def hparams(self):
        return {"momentum": self.momentum, "nesterov": self.nesterov}


class RMSprop(Optimizer):
    kind = "rmsprop"
    n_slots = 1
    default_lr = 0.001

    def __init__(self, lr=None, rho=0.9, epsilon=None, decay=0.0, **kw):
        super().__init__(lr=lr, decay=decay, **kw)
        self.rho = float(rho)
        self.epsilon = EPS if epsilon is None else float(epsilon)

    def hparams(self):
        return {"rho": self.rho, "epsilon": self.epsilon}


class Adadelta(Optimizer):
    kind = "adadelta"
    n_slots = 2
    default_lr = 1.0

    def __init__(self, lr=None, rho=0.95, epsilon=None, decay=0.0, **kw):
        super().__init__(lr=lr, decay=decay, **kw)
        self.rho = float(rho)
        self.epsilon = EPS if epsilon is None else float(epsilon)

    def hparams(self):
        return {"rho": self.rho, "epsilon": self.epsilon}


class Adam(Optimizer):
    kind = "adam"
    n_slots = 2
    default_lr = 0.001

    def __init__(self, lr=None, beta_1=0.9, beta_2=0.999, epsilon=None, decay=0.0, amsgrad=False, **kw):
        super().__init__(lr=lr, decay=decay, **kw)
        if amsgrad:
            raise NotImplementedError("amsgrad")
        self.beta_1, self.beta_2 = float(beta_1), float(beta_2)
        self.epsilon = EPS if epsilon is None else float(epsilon)
        self.amsgrad = False

    def hparams(self):
        return {"beta_1": self.beta_1, "beta_2": self.beta_2, "epsilon": self.epsilon,
                "amsgrad": False}


class Nadam(Optimizer):
    kind = "nadam"
    n_slots = 2
    default_lr = 0.002

    def __init__(self, lr=None, beta_1=0.9, beta_2=0.999, epsilon=None, schedule_decay=0.004, **kw):
        kw.pop("decay", None)
        super().__init__(lr=lr, **kw)
        self.beta_1, self.beta_2 = float(beta_1), float(beta_2)
        self.epsilon = EPS if epsilon is None else float(epsilon)
        self.schedule_decay = float(schedule_decay)
        self.m_schedule = 1.0        # host mirror (device keeps its own copy)

    def hparams(self):
        return {"beta_1": self.beta_1, "beta_2": self.beta_2, "epsilon": self.epsilon,
                "schedule_decay": self.schedule_decay}

    def get_config(self):
        cfg = {"lr": self.lr.get()}
        cfg.update(self.hparams())
        return cfg


# lowercase aliases as accepted by keras.optimizers.get
_BY_NAME = {"sgd": SGD, "rmsprop": RMSprop, "adadelta": Adadelta, "adam": Adam, "nadam": Nadam}


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    if hasattr(identifier, "_base_optimizer"):      # DistributedOptimizer wrapper
        return identifier
    if isinstance(identifier, type) and issubclass(identifier, Optimizer):
        return identifier()
    if isinstance(identifier, str):
        cls = _BY_NAME.get(identifier.lower())
        if cls is None:
            raise ValueError("unknown optimizer %r" % identifier)
        return cls()
    if isinstance(identifier, dict):
        return deserialize(identifier)
    raise ValueError("cannot interpret optimizer %r" % (identifier,))


def deserialize(cfg: dict) -> Optimizer:
    cls = _BY_NAME[cfg["class_name"].lower()]
    return cls.from_config(cfg.get("config", {}))


def serialize(opt: Optimizer) -> dict:
    base = getattr(opt, "_base_optimizer", opt)
    return {"class_name": type(base).__name__, "config": base.get_config()}
