"""Python face of the native ``_h5lite`` HDF5 module (``csrc/io/h5lite.cpp``).

Replaces the h5py calls of the reference (``rpv.py:20-24``; Keras' saver behind
``rpv.py:100-101``).  ``H5File`` is a context manager with a small h5py-like surface:

    with H5File("train.h5") as f:
        hist = f.read_dataset("all_events/hist", 64000)     # first 64000 rows only
        f.attrs("/")["model_config"]                         # str
"""
from __future__ import annotations

import importlib
from typing import Any, Iterable, List, Optional

import numpy as np

_MOD = None


def _native():
    global _MOD
    if _MOD is None:
        try:
            _MOD = importlib.import_module("cori_intml_examples_amd._h5lite")
        except ImportError:
            from .. import _build
            if _build.build_h5() is None:
                raise ImportError("_h5lite unavailable: libhdf5 headers not found (set INTML_HDF5_ROOT)")
            _MOD = importlib.import_module("cori_intml_examples_amd._h5lite")
    return _MOD


def available() -> bool:
    try:
        _native()
        return True
    except Exception:
        return False


def _dec(v):
    if isinstance(v, bytes):
        return v.decode("utf8")
    if isinstance(v, list):
        return [_dec(x) for x in v]
    return v


class _Attrs:
    """dict-like attribute access on one object; strings come back as ``str``."""

    def __init__(self, f: "H5File", path: str):
        self._f, self._p = f, path

    def __getitem__(self, name: str) -> Any:
        v = self._f._h.get_attr(self._p, name)
        if isinstance(v, np.ndarray) and v.ndim == 0:
            return v[()]
        return _dec(v)

    def get(self, name: str, default=None):
        return self[name] if name in self else default

    def __contains__(self, name: str) -> bool:
        return name in self._f._h.attr_names(self._p)

    def keys(self) -> List[str]:
        return list(self._f._h.attr_names(self._p))

    def __setitem__(self, name: str, value: Any) -> None:
        h = self._f._h
        if isinstance(value, (str, bytes)):
            h.set_attr_strings(self._p, name, [value.encode("utf8") if isinstance(value, str) else value], True)
        elif isinstance(value, (list, tuple)) and (len(value) == 0 or isinstance(value[0], (str, bytes))):
            h.set_attr_strings(self._p, name,
                               [v.encode("utf8") if isinstance(v, str) else v for v in value], False)
        else:
            h.set_attr_array(self._p, name, np.asarray(value))


class H5File:
    def __init__(self, path: str, mode: str = "r"):
        self._h = _native().File(str(path), mode)
        self.path = str(path)

    # context manager -------------------------------------------------------------
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        self._h.close()

    def flush(self):
        self._h.flush()

    # structure ---------------------------------------------------------------------
    def __contains__(self, path: str) -> bool:
        return self._h.exists(path)

    def kind(self, path: str) -> str:
        return self._h.kind(path)

    def keys(self, path: str = "/") -> List[str]:
        return list(self._h.keys(path))

    def create_group(self, path: str) -> None:
        self._h.create_group(path)

    def attrs(self, path: str = "/") -> _Attrs:
        return _Attrs(self, path)

    # data ----------------------------------------------------------------------------
    def shape(self, path: str):
        return tuple(int(d) for d in self._h.shape(path))

    def write_dataset(self, path: str, array, gzip: int = 0) -> None:
        self._h.write_dataset(path, np.asarray(array), gzip)

    def read_dataset(self, path: str, n: Optional[int] = None, start: int = 0):
        """Rows ``[start, start+n)`` along axis 0 (all when ``n`` is None)."""
        v = self._h.read_dataset(path, int(start), -1 if n is None else int(n))
        return _dec(v)

    def walk(self, path: str = "/") -> Iterable[str]:
        for k in self.keys(path):
            p = (path.rstrip("/") + "/" + k) if path != "/" else "/" + k
            yield p
            if self.kind(p) == "group":
                yield from self.walk(p)
