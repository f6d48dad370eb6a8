"""ctypes binding to the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of ``bench.py`` -- never by the product package
``nonlocalheatequation_amd``.  The oracle restates
/root/reference/src/2d_nonlocal_serial.cpp (see nlh_oracle.c for the per-line
citations) and is pinned against SURVEY.md Appendix A (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")


class Params(ctypes.Structure):
    _fields_ = [
        ("nx", ctypes.c_long),
        ("ny", ctypes.c_long),
        ("eps", ctypes.c_long),
        ("k", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("dh", ctypes.c_double),
        ("test", ctypes.c_int),
        ("influence", ctypes.c_int),
    ]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER(Params)
        dp = ctypes.POINTER(ctypes.c_double)
        L.nlh_oracle_c2d.argtypes = [P]
        L.nlh_oracle_c2d.restype = ctypes.c_double
        L.nlh_oracle_disk_count.argtypes = [ctypes.c_long]
        L.nlh_oracle_disk_count.restype = ctypes.c_long
        L.nlh_oracle_test_init.argtypes = [P, dp]
        L.nlh_oracle_exact.argtypes = [P, ctypes.c_long, dp]
        L.nlh_oracle_step.argtypes = [P, ctypes.c_long, dp, dp, ctypes.c_int]
        L.nlh_oracle_run.argtypes = [P, ctypes.c_long, dp, ctypes.c_int]
        L.nlh_oracle_errors.argtypes = [P, ctypes.c_long, dp, dp, dp]
        L.nlh_oracle_run_compensated.argtypes = [P, ctypes.c_long, dp, ctypes.c_int]
        L.nlh_oracle_run_tiled.argtypes = [P, ctypes.c_long, ctypes.c_long, ctypes.c_long, dp, ctypes.c_int]
        L.nlh_oracle_run_tiled.restype = ctypes.c_double
        L.nlh_oracle_time_tiles.argtypes = [P, ctypes.c_long, ctypes.c_long, ctypes.c_long, ctypes.c_long,
                                            ctypes.c_long, dp, ctypes.c_int]
        L.nlh_oracle_time_tiles.restype = ctypes.c_double
        L.nlh_oracle_c1d.argtypes = [ctypes.c_long, ctypes.c_double, ctypes.c_double]
        L.nlh_oracle_c1d.restype = ctypes.c_double
        L.nlh_oracle_run_1d.argtypes = [ctypes.c_long, ctypes.c_long, ctypes.c_long, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, ctypes.c_int, dp]
        L.nlh_oracle_errors_1d.argtypes = [ctypes.c_long, ctypes.c_long, ctypes.c_double, ctypes.c_double,
                                           dp, dp, dp]
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def params(nx, ny, eps, k, dt, dh, test, influence=0) -> Params:
    """influence: 0 = J = 1 (the reference), 1 = J(r) = 1 - r (parity unpinned)."""
    return Params(int(nx), int(ny), int(eps), float(k), float(dt), float(dh), int(bool(test)), int(influence))


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def c2d(p: Params) -> float:
    return lib().nlh_oracle_c2d(ctypes.byref(p))


def disk_count(eps: int) -> int:
    return lib().nlh_oracle_disk_count(int(eps))


def test_init(p: Params) -> np.ndarray:
    """IC field, shape (ny, nx) row-major == reference index x + y*nx."""
    u = np.empty((p.ny, p.nx), dtype=np.float64)
    lib().nlh_oracle_test_init(ctypes.byref(p), _dp(u))
    return u


def exact(p: Params, t: int) -> np.ndarray:
    w = np.empty((p.ny, p.nx), dtype=np.float64)
    lib().nlh_oracle_exact(ctypes.byref(p), int(t), _dp(w))
    return w


def step(p: Params, t: int, u: np.ndarray, nthreads: int | None = None) -> np.ndarray:
    u = np.ascontiguousarray(u, dtype=np.float64)
    un = np.empty_like(u)
    lib().nlh_oracle_step(ctypes.byref(p), int(t), _dp(u), _dp(un), nthreads or default_threads())
    return un


def run(p: Params, nt: int, u: np.ndarray | None = None, nthreads: int | None = None) -> np.ndarray:
    u = test_init(p) if u is None else np.array(u, dtype=np.float64, order="C", copy=True)
    lib().nlh_oracle_run(ctypes.byref(p), int(nt), _dp(u), nthreads or default_threads())
    return u


def run_compensated(p: Params, nt: int, u: np.ndarray | None = None, nthreads: int | None = None) -> np.ndarray:
    """The same steps in long double, rounded to double once per node and step
    (J = 1): the reference's arithmetic without the rounding of its N(eps)
    sequential terms (nlh_oracle.c nlh_oracle_run_compensated)."""
    if p.influence != 0:
        raise ValueError("run_compensated: J = 1 only")
    u = test_init(p) if u is None else np.array(u, dtype=np.float64, order="C", copy=True)
    lib().nlh_oracle_run_compensated(ctypes.byref(p), int(nt), _dp(u), nthreads or default_threads())
    return u


def errors(p: Params, time: int, u: np.ndarray) -> tuple[float, float]:
    u = np.ascontiguousarray(u, dtype=np.float64)
    l2 = ctypes.c_double()
    li = ctypes.c_double()
    lib().nlh_oracle_errors(ctypes.byref(p), int(time), _dp(u), ctypes.byref(l2), ctypes.byref(li))
    return l2.value, li.value


def run_tiled(p: Params, nt: int, tiles_x: int, tiles_y: int, u: np.ndarray, nthreads: int) -> float:
    """In-place tiled run (2d_nonlocal_async execution model); returns seconds."""
    assert u.dtype == np.float64 and u.flags.c_contiguous
    return lib().nlh_oracle_run_tiled(ctypes.byref(p), int(nt), int(tiles_x), int(tiles_y), _dp(u), int(nthreads))


def time_tiles(p: Params, t: int, tiles_x: int, tiles_y: int, first: int, ntiles: int, u: np.ndarray,
               nthreads: int) -> float:
    """Seconds of run_tiled's step t over only tiles first .. first+ntiles-1
    (row-major; a bounded timing sample of a lattice too large to step whole);
    u is not changed."""
    assert u.dtype == np.float64 and u.flags.c_contiguous
    return lib().nlh_oracle_time_tiles(ctypes.byref(p), int(t), int(tiles_x), int(tiles_y), int(first), int(ntiles),
                                       _dp(u), int(nthreads))


# ---- 1D solver (src/1d_nonlocal_serial.cpp) ---------------------------------
def test_init_1d(nx: int, dx: float) -> np.ndarray:
    """test_init(): sin(2*pi*(sx*dx)) (1d :124-129)."""
    return np.array([math.sin(2 * math.pi * (sx * dx)) for sx in range(nx)], dtype=np.float64)  # libm sin


def run_1d(nx, nt, eps, k, dt, dx, test, u=None) -> np.ndarray:
    u = test_init_1d(nx, dx) if u is None else np.array(u, dtype=np.float64, copy=True)
    lib().nlh_oracle_run_1d(int(nx), int(nt), int(eps), float(k), float(dt), float(dx), int(bool(test)), _dp(u))
    return u


def errors_1d(nx, time, dt, dx, u) -> tuple[float, float]:
    u = np.ascontiguousarray(u, dtype=np.float64)
    l2 = ctypes.c_double()
    li = ctypes.c_double()
    lib().nlh_oracle_errors_1d(int(nx), int(time), float(dt), float(dx), _dp(u), ctypes.byref(l2), ctypes.byref(li))
    return l2.value, li.value
