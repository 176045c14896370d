"""Independent float64 dense restatement of the KF / EKF math (TEST INFRASTRUCTURE ONLY).

The KF path has no reference counterpart (the firmware
contains no Kalman filter); the north star defines it as

    predict:  x <- F x  (EKF: x <- f(x)),   P <- F P F^T + Q
    update:   S = H P H^T + R,  K = P H^T S^-1,  x += K y,  P -= K H P

This module evaluates exactly those textbook formulas with dense numpy float64
matrices (np.linalg.solve for S^-1, Joseph-stabilised P update), independently of
the Cholesky/packed formulation the oracle and the kernels share, so it checks the
math of both.  Measurements z are taken as given (the fp32 measurement frontends
are pinned separately).
"""
from __future__ import annotations

import numpy as np


def unpack(p, n):
    M = np.zeros((n, n))
    k = 0
    for i in range(n):
        for j in range(i + 1):
            M[i, j] = M[j, i] = p[k]
            k += 1
    return M


def pack(M):
    n = M.shape[0]
    return np.array([M[i, j] for i in range(n) for j in range(i + 1)])


def wrap_pi(a):
    return (a + np.pi) % (2 * np.pi) - np.pi


def kf_update(x, P, H, R, y):
    S = H @ P @ H.T + R
    K = np.linalg.solve(S, H @ P).T          # P H^T S^-1  (S symmetric)
    x = x + K @ y
    I_KH = np.eye(len(x)) - K @ H
    P = I_KH @ P @ I_KH.T + K @ R @ K.T     # Joseph form == P - K H P
    return x, P


# ----------------------------------------------------------------------------- KF6
def kf6_matrices(dt):
    F = np.eye(6)
    for i in range(3):
        F[i, i + 3] = dt
    H = np.zeros((4, 6))
    for a, s in enumerate((2, 5, 3, 4)):
        H[a, s] = 1.0
    return F, H


def kf6_run(x0, P0p, z_seq, q_packed, r_packed, dt, valid=None):
    """x0 [6], P0 packed [21], z_seq [T, 4] -> list of (x, P packed) after each tick."""
    F, H = kf6_matrices(dt)
    Q, R = unpack(q_packed, 6), unpack(r_packed, 4)
    x, P = np.array(x0, float), unpack(P0p, 6)
    out = []
    for t, z in enumerate(z_seq):
        if valid is None or valid[t]:
            y = z - H @ x
            y[0] = _wrap_innov(y[0])
            x, P = kf_update(x, P, H, R, y)
        x = F @ x
        x[2] = _wrap_state(x[2])
        P = F @ P @ F.T + Q
        out.append((x.copy(), pack(P)))
    return out


def _wrap_innov(a):
    if a > np.pi:
        return a - 2 * np.pi
    if a < -np.pi:
        return a + 2 * np.pi
    return a


def _wrap_state(a):
    if a >= np.pi:
        return a - 2 * np.pi
    if a < -np.pi:
        return a + 2 * np.pi
    return a


# ----------------------------------------------------------------------------- EKF9
def ekf9_H():
    H = np.zeros((6, 9))
    H[0, 2] = 1
    H[1, 5] = 1
    H[1, 6] = 1
    H[2, 7] = 1
    H[3, 8] = 1
    H[4, 3] = 1
    H[5, 4] = 1
    return H


def ekf9_run(x0, P0p, z_seq, q_packed, r_packed, dt):
    H = ekf9_H()
    Q, R = unpack(q_packed, 9), unpack(r_packed, 6)
    x, P = np.array(x0, float), unpack(P0p, 9)
    out = []
    for z in z_seq:
        y = z - H @ x
        y[0] = _wrap_innov(y[0])
        x, P = kf_update(x, P, H, R, y)
        th, vbx, vby = x[2], x[3], x[4]
        c, s = np.cos(th), np.sin(th)
        vwx, vwy = vbx * c - vby * s, vbx * s + vby * c
        F = np.eye(9)
        F[0, 2], F[0, 3], F[0, 4] = -vwy * dt, c * dt, -s * dt
        F[1, 2], F[1, 3], F[1, 4] = vwx * dt, s * dt, c * dt
        F[2, 5] = dt
        F[3, 7] = dt
        F[4, 8] = dt
        x = x.copy()
        x[0] += vwx * dt
        x[1] += vwy * dt
        x[2] = _wrap_state(x[2] + x[5] * dt)
        x[3] += x[7] * dt
        x[4] += x[8] * dt
        P = F @ P @ F.T + Q
        out.append((x.copy(), pack(P)))
    return out


# ----------------------------------------------------------------------------- KF12D
def kf12d_matrices(dt):
    F = np.eye(12)
    for p in (0, 1, 2, 6, 7, 8):
        F[p, p + 3] = dt
    H = np.zeros((8, 12))
    for a, s in enumerate((2, 5, 3, 4, 6, 7, 8, 11)):
        H[a, s] = 1.0
    return F, H


def kf12d_run(x0, P0p, z_seq, q_packed, r_packed, dt):
    F, H = kf12d_matrices(dt)
    Q, R = unpack(q_packed, 12), unpack(r_packed, 8)
    x, P = np.array(x0, float), unpack(P0p, 12)
    out = []
    for z in z_seq:
        y = z - H @ x
        y[0] = _wrap_innov(y[0])
        x, P = kf_update(x, P, H, R, y)
        x = F @ x
        x[2] = _wrap_state(x[2])
        P = F @ P @ F.T + Q
        out.append((x.copy(), pack(P)))
    return out


# ----------------------------------------------------------------------------- batched
# The same textbook formulas, vectorised over robots (x [N, n], P [N, n, n]) so that long
# horizons (60 000 ticks x 1000+ robots) run in seconds.  Identical maths to the per-robot
# functions above; tests/test_oracle_kf_fp64.py checks the two agree.
def _wrap_innov_v(a):
    return np.where(a > np.pi, a - 2 * np.pi, np.where(a < -np.pi, a + 2 * np.pi, a))


def _wrap_state_v(a):
    return np.where(a >= np.pi, a - 2 * np.pi, np.where(a < -np.pi, a + 2 * np.pi, a))


def kf_update_batch(x, P, H, R, y, mask=None):
    """x [N,n], P [N,n,n], y [N,m]; H [m,n], R [m,m] shared; mask [N] bool (None = all)."""
    n = x.shape[1]
    HP = H @ P                                          # [N, m, n]
    S = HP @ H.T + R                                    # [N, m, m]
    K = np.linalg.solve(S, HP).transpose(0, 2, 1)       # [N, n, m] = P H^T S^-1
    xn = x + np.einsum("nij,nj->ni", K, y)
    IKH = np.eye(n) - K @ H
    Pn = IKH @ P @ IKH.transpose(0, 2, 1) + K @ R @ K.transpose(0, 2, 1)
    if mask is not None:
        xn = np.where(mask[:, None], xn, x)
        Pn = np.where(mask[:, None, None], Pn, P)
    return xn, Pn


def _tril_idx(n):
    return np.tril_indices(n)


class Kf6Batch:
    """KF6 over N robots in float64: step(z [4, N], valid [N] or None) = one tick."""

    def __init__(self, n, x0, P0p, q_packed, r_packed, dt):
        self.F, self.H = kf6_matrices(dt)
        self.Q, self.R = unpack(q_packed, 6), unpack(r_packed, 4)
        self.x = np.tile(np.asarray(x0, float), (n, 1))
        self.P = np.tile(unpack(P0p, 6), (n, 1, 1))

    def step(self, z, valid=None):
        y = z.T - self.x @ self.H.T
        y[:, 0] = _wrap_innov_v(y[:, 0])
        m = None if valid is None else np.asarray(valid).astype(bool)
        self.x, self.P = kf_update_batch(self.x, self.P, self.H, self.R, y, m)
        self.x = self.x @ self.F.T
        self.x[:, 2] = _wrap_state_v(self.x[:, 2])
        self.P = self.F @ self.P @ self.F.T + self.Q

    def packed(self):
        """(x [n, N], P packed [n(n+1)/2, N]) in the engine's plane layout"""
        i, j = _tril_idx(6)
        return self.x.T.copy(), self.P[:, i, j].T.copy()


class Ekf9Batch:
    """EKF9 over N robots in float64 (same f(x) and F as ekf9_run)."""

    def __init__(self, n, x0, P0p, q_packed, r_packed, dt):
        self.H = ekf9_H()
        self.Q, self.R = unpack(q_packed, 9), unpack(r_packed, 6)
        self.dt = dt
        self.x = np.tile(np.asarray(x0, float), (n, 1))
        self.P = np.tile(unpack(P0p, 9), (n, 1, 1))

    def step(self, z, valid=None):
        dt = self.dt
        y = z.T - self.x @ self.H.T
        y[:, 0] = _wrap_innov_v(y[:, 0])
        m = None if valid is None else np.asarray(valid).astype(bool)
        x, P = kf_update_batch(self.x, self.P, self.H, self.R, y, m)
        th, vbx, vby = x[:, 2], x[:, 3], x[:, 4]
        c, s = np.cos(th), np.sin(th)
        vwx, vwy = vbx * c - vby * s, vbx * s + vby * c
        n = x.shape[0]
        F = np.tile(np.eye(9), (n, 1, 1))
        F[:, 0, 2], F[:, 0, 3], F[:, 0, 4] = -vwy * dt, c * dt, -s * dt
        F[:, 1, 2], F[:, 1, 3], F[:, 1, 4] = vwx * dt, s * dt, c * dt
        F[:, 2, 5] = dt
        F[:, 3, 7] = dt
        F[:, 4, 8] = dt
        x = x.copy()
        x[:, 0] += vwx * dt
        x[:, 1] += vwy * dt
        x[:, 2] = _wrap_state_v(x[:, 2] + x[:, 5] * dt)
        x[:, 3] += x[:, 7] * dt
        x[:, 4] += x[:, 8] * dt
        self.x = x
        self.P = F @ P @ F.transpose(0, 2, 1) + self.Q

    def packed(self):
        i, j = _tril_idx(9)
        return self.x.T.copy(), self.P[:, i, j].T.copy()


class Kf12dBatch:
    """KF12D over N robots in float64."""

    def __init__(self, n, x0, P0p, q_packed, r_packed, dt):
        self.F, self.H = kf12d_matrices(dt)
        self.Q, self.R = unpack(q_packed, 12), unpack(r_packed, 8)
        self.x = np.tile(np.asarray(x0, float), (n, 1))
        self.P = np.tile(unpack(P0p, 12), (n, 1, 1))

    def step(self, z, valid=None):
        y = z.T - self.x @ self.H.T
        y[:, 0] = _wrap_innov_v(y[:, 0])
        m = None if valid is None else np.asarray(valid).astype(bool)
        self.x, self.P = kf_update_batch(self.x, self.P, self.H, self.R, y, m)
        self.x = self.x @ self.F.T
        self.x[:, 2] = _wrap_state_v(self.x[:, 2])
        self.P = self.F @ self.P @ self.F.T + self.Q

    def packed(self):
        i, j = _tril_idx(12)
        return self.x.T.copy(), self.P[:, i, j].T.copy()


# ----------------------------------------------------------------------------- dense C (fast)
class DenseC:
    """The same textbook formulas in C (oracle/kf_dense_ref.c: full matrices, LU solve, Joseph
    update), batched over robots with OpenMP: the long-horizon reference.  model "kf6" | "ekf9";
    q / r packed (as the engine's config), dt float; step(z [m, N] float64, valid [N] u8|None)."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            import ctypes as C
            import os
            import subprocess
            here = os.path.dirname(os.path.abspath(__file__))
            subprocess.run(["make", "-s", "libkfref.so"], cwd=here, check=True, stdout=subprocess.DEVNULL)
            L = C.CDLL(os.path.join(here, "libkfref.so"))
            f64 = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
            for name in ("dref_kf6_step", "dref_ekf9_step"):
                fn = getattr(L, name)
                fn.argtypes = [C.c_int64, f64, f64, f64, C.c_void_p, f64, f64, C.c_double]
                fn.restype = None
            cls._lib = L
        return cls._lib

    def __init__(self, model, n, x0, P0p, q_packed, r_packed, dt):
        self.model, self.n, self.dt = model, n, float(dt)
        nx, m = (6, 4) if model == "kf6" else (9, 6)
        self.nx, self.m = nx, m
        self.Q = np.ascontiguousarray(unpack(q_packed, nx))
        self.R = np.ascontiguousarray(unpack(r_packed, m))
        self.x = np.ascontiguousarray(np.tile(np.asarray(x0, float), (n, 1)))
        self.P = np.ascontiguousarray(np.tile(unpack(P0p, nx), (n, 1, 1)))
        self.fn = getattr(self.lib(), "dref_kf6_step" if model == "kf6" else "dref_ekf9_step")

    def step(self, z, valid=None):
        import ctypes as C
        z = np.ascontiguousarray(z, np.float64)
        v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
        self.fn(self.n, self.x, self.P, z, None if v is None else v.ctypes.data_as(C.c_void_p),
                self.Q, self.R, self.dt)

    def packed(self):
        i, j = _tril_idx(self.nx)
        return self.x.T.copy(), self.P[:, i, j].T.copy()
