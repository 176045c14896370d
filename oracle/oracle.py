"""ctypes bindings for the oracle (liboracle.so) and the reference WT901 SDK build
(_ref/libwit_ref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libwit_ref.so")

TRIG_TABLE512 = 0
TRIG_LIBM = 1

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_vp = C.c_void_p


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and _ref/libwit_ref.so when the reference is present)."""
    kw = dict(cwd=HERE, check=True)
    if quiet:
        kw.update(stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-s", "liboracle.so"], **kw)
    if os.path.isdir("/root/reference/lib/wt901c"):
        subprocess.run(["make", "-s", "ref"], **kw)


class Wt901State(C.Structure):
    _fields_ = [
        ("buf", C.c_uint8 * 256),
        ("cnt", C.c_uint32),
        ("read_reg_index", C.c_uint32),
        ("reg", C.c_int16 * 0x90),
        ("flags", C.c_uint8),
        ("is_error", C.c_uint8),
        ("q_init", C.c_float * 4),
        ("data", C.c_float * 16),
        ("ncb", C.c_uint32),
        ("cb_reg", C.c_uint16 * 64),
        ("cb_num", C.c_uint16 * 64),
    ]


class M2006State(C.Structure):
    _fields_ = [
        ("micro", C.c_int16),
        ("angle", C.c_int16),
        ("rpm", C.c_int16),
        ("curr", C.c_int16),
        ("dlt_out_angle_rad", C.c_float),
        ("speed_radps", C.c_float),
        ("head", C.c_uint8),
        ("dir", C.c_int8),
        ("angle_sum", C.c_int64),
        ("iir_prev_y", C.c_float),
        ("iir_prev_x", C.c_float),
    ]


class Kf6Params(C.Structure):
    _fields_ = [("dt", C.c_float), ("dt2", C.c_float), ("q", C.c_float * 21),
                ("r", C.c_float * 10), ("trig", C.c_int)]


class Ekf9Params(C.Structure):
    _fields_ = [("dt", C.c_float), ("dt2", C.c_float), ("q", C.c_float * 45),
                ("r", C.c_float * 21), ("trig", C.c_int)]


class Kf12dParams(C.Structure):
    _fields_ = [("dt", C.c_double), ("dt2", C.c_double), ("q", C.c_double * 78),
                ("r", C.c_double * 36)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_deg2rad.restype = C.c_float
        L.orc_deg2rad.argtypes = [C.c_float]
        L.orc_normalize_rad_0to2pi.restype = C.c_float
        L.orc_normalize_rad_0to2pi.argtypes = [C.c_float]
        L.orc_normalize_deg_0to360.restype = C.c_float
        L.orc_normalize_deg_0to360.argtypes = [C.c_float]
        L.orc_sin.restype = C.c_float
        L.orc_sin.argtypes = [C.c_float, C.c_int]
        L.orc_cos.restype = C.c_float
        L.orc_cos.argtypes = [C.c_float, C.c_int]
        L.orc_eval_trig.argtypes = [_f32p, _f32p, _f32p, C.c_size_t, C.c_int]
        L.orc_sin_table.argtypes = [_f32p]
        L.orc_mdir_to_vdir.argtypes = [_f32p, _f32p]
        L.orc_vdir_to_mdir.argtypes = [_f32p, _f32p]
        L.orc_wt901_reset.argtypes = [C.POINTER(Wt901State), C.c_uint32]
        L.orc_wt901_update.argtypes = [C.POINTER(Wt901State), _u8p, C.c_uint32, C.c_int]
        L.orc_wt901_is_com_comp.argtypes = [C.POINTER(Wt901State), _u8p, C.c_uint32]
        L.orc_wt901_is_com_comp.restype = C.c_int
        L.orc_m2006_reset.argtypes = [C.POINTER(M2006State), C.c_int]
        L.orc_m2006_rx.argtypes = [C.POINTER(M2006State), _u8p, C.c_int16]
        L.orc_rs_tick.argtypes = [C.c_size_t, _f32p, _f32p, _i64p, _vp, _i64p, _i16p,
                                  C.c_int, C.c_int, C.c_int]
        L.orc_kf6_tick.argtypes = [C.c_size_t, _f32p, _f32p, _vp, _vp, _vp, _vp,
                                   C.POINTER(Kf6Params), C.c_int, C.c_int, C.c_int]
        L.orc_kf6_measure.argtypes = [C.c_size_t, _f32p, _f32p, _i16p, _f32p, C.c_int]
        L.orc_ekf9_tick.argtypes = [C.c_size_t, _f32p, _f32p, _vp, _vp,
                                    C.POINTER(Ekf9Params), C.c_int, C.c_int, C.c_int]
        L.orc_ekf9_measure.argtypes = [C.c_size_t, _i16p, _f32p]
        L.orc_kf12d_tick.argtypes = [C.c_size_t, _f64p, _f64p, _vp, _vp,
                                     C.POINTER(Kf12dParams), C.c_int, C.c_int, C.c_int]
        L.orc_ens_record_len.restype = C.c_size_t
        L.orc_ens_record_len.argtypes = [C.c_int]
        L.orc_ens_partial_f32.argtypes = [C.c_size_t, C.c_int, _f32p, C.c_size_t, C.c_size_t, _f64p]
        L.orc_ens_partial_f64.argtypes = [C.c_size_t, C.c_int, _f64p, C.c_size_t, C.c_size_t, _f64p]
        L.orc_ens_combine.argtypes = [C.c_int, _f64p, _f64p, _f64p]
        L.orc_ens_finalize.argtypes = [C.c_int, _f64p, _f64p, _f64p]
        L.orc_max_threads.restype = C.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------------------------- scalar
def deg2rad(d: float) -> float:
    return lib().orc_deg2rad(d)


def normalize_rad_0to2pi(d: float) -> float:
    return lib().orc_normalize_rad_0to2pi(d)


def normalize_deg_0to360(d: float) -> float:
    return lib().orc_normalize_deg_0to360(d)


def eval_trig(x, trig=TRIG_TABLE512):
    x = np.ascontiguousarray(x, np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().orc_eval_trig(x, s, c, x.size, trig)
    return s, c


def sin_table():
    t = np.empty(513, np.float32)
    lib().orc_sin_table(t)
    return t


def mdir_to_vdir(m):
    m = np.ascontiguousarray(m, np.float32)
    v = np.empty(3, np.float32)
    lib().orc_mdir_to_vdir(m, v)
    return v


# ----------------------------------------------------------------------------- WT901
class Wt901:
    """One IMU_IF_WT901C instance (parser + register file + Data page)."""

    def __init__(self, read_reg_index: int = 0x51):
        self.s = Wt901State()
        lib().orc_wt901_reset(C.byref(self.s), read_reg_index)

    def update(self, data: bytes | np.ndarray, latch_qinit: bool = False):
        b = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        b = np.ascontiguousarray(b, np.uint8)
        if b.size == 0:
            b = np.zeros(1, np.uint8)
            lib().orc_wt901_update(C.byref(self.s), b, 0, int(latch_qinit))
        else:
            lib().orc_wt901_update(C.byref(self.s), b, b.size, int(latch_qinit))

    def feed(self, data) -> bool:
        b = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        if b.size == 0:
            b = np.zeros(1, np.uint8)
            return bool(lib().orc_wt901_is_com_comp(C.byref(self.s), b, 0))
        return bool(lib().orc_wt901_is_com_comp(C.byref(self.s), b, b.size))

    def take_cb(self):
        n = self.s.ncb
        out = [(self.s.cb_reg[i], self.s.cb_num[i]) for i in range(n)]
        self.s.ncb = 0
        return out

    @property
    def regs(self):
        return np.ctypeslib.as_array(self.s.reg).copy()

    @property
    def data(self):
        return np.ctypeslib.as_array(self.s.data).copy()

    @property
    def is_error(self):
        return bool(self.s.is_error)

    @property
    def parser(self):
        return bytes(self.s.buf[: self.s.cnt])


# ----------------------------------------------------------------------------- CAN
class M2006:
    def __init__(self, direction: int = 1):
        self.s = M2006State()
        lib().orc_m2006_reset(C.byref(self.s), direction)

    def rx(self, frame, micro: int):
        f = np.ascontiguousarray(np.frombuffer(bytes(frame), np.uint8))
        lib().orc_m2006_rx(C.byref(self.s), f, int(np.int16(micro)))


# ----------------------------------------------------------------------------- RS tick
def rs_tick(pos, vel, prev, yaw_deg, angle_sum, rpm, trig=TRIG_TABLE512, do_correct=True,
            do_predict=True):
    n = pos.shape[1]
    lib().orc_rs_tick(n, pos, vel, prev, _ptr(yaw_deg), angle_sum, rpm, trig, int(do_correct),
                      int(do_predict))


# ----------------------------------------------------------------------------- KF
def kf6_params(dt, q_packed, r_packed, trig=TRIG_TABLE512):
    p = Kf6Params()
    p.dt = np.float32(dt)
    p.dt2 = np.float32(np.float32(dt) * np.float32(dt))
    for i, v in enumerate(np.asarray(q_packed, np.float32)):
        p.q[i] = v
    for i, v in enumerate(np.asarray(r_packed, np.float32)):
        p.r[i] = v
    p.trig = trig
    return p


def kf6_tick(x, P, yaw, gz, rpm, valid, prm, do_update=True, do_predict=True, nthreads=1):
    n = x.shape[1]
    lib().orc_kf6_tick(n, x, P, _ptr(yaw), _ptr(gz), _ptr(rpm), _ptr(valid), C.byref(prm),
                       int(do_update), int(do_predict), nthreads)


def kf6_measure(yaw, gz, rpm, trig=TRIG_TABLE512):
    n = yaw.size
    z = np.empty((4, n), np.float32)
    lib().orc_kf6_measure(n, yaw, gz, rpm, z, trig)
    return z


def ekf9_params(dt, q_packed, r_packed, trig=TRIG_TABLE512):
    p = Ekf9Params()
    p.dt = np.float32(dt)
    p.dt2 = np.float32(np.float32(dt) * np.float32(dt))
    for i, v in enumerate(np.asarray(q_packed, np.float32)):
        p.q[i] = v
    for i, v in enumerate(np.asarray(r_packed, np.float32)):
        p.r[i] = v
    p.trig = trig
    return p


def ekf9_tick(x, P, raw, valid, prm, do_update=True, do_predict=True, nthreads=1):
    n = x.shape[1]
    lib().orc_ekf9_tick(n, x, P, _ptr(raw), _ptr(valid), C.byref(prm), int(do_update),
                        int(do_predict), nthreads)


def ekf9_measure(raw):
    n = raw.shape[0]
    z = np.empty((6, n), np.float32)
    lib().orc_ekf9_measure(n, np.ascontiguousarray(raw, np.int16), z)
    return z


def kf12d_params(dt, q_packed, r_packed):
    p = Kf12dParams()
    p.dt = float(dt)
    p.dt2 = float(dt) * float(dt)
    for i, v in enumerate(np.asarray(q_packed, np.float64)):
        p.q[i] = v
    for i, v in enumerate(np.asarray(r_packed, np.float64)):
        p.r[i] = v
    return p


def kf12d_tick(x, P, z, valid, prm, do_update=True, do_predict=True, nthreads=1):
    n = x.shape[1]
    lib().orc_kf12d_tick(n, x, P, _ptr(z), _ptr(valid), C.byref(prm), int(do_update),
                         int(do_predict), nthreads)


# ----------------------------------------------------------------------------- ensemble
def ens_partial(x, lo=0, hi=None):
    nx, n = x.shape
    hi = n if hi is None else hi
    rec = np.zeros(lib().orc_ens_record_len(nx), np.float64)
    if x.dtype == np.float32:
        lib().orc_ens_partial_f32(n, nx, np.ascontiguousarray(x), lo, hi, rec)
    else:
        lib().orc_ens_partial_f64(n, nx, np.ascontiguousarray(x, np.float64), lo, hi, rec)
    return rec


def ens_combine(nx, a, b):
    out = np.zeros_like(a)
    lib().orc_ens_combine(nx, np.ascontiguousarray(a), np.ascontiguousarray(b), out)
    return out


def ens_finalize(nx, rec):
    mean = np.zeros(nx, np.float64)
    cov = np.zeros(nx * (nx + 1) // 2, np.float64)
    lib().orc_ens_finalize(nx, np.ascontiguousarray(rec), mean, cov)
    return mean, cov


def max_threads() -> int:
    return lib().orc_max_threads()


# ----------------------------------------------------------------------------- reference SDK
class RefWt901:
    """The reference's own lib/wt901c/wit_c_sdk.c (oracle/_ref/libwit_ref.so).

    Only available where /root/reference existed at build time; the fixtures it
    produced are committed under tests/golden/."""

    _l = None

    def __init__(self, read_reg_index: int = 0x51):
        if RefWt901._l is None:
            if not os.path.exists(REF_PATH):
                raise FileNotFoundError(REF_PATH)
            L = C.CDLL(REF_PATH)
            L.ref_wt901_begin.argtypes = [C.c_uint32]
            L.ref_wt901_begin.restype = C.c_int
            L.ref_wt901_feed.argtypes = [_u8p, C.c_uint32]
            L.ref_wt901_regs.argtypes = [_i16p]
            L.ref_wt901_take_cb.argtypes = [_u16p, _u16p, C.c_uint32]
            L.ref_wt901_take_cb.restype = C.c_uint32
            RefWt901._l = L
        rc = RefWt901._l.ref_wt901_begin(read_reg_index)
        if rc != 0:
            raise RuntimeError(f"WitReadReg failed: {rc}")

    def feed(self, data):
        b = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
        if b.size:
            RefWt901._l.ref_wt901_feed(b, b.size)

    def regs(self):
        out = np.zeros(0x90, np.int16)
        RefWt901._l.ref_wt901_regs(out)
        return out

    def take_cb(self):
        r = np.zeros(4096, np.uint16)
        m = np.zeros(4096, np.uint16)
        n = RefWt901._l.ref_wt901_take_cb(r, m, 4096)
        return list(zip(r[:n].tolist(), m[:n].tolist()))
