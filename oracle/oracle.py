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
REF_CTRL_PATH = os.path.join(HERE, "_ref", "libctrl_ref.so")

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
    subprocess.run(["make", "-s", "liboracle.so", "libkfref.so", "libcpuport_v3.so", "libcpuport_v4.so"], **kw)
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


class Interp(C.Structure):  # orc_interp (util_vel_interp.hpp:25-157)
    _fields_ = [(f, C.c_float) for f in ("vel_tgt", "acl_max", "jerk_p", "jerk_m", "dt1", "dt2",
                                          "dt3", "vel_ini", "acl_ini", "dt", "vel_now", "acl_now")]


class Pid(C.Structure):  # orc_pid (util_controller.hpp FF_PI_D state)
    _fields_ = [(f, C.c_float) for f in ("val", "integ", "lpf_y", "lpf_x", "tgt", "ctrl")]


class CtrlParams(C.Structure):
    _fields_ = [(f, C.c_float) for f in ("freq", "dt", "ff_gain", "p_gain", "i_gain", "d_gain",
                                          "i_limit", "ff_limit", "a1", "b0", "b1", "ts")] + \
               [("curr_limit_raw", C.c_int16)]


class Ctrl(C.Structure):  # orc_ctrl: one robot's control state
    _fields_ = [("ax", Interp * 3), ("pid", Pid * 4), ("curr", C.c_int16 * 4),
                ("vel_tgt", C.c_float * 3), ("power", C.c_uint8)]


class VehicleInfo(C.Structure):  # orc_vehicle_info (VehicleInfo.msg layout, 84 B)
    _fields_ = [("pos_x", C.c_int32), ("pos_y", C.c_int32), ("pos_theta", C.c_float),
                ("vel_x", C.c_int32), ("vel_y", C.c_int32), ("vel_theta", C.c_float),
                ("imu_fault", C.c_uint8), ("pad_", C.c_uint8 * 3), ("imu_q", C.c_float * 4),
                ("imu_g", C.c_float * 3), ("imu_a", C.c_float * 3), ("floor", C.c_uint8 * 8),
                ("cam_pitch", C.c_float), ("fault", C.c_uint32)]


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
        L.orc_wt901_update_batch.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
        L.orc_wt901_update_batch.restype = None
        L.orc_can_ingest_batch.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_can_ingest_batch.restype = None
        L.orc_rs_tick.argtypes = [C.c_size_t, _f32p, _f32p, _i64p, _vp, _i64p, _i16p,
                                  C.c_int, C.c_int, C.c_int]
        L.orc_kf6_tick.argtypes = [C.c_size_t, _f32p, _f32p, _vp, _vp, _vp, _vp,
                                   C.POINTER(Kf6Params), C.c_int, C.c_int, C.c_int]
        L.orc_kf6_tick_comp.argtypes = [C.c_size_t, _f32p, _f32p, _f32p, _vp, _vp, _vp, _vp,
                                        C.POINTER(Kf6Params), C.c_int, C.c_int, C.c_int]
        L.orc_kf6_measure.argtypes = [C.c_size_t, _f32p, _f32p, _i16p, _f32p, C.c_int]
        L.orc_ekf9_tick.argtypes = [C.c_size_t, _f32p, _f32p, _vp, _vp,
                                    C.POINTER(Ekf9Params), C.c_int, C.c_int, C.c_int]
        L.orc_ekf9_tick_comp.argtypes = [C.c_size_t, _f32p, _f32p, _f32p, _vp, _vp,
                                         C.POINTER(Ekf9Params), C.c_int, C.c_int, C.c_int]
        L.orc_ekf9_measure.argtypes = [C.c_size_t, _i16p, _f32p]
        L.orc_kf12d_tick.argtypes = [C.c_size_t, _f64p, _f64p, _vp, _vp,
                                     C.POINTER(Kf12dParams), C.c_int, C.c_int, C.c_int]
        L.orc_kf12d_cinv.restype = C.c_int
        L.orc_kf12d_cinv.argtypes = [_f64p, _f64p]
        L.orc_ens_record_len.restype = C.c_size_t
        L.orc_ens_record_len.argtypes = [C.c_int]
        L.orc_ens_partial_f32.argtypes = [C.c_size_t, C.c_int, _f32p, C.c_size_t, C.c_size_t, _f64p]
        L.orc_ens_partial_f64.argtypes = [C.c_size_t, C.c_int, _f64p, C.c_size_t, C.c_size_t, _f64p]
        L.orc_ens_combine.argtypes = [C.c_int, _f64p, _f64p, _f64p]
        L.orc_ens_finalize.argtypes = [C.c_int, _f64p, _f64p, _f64p]
        L.orc_max_threads.restype = C.c_int
        L.orc_ctrl_params_make.argtypes = [C.POINTER(CtrlParams)] + [C.c_float] * 9 + [C.c_int16]
        L.orc_interp_reset.argtypes = [C.POINTER(Interp)]
        L.orc_interp_set.argtypes = [C.POINTER(Interp), C.c_float, C.c_float, C.c_float]
        L.orc_interp_update.argtypes = [C.POINTER(Interp), C.c_float]
        L.orc_interp_update.restype = C.c_float
        L.orc_pid_reset.argtypes = [C.POINTER(Pid)]
        L.orc_pid_update.argtypes = [C.POINTER(Pid), C.POINTER(CtrlParams), C.c_float]
        L.orc_pid_update.restype = C.c_float
        L.orc_curr_to_raw.argtypes = [C.c_float, C.c_int, C.c_int16]
        L.orc_curr_to_raw.restype = C.c_int16
        L.orc_can_tx.argtypes = [_i16p, _u8p]
        L.orc_ctrl_reset.argtypes = [C.POINTER(Ctrl)]
        L.orc_ctrl_step_batch.argtypes = [C.c_size_t, _vp, C.POINTER(CtrlParams), _i16p, _vp]
        L.orc_f2i32_arm.argtypes = [C.c_float]
        L.orc_f2i32_arm.restype = C.c_int32
        L.orc_f2u32_arm.argtypes = [C.c_float]
        L.orc_f2u32_arm.restype = C.c_uint32
        L.orc_vehicle_info_fill.argtypes = [C.POINTER(VehicleInfo)] + [C.c_float] * 6 + \
            [_f32p, C.c_uint8, _vp, C.c_float, C.c_uint32]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------------------------- CPU baseline port
_port = None


def port_isa() -> str:
    """the widest cpu_port build this host runs: 'v4' (AVX-512 F/BW/CD/DQ/VL) or 'v3' (AVX2)"""
    flags = set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        pass
    return "v4" if {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"} <= flags else "v3"


def port():
    """oracle/cpu_port.c (bench.py's CPU baseline; bit-exact to orc_kf6_tick / orc_rs_tick)"""
    global _port
    if _port is None:
        path = os.path.join(HERE, f"libcpuport_{port_isa()}.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.port_kf6_tick.argtypes = [C.c_size_t, _f32p, _f32p, _vp, _vp, _vp, C.POINTER(Kf6Params), C.c_int]
        L.port_kf6_tick.restype = C.c_int
        L.port_rs_tick.argtypes = [C.c_size_t, _f32p, _f32p, _i64p, _vp, _i64p, _i16p, C.c_int, C.c_int]
        L.port_rs_tick.restype = C.c_int
        L.port_max_threads.restype = C.c_int
        L.isa = port_isa()
        _port = L
    return _port


def port_kf6_tick(x, P, yaw, gz, rpm, prm, nthreads=0):
    """the tuned KF6 tick (no validity mask, TABLE512): same bits as kf6_tick"""
    n = x.shape[1]
    assert port().port_kf6_tick(n, x, P, _ptr(yaw), _ptr(gz), _ptr(rpm), C.byref(prm), nthreads) == 0


def port_rs_tick(pos, vel, prev, yaw_deg, angle_sum, rpm, nthreads=0):
    """the tuned reference-semantics tick (TABLE512): same bits as rs_tick"""
    n = pos.shape[1]
    assert port().port_rs_tick(n, pos, vel, prev, _ptr(yaw_deg), angle_sum, rpm, TRIG_TABLE512, nthreads) == 0


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


def _struct_view(arr, cls):
    """numpy structured view of a ctypes array of `cls`, laid out from the ctypes field offsets"""
    names, formats, offsets = [], [], []
    for name, ct in cls._fields_:
        base, shape = ct, ()
        while hasattr(base, "_length_"):
            shape += (base._length_,)
            base = base._type_
        names.append(name)
        formats.append((np.dtype(base), shape) if shape else np.dtype(base))
        offsets.append(getattr(cls, name).offset)
    dt = np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": C.sizeof(cls)})
    return np.frombuffer(arr, dtype=dt)


class Wt901Batch:
    """n IMU_IF_WT901C instances updated by one C call per poll (orc_wt901_update_batch, the
    per-instance orc_wt901_update in a loop)."""

    def __init__(self, n: int, read_reg_index: int = 0x51):
        self.n = n
        self.s = (Wt901State * n)()
        for i in range(n):
            lib().orc_wt901_reset(C.byref(self.s[i]), read_reg_index)

    def update(self, buf, lens, latch_qinit: bool = False):
        """buf [n][stride] uint8 rows, lens [n]: one poll per instance"""
        buf = np.ascontiguousarray(buf, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        assert buf.shape[0] == self.n and lens.shape == (self.n,)
        lib().orc_wt901_update_batch(self.n, C.cast(self.s, C.c_void_p), buf.ctypes.data_as(C.c_void_p),
                                     buf.shape[1], lens.ctypes.data_as(C.c_void_p), int(latch_qinit))

    @property
    def data(self):
        """[16][n] Data pages"""
        return np.ascontiguousarray(_struct_view(self.s, Wt901State)["data"].T)

    @property
    def is_error(self):
        return _struct_view(self.s, Wt901State)["is_error"].copy()


class MotorBatch:
    """n robots' four MOTOR_IF_M2006 instances fed by one C call per tick (orc_can_ingest_batch)."""

    def __init__(self, n: int, dirs=(1, 1, -1, -1)):
        self.n = n
        self.m = (M2006State * (4 * n))()
        for i in range(n):
            for w in range(4):
                lib().orc_m2006_reset(C.byref(self.m[4 * i + w]), int(dirs[w]))

    def rx(self, frames, stamps):
        """frames [n][4][8] uint8, stamps [n][4] int16, every wheel present"""
        frames = np.ascontiguousarray(frames, np.uint8)
        stamps = np.ascontiguousarray(stamps, np.int16)
        assert frames.shape == (self.n, 4, 8) and stamps.shape == (self.n, 4)
        lib().orc_can_ingest_batch(self.n, C.cast(self.m, C.c_void_p), frames.ctypes.data_as(C.c_void_p),
                                   stamps.ctypes.data_as(C.c_void_p), None)

    def field(self, name):
        """[n][4] of one M2006 field"""
        return _struct_view(self.m, M2006State)[name].reshape(self.n, 4).copy()


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


def kf6_tick_comp(x, P, lo, yaw, gz, rpm, valid, prm, do_update=True, do_predict=True, nthreads=1):
    """KF6 with compensated positions (FMSKF_CFG_COMP_POS): lo [5][n] float32, the low parts of
    px, py, P00, P10, P11 (oracle/fmskf_oracle.c orc_kf6_tick_comp)"""
    n = x.shape[1]
    assert lo.shape == (5, n) and lo.dtype == np.float32 and lo.flags.c_contiguous
    lib().orc_kf6_tick_comp(n, x, P, lo, _ptr(yaw), _ptr(gz), _ptr(rpm), _ptr(valid), C.byref(prm),
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
    """x [10, n]: the 9 states and, in row 9, the compensated heading's low part (zero at start;
    the library keeps it as a hidden row: its x[2] is row 2 here, bit for bit)"""
    if x.shape[0] != 10:
        raise ValueError("ekf9_tick: x needs 10 rows (row 9: the heading's low part)")
    n = x.shape[1]
    lib().orc_ekf9_tick(n, x, P, _ptr(raw), _ptr(valid), C.byref(prm), int(do_update),
                        int(do_predict), nthreads)


def ekf9_tick_comp(x, P, clo, raw, valid, prm, do_update=True, do_predict=True, nthreads=1):
    """EKF9 with compensated positions (FMSKF_CFG_COMP_POS): clo [5][n] float32 (px, py, P00,
    P10, P11 low parts); x [10][n] keeps the heading's low part in row 9 as ekf9_tick"""
    n = x.shape[1]
    assert clo.shape == (5, n) and clo.dtype == np.float32 and clo.flags.c_contiguous
    lib().orc_ekf9_tick_comp(n, x, P, clo, _ptr(raw), _ptr(valid), C.byref(prm), int(do_update),
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


def kf12d_cinv(r_packed):
    """(ok, Cinv packed [36]) of R = C C^T; ok False when R is not positive definite."""
    ci = np.zeros(36, np.float64)
    ok = lib().orc_kf12d_cinv(np.ascontiguousarray(r_packed, np.float64), ci)
    return ok, ci


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


# ----------------------------------------------------------------------------- control step
# VD_task_main.cpp:86-89 (FF_PI_D(100 Hz, FF 0.0075, P 0.02, I 0.01, D 0, I-lim 0.5, LPF 10 Hz)),
# :157-160 (FF limit 1), :95-97 (interpolators at 1/1000 s), VD_motor_if_m2006.hpp:62 (3000)
CTRL_DEFAULTS = dict(c_freq=100.0, ff=0.0075, pg=0.02, ig=0.01, dg=0.0, ilim=0.5, lpf=10.0,
                     fflim=1.0, ts=np.float32(1.0) / np.float32(1000.0), clim=3000)


def ctrl_params(**kw):
    a = dict(CTRL_DEFAULTS)
    a.update(kw)
    p = CtrlParams()
    lib().orc_ctrl_params_make(C.byref(p), a["c_freq"], a["ff"], a["pg"], a["ig"], a["dg"],
                               a["ilim"], a["lpf"], a["fflim"], float(a["ts"]), int(a["clim"]))
    return p


class CtrlBatch:
    """n robots' VEHICLE_CTRL control state (orc_ctrl array)."""

    def __init__(self, n, prm=None, motor_dir=(1, 1, -1, -1)):
        self.n = n
        self.c = (Ctrl * n)()
        for i in range(n):
            lib().orc_ctrl_reset(C.byref(self.c[i]))
        self.p = prm if prm is not None else ctrl_params()
        self.dir = np.ascontiguousarray(np.asarray(motor_dir, np.int8))

    def set_power(self, on):
        on = np.broadcast_to(np.asarray(on, np.uint8), (self.n,))
        for i in range(self.n):
            self.c[i].power = int(on[i])

    def set_target_vel(self, vel, acl, jrk, mask=None):
        """vel/acl/jrk [3][n] (x, y, th) -> VelInterpConstJerk::set_target_params per axis"""
        vel, acl, jrk = (np.asarray(a, np.float32) for a in (vel, acl, jrk))
        for i in range(self.n):
            if mask is not None and not mask[i]:
                continue
            for a in range(3):
                lib().orc_interp_set(C.byref(self.c[i].ax[a]), float(vel[a, i]), float(acl[a, i]),
                                     float(jrk[a, i]))

    def step(self, rpm):
        rpm = np.ascontiguousarray(rpm, np.int16)
        lib().orc_ctrl_step_batch(self.n, C.cast(self.c, C.c_void_p), C.byref(self.p), rpm,
                                  self.dir.ctypes.data_as(C.c_void_p))

    def curr(self):
        return np.array([[self.c[i].curr[w] for w in range(4)] for i in range(self.n)], np.int16)

    def vel_tgt(self):
        return np.array([[self.c[i].vel_tgt[a] for i in range(self.n)] for a in range(3)], np.float32)

    def wheel(self, field):
        """FF_PI_D field ('tgt', 'ctrl', 'val', 'integ', ...) as [4][n]"""
        return np.array([[getattr(self.c[i].pid[w], field) for i in range(self.n)]
                         for w in range(4)], np.float32)


def can_tx(cur):
    cur = np.ascontiguousarray(cur, np.int16).reshape(-1, 4)
    out = np.zeros((cur.shape[0], 8), np.uint8)
    for i in range(cur.shape[0]):
        row = np.ascontiguousarray(out[i])
        lib().orc_can_tx(np.ascontiguousarray(cur[i]), row)
        out[i] = row
    return out


def f2i32_arm(f) -> int:
    return lib().orc_f2i32_arm(float(np.float32(f)))


def f2u32_arm(f) -> int:
    return lib().orc_f2u32_arm(float(np.float32(f)))


def vehicle_info(px, py, pth, vx, vy, vth, imu_data, is_error, floor=None, cam_pitch=0.0,
                 fault=0):
    """[n] VehicleInfo records (RM_task_main.cpp:772-823) as a structured numpy array"""
    n = len(px)
    out = (VehicleInfo * n)()
    for i in range(n):
        fl = None if floor is None else np.ascontiguousarray(floor[i], np.uint8)
        lib().orc_vehicle_info_fill(C.byref(out[i]), float(px[i]), float(py[i]), float(pth[i]),
                                    float(vx[i]), float(vy[i]), float(vth[i]),
                                    np.ascontiguousarray(imu_data[:, i], np.float32),
                                    int(is_error[i]), _ptr(fl),
                                    float(np.broadcast_to(cam_pitch, (n,))[i]),
                                    int(np.broadcast_to(fault, (n,))[i]))
    return np.frombuffer(bytes(out), dtype=VEHICLE_INFO_DTYPE).copy()


VEHICLE_INFO_DTYPE = np.dtype([("pos_x", "<i4"), ("pos_y", "<i4"), ("pos_theta", "<f4"),
                               ("vel_x", "<i4"), ("vel_y", "<i4"), ("vel_theta", "<f4"),
                               ("imu_fault", "u1"), ("pad_", "u1", 3), ("imu_q", "<f4", 4),
                               ("imu_g", "<f4", 3), ("imu_a", "<f4", 3), ("floor", "u1", 8),
                               ("cam_pitch", "<f4"), ("fault", "<u4")])


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


# ----------------------------------------------------------------------------- reference FF_PI_D
class RefFfPiD:
    """The reference's own UTIL::FF_PI_D (src/Utility/util_controller.hpp), compiled from
    /root/reference into oracle/_ref/libctrl_ref.so.  Only where the reference existed at build
    time; the fixtures it produced are committed under tests/golden/."""

    _l = None

    @classmethod
    def lib(cls):
        if cls._l is None:
            if not os.path.exists(REF_CTRL_PATH):
                raise FileNotFoundError(REF_CTRL_PATH)
            L = C.CDLL(REF_CTRL_PATH)
            L.ref_ffpid_run.argtypes = [C.c_float] * 8 + [C.c_int, _f32p, _f32p, _vp, _f32p, _f32p, _f32p]
            L.ref_iir1_run.argtypes = [C.c_float] * 3 + [C.c_int, _f32p, _f32p]
            cls._l = L
        return cls._l

    @classmethod
    def run(cls, tgt, val, reset=None, c_freq=100.0, ff=0.0075, pg=0.02, ig=0.01, dg=0.0, ilim=0.5,
            lpf=10.0, fflim=1.0):
        tgt = np.ascontiguousarray(tgt, np.float32)
        val = np.ascontiguousarray(val, np.float32)
        n = tgt.size
        ctrl, now_val, target = (np.zeros(n, np.float32) for _ in range(3))
        rs = None if reset is None else np.ascontiguousarray(reset, np.uint8)
        cls.lib().ref_ffpid_run(c_freq, ff, pg, ig, dg, ilim, lpf, fflim, n, tgt, val, _ptr(rs),
                                ctrl, now_val, target)
        return ctrl, now_val, target
