"""ctypes binding of libfmskf.so (include/fmskf.h).

The library is the product: every compute entry point launches a gfx950 HIP
kernel.  There is no CPU fallback -- if the shared library or a GPU is missing,
calls raise FmskfError.

torch (when importable) is imported BEFORE libfmskf.so is loaded so that both
resolve libamdhip64.so.7 to the same HIP runtime instance (torch's bundled
copy carries that soname); device pointers and hipStream_t handles can then be
exchanged with torch tensors/streams freely.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # share torch's HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C ABI itself
    torch = None

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FMSKF_LIB", os.path.join(PKG_ROOT, "lib", "libfmskf.so"))

OK, EINVAL, ENOMEM, EDEVICE, ERCCL, ENOTSUP = range(6)
MODEL_RS, MODEL_KF6, MODEL_EKF9, MODEL_KF12D = range(4)
TRIG_TABLE512, TRIG_LIBM = 0, 1
MEM_HOST, MEM_DEVICE = 0, 1
ABI_VERSION = 3
CFG_COMP_POS = 1

MODEL_NAMES = {"rs": MODEL_RS, "kf6": MODEL_KF6, "ekf9": MODEL_EKF9, "kf12d": MODEL_KF12D}


class FmskfError(RuntimeError):
    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"{what}: status {code}: {msg}")
        self.code = code


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("model", C.c_uint32),
        ("n_instances", C.c_uint64),
        ("device", C.c_int32),
        ("trig", C.c_uint32),
        ("dt", C.c_double),
        ("q", C.c_double * 78),
        ("r", C.c_double * 36),
        ("p0", C.c_double * 78),
        ("motor_dir", C.c_int8 * 4),
        ("imu_read_reg", C.c_uint32),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class TickInputs(C.Structure):
    _fields_ = [
        ("mem", C.c_uint32),
        ("angle_sum_pitch", C.c_uint32),
        ("yaw_deg", C.c_void_p),
        ("gyro_z_dps", C.c_void_p),
        ("rpm", C.c_void_p),
        ("angle_sum", C.c_void_p),
        ("raw", C.c_void_p),
        ("z", C.c_void_p),
        ("valid", C.c_void_p),
        ("kf6_rec", C.c_void_p),
    ]


class CtrlParams(C.Structure):
    _fields_ = [(f, C.c_float) for f in ("ctrl_freq_hz", "ff_gain", "p_gain", "i_gain", "d_gain",
                                          "i_limit", "lpf_freq_hz", "ff_limit", "interp_ts")] + \
               [("curr_limit_raw", C.c_int16), ("reserved", C.c_int16)]


class VehicleInfo(C.Structure):
    _fields_ = [("pos_x", C.c_int32), ("pos_y", C.c_int32), ("pos_theta", C.c_float),
                ("vel_x", C.c_int32), ("vel_y", C.c_int32), ("vel_theta", C.c_float),
                ("imu_fault", C.c_uint8), ("pad_", C.c_uint8 * 3), ("imu_q", C.c_float * 4),
                ("imu_g", C.c_float * 3), ("imu_a", C.c_float * 3), ("floor", C.c_uint8 * 8),
                ("cam_pitch", C.c_float), ("fault", C.c_uint32)]


# every symbol include/fmskf.h declares, with its ctypes signature
_H = C.c_void_p
_P = C.c_void_p
SIGNATURES = {
    "fmskf_config_init": (C.c_int, [C.POINTER(Config), C.c_uint32, C.c_uint64]),
    "fmskf_create": (C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "fmskf_destroy": (C.c_int, [_H]),
    "fmskf_reset": (C.c_int, [_H]),
    "fmskf_set_stream": (C.c_int, [_H, _P]),
    "fmskf_sync": (C.c_int, [_H]),
    "fmskf_get_config": (C.c_int, [_H, C.POINTER(Config)]),
    "fmskf_strerror": (C.c_char_p, [C.c_int]),
    "fmskf_last_error": (C.c_char_p, []),
    "fmskf_abi_version": (C.c_int, []),
    "fmskf_model_dims": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32)]),
    "fmskf_ingest_wt901": (C.c_int, [_H, _P, C.c_uint32, _P, C.c_int, C.c_uint32]),
    "fmskf_ingest_can": (C.c_int, [_H, _P, _P, _P, C.c_uint32]),
    "fmskf_correct": (C.c_int, [_H, C.POINTER(TickInputs)]),
    "fmskf_predict": (C.c_int, [_H, C.POINTER(TickInputs)]),
    "fmskf_tick": (C.c_int, [_H, C.POINTER(TickInputs)]),
    "fmskf_tick_many": (C.c_int, [_H, C.POINTER(TickInputs), C.c_uint32, C.c_uint64]),
    "fmskf_get_pose": (C.c_int, [_H, _P, _P, _P, C.c_uint32]),
    "fmskf_get_vel": (C.c_int, [_H, _P, _P, _P, C.c_uint32]),
    "fmskf_get_state": (C.c_int, [_H, _P, _P, C.c_uint32]),
    "fmskf_set_state": (C.c_int, [_H, _P, _P, C.c_uint32]),
    "fmskf_get_prev_sum": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_get_imu": (C.c_int, [_H, _P, _P, C.c_uint32]),
    "fmskf_get_imu_regs": (C.c_int, [_H, _P, _P, C.c_uint32]),
    "fmskf_get_motors": (C.c_int, [_H, _P, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_get_motor_status": (C.c_int, [_H, _P, _P, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_get_state_lo": (C.c_int, [_H, _P, C.POINTER(C.c_uint32), C.c_uint32]),
    "fmskf_set_state_lo": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_get_counters": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_ensemble_record_len": (C.c_int, [_H, C.POINTER(C.c_uint32)]),
    "fmskf_ensemble_partial": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_ensemble_combine": (C.c_int, [C.c_uint32, _P, C.c_uint32, _P, _P]),
    "fmskf_tick_ensemble": (C.c_int, [_H, C.POINTER(TickInputs), _P, C.c_uint32]),
    "fmskf_graph_begin": (C.c_int, [_H]),
    "fmskf_graph_end": (C.c_int, [_H]),
    "fmskf_graph_launch": (C.c_int, [_H, C.c_uint32]),
    "fmskf_comm_unique_id": (C.c_int, [_P]),
    "fmskf_comm_init": (C.c_int, [_H, _P, C.c_int, C.c_int]),
    "fmskf_comm_info": (C.c_int, [_H, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "fmskf_rccl_library": (C.c_char_p, []),
    "fmskf_ensemble_stats": (C.c_int, [_H, _P, _P]),
    "fmskf_tick_ensemble_begin": (C.c_int, [_H, C.POINTER(TickInputs)]),
    "fmskf_ensemble_begin": (C.c_int, [_H]),
    "fmskf_ensemble_end": (C.c_int, [_H, _P, _P]),
    "fmskf_ensemble_end_count": (C.c_int, [_H, _P, _P, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
    "fmskf_ensemble_exchange_ms": (C.c_int, [_H, C.POINTER(C.c_float)]),
    "fmskf_ctrl_params_init": (C.c_int, [C.POINTER(CtrlParams)]),
    "fmskf_set_ctrl_params": (C.c_int, [_H, C.POINTER(CtrlParams)]),
    "fmskf_set_power": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_set_target_vel": (C.c_int, [_H, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_control": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_can_tx": (C.c_int, [_H, _P, C.c_uint32]),
    "fmskf_isr_tick": (C.c_int, [_H, _P, _P, C.c_uint32]),
    "fmskf_isr_tick_can": (C.c_int, [_H, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_save_state": (C.c_int, [_H, C.c_char_p]),
    "fmskf_load_state": (C.c_int, [_H, C.c_char_p]),
    "fmskf_get_ctrl": (C.c_int, [_H, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_export_vehicle_info": (C.c_int, [_H, _P, _P, _P, _P, C.c_uint32]),
    "fmskf_eval_trig": (C.c_int, [_H, _P, _P, _P, C.c_uint64, C.c_uint32]),
    "fmskf_set_timing": (C.c_int, [_H, C.c_int]),
    "fmskf_last_kernel_ms": (C.c_int, [_H, C.POINTER(C.c_float)]),
    "fmskf_kernel_time_total": (C.c_int, [_H, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
}

_lib = None


def load():
    """Load libfmskf.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FmskfError(EDEVICE, "load", f"{LIB_PATH} missing: run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code: int, what: str) -> None:
    if code != OK:
        msg = load().fmskf_last_error()
        raise FmskfError(code, what, msg.decode() if msg else "")
