"""Python host mirror of the C ABI: one Engine = one fmskf handle = N robots.

Inputs may be numpy arrays (host memory; copied to the device on the handle's
stream) or torch CUDA tensors (device memory, zero copy).  Outputs are numpy
arrays (host readout synchronises the stream).  Array layouts are the SoA
planes documented in include/fmskf.h.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import (MEM_DEVICE, MEM_HOST, MODEL_EKF9, MODEL_KF6, MODEL_KF12D, MODEL_NAMES,
                   MODEL_RS, TRIG_LIBM, TRIG_TABLE512, Config, CtrlParams, ENOTSUP, FmskfError,
                   TickInputs, check, load)

# fmskf_vehicle_info (include/fmskf.h): the VehicleInfo message layout, 84 bytes
VEHICLE_INFO_DTYPE = np.dtype([("pos_x", "<i4"), ("pos_y", "<i4"), ("pos_theta", "<f4"),
                               ("vel_x", "<i4"), ("vel_y", "<i4"), ("vel_theta", "<f4"),
                               ("imu_fault", "u1"), ("pad_", "u1", 3), ("imu_q", "<f4", 4),
                               ("imu_g", "<f4", 3), ("imu_a", "<f4", 3), ("floor", "u1", 8),
                               ("cam_pitch", "<f4"), ("fault", "<u4")])

# fmskf_kf6_record (include/fmskf.h): one robot's KF6 tick record, 16 bytes
KF6_RECORD_DTYPE = np.dtype([("yaw_deg", "<f4"), ("gyro_z_dps", "<f4"), ("rpm", "<i2", 4)])

_DTYPES = {
    "yaw_deg": np.float32, "gyro_z_dps": np.float32, "rpm": np.int16, "angle_sum": np.int64,
    "raw": np.int16, "z": np.float64, "valid": np.uint8, "kf6_rec": np.int32,
}


# elements per instance-tick of each input (fmskf_tick_inputs, include/fmskf.h)
_PER_TICK = {"yaw_deg": 1, "gyro_z_dps": 1, "rpm": 4, "angle_sum": 4, "raw": 8, "z": 8, "valid": 1,
             "kf6_rec": 4}


def kf6_records(yaw_deg, gyro_z_dps, rpm):
    """Pack KF6 inputs ([..., N] yaw and gyro, [..., N, 4] rpm; numpy or torch) into
    fmskf_kf6_record's: numpy -> [..., N] KF6_RECORD_DTYPE, torch -> [..., N, 4] int32."""
    if _is_torch(yaw_deg):
        import torch
        rec = torch.empty(tuple(yaw_deg.shape) + (4,), dtype=torch.int32, device=yaw_deg.device)
        rec[..., 0] = yaw_deg.view(torch.int32)
        rec[..., 1] = gyro_z_dps.view(torch.int32)
        rec[..., 2:] = rpm.contiguous().view(torch.int32)
        return rec
    rec = np.empty(np.shape(yaw_deg), KF6_RECORD_DTYPE)
    rec["yaw_deg"] = yaw_deg
    rec["gyro_z_dps"] = gyro_z_dps
    rec["rpm"] = rpm
    return rec


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


class _Args:
    """Collects pointers of one call; all arrays must live in the same memory space."""

    def __init__(self):
        self.mem = None
        self.keep = []

    def ptr(self, a, dtype=None):
        if a is None:
            return None
        if _is_torch(a):
            if not a.is_cuda:
                a = a.numpy()
            else:
                if not a.is_contiguous():
                    raise ValueError("torch inputs must be contiguous")
                self._set(MEM_DEVICE)
                self.keep.append(a)
                return C.c_void_p(a.data_ptr())
        arr = np.ascontiguousarray(a, dtype=dtype) if dtype is not None else np.ascontiguousarray(a)
        self._set(MEM_HOST)
        self.keep.append(arr)
        return arr.ctypes.data_as(C.c_void_p)

    def _set(self, mem):
        if self.mem is None:
            self.mem = mem
        elif self.mem != mem:
            raise ValueError("mixing host and device arrays in one call")


class Engine:
    """Batched IMU + mecanum-odometry estimator over N robots on one GPU."""

    def __init__(self, model="kf6", n=1, device=0, trig=TRIG_TABLE512, dt=None, q=None, r=None,
                 p0=None, motor_dir=None, imu_read_reg=None, flags=0):
        L = load()
        self.model = MODEL_NAMES[model] if isinstance(model, str) else int(model)
        self.n = int(n)
        cfg = Config()
        check(L.fmskf_config_init(C.byref(cfg), self.model, self.n), "config_init")
        cfg.device = int(device)
        cfg.trig = int(trig)
        if dt is not None:
            cfg.dt = float(dt)
        for name, val in (("q", q), ("r", r), ("p0", p0)):
            if val is not None:
                dst = getattr(cfg, name)
                v = np.asarray(val, np.float64).ravel()
                for k in range(len(dst)):
                    dst[k] = float(v[k]) if k < v.size else 0.0
        if motor_dir is not None:
            for k in range(4):
                cfg.motor_dir[k] = int(motor_dir[k])
        if imu_read_reg is not None:
            cfg.imu_read_reg = int(imu_read_reg)
        cfg.flags = int(flags)  # FMSKF_CFG_* (CFG_COMP_POS: KF6 compensated positions)
        self.cfg = cfg
        h = C.c_void_p()
        check(L.fmskf_create(C.byref(cfg), C.byref(h)), "create")
        self.h = h
        nx, m, eb = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(L.fmskf_model_dims(self.model, C.byref(nx), C.byref(m), C.byref(eb)), "model_dims")
        self.nx, self.m, self.elem = nx.value, m.value, eb.value
        self.np_ = self.nx * (self.nx + 1) // 2
        self.dtype = np.float64 if self.elem == 8 else np.float32

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "h", None):
            load().fmskf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def reset(self):
        check(load().fmskf_reset(self.h), "reset")

    def sync(self):
        check(load().fmskf_sync(self.h), "sync")

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream, a raw hipStream_t (int) or None (default stream)."""
        if stream is not None and hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        check(load().fmskf_set_stream(self.h, C.c_void_p(stream) if stream else None), "set_stream")

    def set_timing(self, enable=True):
        check(load().fmskf_set_timing(self.h, int(enable)), "set_timing")

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        check(load().fmskf_last_kernel_ms(self.h, C.byref(ms)), "last_kernel_ms")
        return ms.value

    def kernel_time_total(self):
        """(sum of per-launch kernel times in ms, number of launches) since set_timing."""
        tot, cnt = C.c_double(), C.c_uint32()
        check(load().fmskf_kernel_time_total(self.h, C.byref(tot), C.byref(cnt)),
              "kernel_time_total")
        return tot.value, cnt.value

    # ------------------------------------------------------------------ ingest
    def ingest_wt901(self, data, lens, latch_qinit=False):
        """data: [N, stride] uint8 (one poll's UART bytes per robot), lens: [N] uint32."""
        a = _Args()
        stride = int(data.shape[1]) if hasattr(data, "shape") else 0
        pb = a.ptr(data, np.uint8)
        pl = a.ptr(lens, np.uint32)
        check(load().fmskf_ingest_wt901(self.h, pb, stride, pl, int(latch_qinit), a.mem),
              "ingest_wt901")

    def ingest_can(self, frames, stamps, present=None):
        """frames: [N, 4, 8] uint8, stamps: [N, 4] int16, present: [N] uint8 bitmask."""
        a = _Args()
        pf = a.ptr(frames, np.uint8)
        ps = a.ptr(stamps, np.int16)
        pp = a.ptr(present, np.uint8)
        check(load().fmskf_ingest_can(self.h, pf, ps, pp, a.mem), "ingest_can")

    # ------------------------------------------------------------------ ticks
    def _inputs(self, kw, n_ticks=1, stride=None):
        a = _Args()
        ti = TickInputs()
        unknown = set(kw) - set(_PER_TICK)
        if unknown:
            raise TypeError(f"unknown tick inputs: {sorted(unknown)}")
        stride = self.n if stride is None else stride
        for name in ("yaw_deg", "gyro_z_dps", "rpm", "angle_sum", "raw", "z", "valid", "kf6_rec"):
            v = kw.get(name)
            if name == "kf6_rec" and isinstance(v, np.ndarray) and v.dtype.names:
                v = np.ascontiguousarray(v).view(np.int32)
            if v is not None:
                # the C ABI takes bare pointers: check extents here, before the kernel reads
                need = ((int(n_ticks) - 1) * int(stride) + self.n) * _PER_TICK[name]
                nd = v.dim() if _is_torch(v) else np.ndim(v)
                if name == "angle_sum" and n_ticks == 1 and nd == 2 and v.shape[0] == 4 \
                        and v.shape[1] > self.n:
                    ti.angle_sum_pitch = int(v.shape[1])  # padded [4][pitch] planes
                    need = 3 * int(v.shape[1]) + self.n
                have = v.numel() if _is_torch(v) else np.size(v)
                if have < need:
                    raise ValueError(f"{name}: {have} elements, {n_ticks} tick(s) need {need}")
                if _is_torch(v) and v.is_cuda and str(v.dtype) != "torch." + np.dtype(_DTYPES[name]).name:
                    raise TypeError(f"{name}: dtype {v.dtype}, expected {np.dtype(_DTYPES[name]).name}")
            p = a.ptr(v, _DTYPES[name])
            setattr(ti, name, p.value if p is not None else None)
        ti.mem = MEM_HOST if a.mem is None else a.mem
        return ti, a

    def correct(self, **kw):
        ti, _keep = self._inputs(kw)
        check(load().fmskf_correct(self.h, C.byref(ti)), "correct")

    def predict(self, **kw):
        ti, _keep = self._inputs(kw)
        check(load().fmskf_predict(self.h, C.byref(ti)), "predict")

    def tick(self, **kw):
        ti, _keep = self._inputs(kw)
        check(load().fmskf_tick(self.h, C.byref(ti)), "tick")

    def prepare(self, **kw):
        """Pre-built fmskf_tick_inputs for a hot loop: returns an opaque object to pass to
        tick_prepared() (keeps the arrays alive)."""
        ti, keep = self._inputs(kw)
        return (ti, keep, C.byref(ti))

    def tick_prepared(self, prepared, _tick=None):
        rc = (_tick or load().fmskf_tick)(self.h, prepared[2])
        if rc:
            check(rc, "tick")

    def tick_many(self, n_ticks, tick_stride=None, **kw):
        stride = self.n if tick_stride is None else int(tick_stride)
        ti, _keep = self._inputs(kw, n_ticks, stride)
        check(load().fmskf_tick_many(self.h, C.byref(ti), int(n_ticks), stride), "tick_many")

    # ------------------------------------------------------------------ readout
    def get_state(self):
        x = np.empty((self.nx, self.n), self.dtype)
        P = np.empty((self.np_, self.n), self.dtype) if self.m else None
        check(load().fmskf_get_state(self.h, x.ctypes.data_as(C.c_void_p),
                                     P.ctypes.data_as(C.c_void_p) if P is not None else None,
                                     MEM_HOST), "get_state")
        return x, P

    def set_state(self, x, P=None):
        a = _Args()
        px = a.ptr(x, self.dtype)
        pP = a.ptr(P, self.dtype) if P is not None else None
        check(load().fmskf_set_state(self.h, px, pP, a.mem), "set_state")

    def get_state_lo(self):
        """the hidden low-part rows [rows][N] float32 (EKF9: the heading; KF6 with CFG_COMP_POS:
        px, py, P00, P10, P11), or None when the model keeps none"""
        rows = C.c_uint32()
        check(load().fmskf_get_state_lo(self.h, None, C.byref(rows), MEM_HOST), "get_state_lo")
        if rows.value == 0:
            return None
        lo = np.empty((rows.value, self.n), np.float32)
        check(load().fmskf_get_state_lo(self.h, lo.ctypes.data_as(C.c_void_p), C.byref(rows), MEM_HOST),
              "get_state_lo")
        return lo

    def set_state_lo(self, lo):
        """restore the hidden low-part rows: `lo` must be [rows][N] float32 (host or device),
        rows as get_state_lo returns them"""
        if lo is None:
            raise ValueError("set_state_lo: lo is None")
        rows = C.c_uint32()
        check(load().fmskf_get_state_lo(self.h, None, C.byref(rows), MEM_HOST), "get_state_lo")
        if rows.value == 0:
            raise FmskfError(ENOTSUP, "set_state_lo", "this model keeps no low-part rows")
        want = (rows.value, self.n)
        if tuple(lo.shape) != want:
            raise ValueError(f"set_state_lo: shape {tuple(lo.shape)}, want {want}")
        if _is_torch(lo):
            import torch
            if lo.dtype != torch.float32:
                raise ValueError(f"set_state_lo: dtype {lo.dtype}, want float32")
        elif np.asarray(lo).dtype != np.float32:
            raise ValueError(f"set_state_lo: dtype {np.asarray(lo).dtype}, want float32")
        a = _Args()
        check(load().fmskf_set_state_lo(self.h, a.ptr(lo, np.float32), a.mem), "set_state_lo")

    def save_state(self, path):
        """fmskf_save_state: checkpoint every per-robot array of the handle to `path`"""
        check(load().fmskf_save_state(self.h, str(path).encode()), "save_state")

    def load_state(self, path):
        """fmskf_load_state: resume from a checkpoint of a handle of the same model and N"""
        check(load().fmskf_load_state(self.h, str(path).encode()), "load_state")

    def get_pose(self):
        out = np.empty((3, self.n), np.float32)
        p = [out[k].ctypes.data_as(C.c_void_p) for k in range(3)]
        check(load().fmskf_get_pose(self.h, *p, MEM_HOST), "get_pose")
        return out

    def get_vel(self):
        out = np.empty((3, self.n), np.float32)
        p = [out[k].ctypes.data_as(C.c_void_p) for k in range(3)]
        check(load().fmskf_get_vel(self.h, *p, MEM_HOST), "get_vel")
        return out

    def get_prev_sum(self):
        out = np.empty((4, self.n), np.int64)
        check(load().fmskf_get_prev_sum(self.h, out.ctypes.data_as(C.c_void_p), MEM_HOST),
              "get_prev_sum")
        return out

    def get_imu(self):
        data = np.empty((16, self.n), np.float32)
        err = np.empty(self.n, np.uint8)
        check(load().fmskf_get_imu(self.h, data.ctypes.data_as(C.c_void_p),
                                   err.ctypes.data_as(C.c_void_p), MEM_HOST), "get_imu")
        return data, err

    def get_imu_regs(self):
        regs = np.empty((0x90, self.n), np.int16)
        pend = np.empty(self.n, np.uint8)
        check(load().fmskf_get_imu_regs(self.h, regs.ctypes.data_as(C.c_void_p),
                                        pend.ctypes.data_as(C.c_void_p), MEM_HOST), "get_imu_regs")
        return regs, pend

    def get_motors(self):
        ang = np.empty((self.n, 4), np.int16)
        rpm = np.empty((self.n, 4), np.int16)
        cur = np.empty((self.n, 4), np.int16)
        s = np.empty((4, self.n), np.int64)
        spd = np.empty((4, self.n), np.float32)
        check(load().fmskf_get_motors(self.h, *(a.ctypes.data_as(C.c_void_p)
                                                for a in (ang, rpm, cur, s, spd)), MEM_HOST),
              "get_motors")
        return dict(angle=ang, rpm=rpm, curr=cur, angle_sum=s, speed_radps=spd)

    def get_motor_status(self):
        """MOTOR_IF_M2006::get_status_latest of every wheel: [N][4] each of s16_microsec_id,
        s16_rawAngle, s16_rawSpeedRpm, s16_rawCurr, flt_dltOutAngle_rad, flt_SpeedRadPS"""
        out = dict(microsec_id=np.empty((self.n, 4), np.int16), angle=np.empty((self.n, 4), np.int16),
                   rpm=np.empty((self.n, 4), np.int16), curr=np.empty((self.n, 4), np.int16),
                   dlt_out_angle_rad=np.empty((self.n, 4), np.float32),
                   speed_radps=np.empty((self.n, 4), np.float32))
        check(load().fmskf_get_motor_status(self.h, *(a.ctypes.data_as(C.c_void_p) for a in out.values()),
                                            MEM_HOST), "get_motor_status")
        return out

    # ------------------------------------------------------------------ HIP graph
    def graph_begin(self):
        check(load().fmskf_graph_begin(self.h), "graph_begin")

    def graph_end(self):
        check(load().fmskf_graph_end(self.h), "graph_end")

    def graph_launch(self, times=1):
        check(load().fmskf_graph_launch(self.h, int(times)), "graph_launch")

    # ------------------------------------------------------------------ native RCCL path
    def comm_init(self, unique_id: bytes, rank: int, world: int):
        """fmskf_comm_init: an RCCL communicator owned by this handle (one process per GPU)"""
        b = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        check(load().fmskf_comm_init(self.h, b, int(rank), int(world)), "comm_init")

    def comm_info(self):
        """(world, rank) of the handle's communicator as RCCL reports them (ncclCommCount,
        ncclCommUserRank)"""
        w, r = C.c_int(), C.c_int()
        check(load().fmskf_comm_info(self.h, C.byref(w), C.byref(r)), "comm_info")
        return w.value, r.value

    def ensemble_stats(self):
        """(mean [n], cov packed [n(n+1)/2]) over all ranks of the communicator (or this
        handle alone): device record, ncclAllGather, rank-order fold"""
        nx = self.nx
        mean = np.empty(nx, np.float64)
        cov = np.empty(nx * (nx + 1) // 2, np.float64)
        check(load().fmskf_ensemble_stats(self.h, mean.ctypes.data_as(C.c_void_p),
                                          cov.ctypes.data_as(C.c_void_p)), "ensemble_stats")
        return mean, cov

    def tick_ensemble_begin(self, prepared=None, **kw):
        """fmskf_tick_ensemble_begin: one tick whose kernel also writes this rank's ensemble
        record; fold + all-gather + copy-out run on the handle's side stream (no host wait).
        `prepared` (from prepare()) or tick inputs as keywords."""
        if prepared is not None:
            ref = prepared[2]
        else:
            ti, _keep = self._inputs(kw)
            ref = C.byref(ti)
        check(load().fmskf_tick_ensemble_begin(self.h, ref), "tick_ensemble_begin")

    def ensemble_begin(self):
        """fmskf_ensemble_begin: the stand-alone record of the current state, asynchronously"""
        check(load().fmskf_ensemble_begin(self.h), "ensemble_begin")

    def ensemble_end(self):
        """fmskf_ensemble_end: (mean, cov packed) of the oldest pending begin"""
        nx = self.nx
        mean = np.empty(nx, np.float64)
        cov = np.empty(nx * (nx + 1) // 2, np.float64)
        check(load().fmskf_ensemble_end(self.h, mean.ctypes.data_as(C.c_void_p),
                                        cov.ctypes.data_as(C.c_void_p)), "ensemble_end")
        return mean, cov

    def ensemble_end_count(self):
        """fmskf_ensemble_end_count: (mean, cov packed, robots the gathered records count,
        records folded) of the oldest pending begin"""
        nx = self.nx
        mean = np.empty(nx, np.float64)
        cov = np.empty(nx * (nx + 1) // 2, np.float64)
        cnt, nrec = C.c_double(), C.c_uint32()
        check(load().fmskf_ensemble_end_count(self.h, mean.ctypes.data_as(C.c_void_p),
                                              cov.ctypes.data_as(C.c_void_p), C.byref(cnt), C.byref(nrec)),
              "ensemble_end_count")
        return mean, cov, cnt.value, nrec.value

    def ensemble_exchange_ms(self) -> float:
        """fmskf_ensemble_exchange_ms: the side stream's all-gather + copy-out time of the result
        the last ensemble_end collected (ms), -1 when it needed no exchange"""
        ms = C.c_float()
        check(load().fmskf_ensemble_exchange_ms(self.h, C.byref(ms)), "ensemble_exchange_ms")
        return ms.value

    # ------------------------------------------------------------------ control step
    def set_ctrl_params(self, **kw):
        """FF_PI_D / interpolator / current-limit parameters (fmskf_ctrl_params); unspecified
        fields keep the firmware defaults (VD_task_main.cpp:86-97,157-160)."""
        p = CtrlParams()
        check(load().fmskf_ctrl_params_init(C.byref(p)), "ctrl_params_init")
        for k, v in kw.items():
            setattr(p, k, v)
        check(load().fmskf_set_ctrl_params(self.h, C.byref(p)), "set_ctrl_params")

    def set_power(self, on=None):
        a = _Args()
        p = a.ptr(None if on is None else np.broadcast_to(np.asarray(on, np.uint8), (self.n,)),
                  np.uint8)
        check(load().fmskf_set_power(self.h, p, MEM_HOST if a.mem is None else a.mem), "set_power")

    def set_target_vel(self, vel, acl, jrk, mask=None):
        """vel/acl/jrk [3][N] (x mm/s, y mm/s, th rad/s)"""
        a = _Args()
        ps = [a.ptr(v, np.float32) for v in (vel, acl, jrk)]
        for name, v in zip(("vel", "acl", "jrk"), (vel, acl, jrk)):
            have = v.numel() if _is_torch(v) else np.size(v)
            if have < 3 * self.n:
                raise ValueError(f"{name}: {have} elements, need 3*N = {3 * self.n}")
        pm = a.ptr(mask, np.uint8)
        check(load().fmskf_set_target_vel(self.h, *ps, pm, MEM_HOST if a.mem is None else a.mem),
              "set_target_vel")

    def control(self, rpm=None):
        a = _Args()
        if rpm is not None:
            have = rpm.numel() if _is_torch(rpm) else np.size(rpm)
            if have < 4 * self.n:
                raise ValueError(f"rpm: {have} elements, need 4*N = {4 * self.n}")
        p = a.ptr(rpm, np.int16)
        check(load().fmskf_control(self.h, p, MEM_HOST if a.mem is None else a.mem), "control")

    def can_tx(self, out=None):
        """CAN_CTRL::tx_routine payloads [N][8] (host numpy, or into a device tensor `out`)"""
        if out is not None and _is_torch(out) and out.is_cuda:
            check(load().fmskf_can_tx(self.h, C.c_void_p(out.data_ptr()), MEM_DEVICE), "can_tx")
            return out
        f = np.empty((self.n, 8), np.uint8)
        check(load().fmskf_can_tx(self.h, f.ctypes.data_as(C.c_void_p), MEM_HOST), "can_tx")
        return f

    def isr_tick(self, frames=True, out=None, **kw):
        """VDT::can_tx_routine_intr in one call (fmskf_isr_tick): correct, update (estimator +
        control), tx_routine.  Inputs as tick(); returns the [N][8] frames (host numpy, or the
        device tensor `out`), or None with frames=False."""
        ti, _keep = self._inputs(kw)
        if out is not None and _is_torch(out) and out.is_cuda:
            check(load().fmskf_isr_tick(self.h, C.byref(ti), C.c_void_p(out.data_ptr()), MEM_DEVICE),
                  "isr_tick")
            return out
        if not frames:
            check(load().fmskf_isr_tick(self.h, C.byref(ti), None, MEM_HOST), "isr_tick")
            return None
        f = np.empty((self.n, 8), np.uint8)
        check(load().fmskf_isr_tick(self.h, C.byref(ti), f.ctypes.data_as(C.c_void_p), MEM_HOST),
              "isr_tick")
        return f

    def isr_tick_can(self, can_frames, can_stamps, frames=True, out=None, **kw):
        """The tick's CAN RX and the ISR in one call (fmskf_isr_tick_can): ingest_can(can_frames,
        can_stamps) then isr_tick(**kw), one kernel for RS, KF6 and EKF9.  can_frames [N, 4, 8] uint8,
        can_stamps [N, 4] int16, both host arrays or both device tensors; the [N][8] TX frames
        come back the same way (numpy, or the device tensor `out`), None with frames=False."""
        a = _Args()
        pf = a.ptr(can_frames, np.uint8)
        ps = a.ptr(can_stamps, np.int16)
        for name, v, per in (("can_frames", can_frames, 32), ("can_stamps", can_stamps, 4)):
            have = v.numel() if _is_torch(v) else np.size(v)
            if have < per * self.n:
                raise ValueError(f"{name}: {have} elements, need {per}*N = {per * self.n}")
        mem = MEM_HOST if a.mem is None else a.mem
        ti, _keep = self._inputs(kw)
        if not frames:
            check(load().fmskf_isr_tick_can(self.h, pf, ps, C.byref(ti), None, mem), "isr_tick_can")
            return None
        if mem == MEM_DEVICE:
            import torch
            if out is None:
                out = torch.empty((self.n, 8), dtype=torch.uint8, device=can_frames.device)
            if not (_is_torch(out) and out.is_cuda):
                raise TypeError("device CAN frames need a device `out`")
            check(load().fmskf_isr_tick_can(self.h, pf, ps, C.byref(ti), C.c_void_p(out.data_ptr()), mem),
                  "isr_tick_can")
            return out
        if out is not None:  # one mem flag covers the CAN buffers and the TX frames
            raise TypeError("host CAN frames: the TX frames come back as a numpy array (out=None)")
        f = np.empty((self.n, 8), np.uint8)
        check(load().fmskf_isr_tick_can(self.h, pf, ps, C.byref(ti), f.ctypes.data_as(C.c_void_p), mem),
              "isr_tick_can")
        return f

    def get_ctrl(self):
        vt = np.empty((3, self.n), np.float32)
        cur = np.empty((self.n, 4), np.int16)
        wt = np.empty((4, self.n), np.float32)
        wc = np.empty((4, self.n), np.float32)
        check(load().fmskf_get_ctrl(self.h, *(x.ctypes.data_as(C.c_void_p) for x in (vt, cur, wt, wc)),
                                    MEM_HOST), "get_ctrl")
        return dict(vel_tgt=vt, curr=cur, wheel_tgt=wt, wheel_ctrl=wc)

    def export_vehicle_info(self, floor=None, cam_pitch=None, fault=None):
        """[N] VehicleInfo records (structured numpy array, VEHICLE_INFO_DTYPE)"""
        a = _Args()
        pf = a.ptr(floor, np.uint8)
        pc = a.ptr(cam_pitch, np.float32)
        pu = a.ptr(fault, np.uint32)
        mem = MEM_HOST if a.mem is None else a.mem
        if mem != MEM_HOST:
            raise ValueError("export_vehicle_info: host inputs only from Python")
        out = np.empty(self.n, VEHICLE_INFO_DTYPE)
        check(load().fmskf_export_vehicle_info(self.h, out.ctypes.data_as(C.c_void_p), pf, pc, pu,
                                               MEM_HOST), "export_vehicle_info")
        return out

    def get_counters(self):
        out = (C.c_uint64 * 8)()
        check(load().fmskf_get_counters(self.h, out, 8), "get_counters")
        return list(out)

    # ------------------------------------------------------------------ ensemble
    def ensemble_record_len(self) -> int:
        v = C.c_uint32()
        check(load().fmskf_ensemble_record_len(self.h, C.byref(v)), "ensemble_record_len")
        return v.value

    def ensemble_partial(self, out=None):
        """This rank's {count, mean, M2} record: numpy (host) or into a torch CUDA tensor."""
        if out is not None and _is_torch(out) and out.is_cuda:
            check(load().fmskf_ensemble_partial(self.h, C.c_void_p(out.data_ptr()), MEM_DEVICE),
                  "ensemble_partial")
            return out
        rec = np.empty(self.ensemble_record_len(), np.float64)
        check(load().fmskf_ensemble_partial(self.h, rec.ctypes.data_as(C.c_void_p), MEM_HOST),
              "ensemble_partial")
        return rec

    def tick_ensemble(self, out=None, **kw):
        """fmskf_tick_ensemble: one tick plus this rank's record of the post-tick state"""
        ti, _keep = self._inputs(kw)
        return self._tick_ens(C.byref(ti), out)

    def tick_ensemble_prepared(self, prepared, out=None):
        return self._tick_ens(prepared[2], out)

    def _tick_ens(self, ti_ref, out):
        if out is not None and _is_torch(out) and out.is_cuda:
            check(load().fmskf_tick_ensemble(self.h, ti_ref, C.c_void_p(out.data_ptr()), MEM_DEVICE),
                  "tick_ensemble")
            return out
        rec = np.empty(self.ensemble_record_len(), np.float64)
        check(load().fmskf_tick_ensemble(self.h, ti_ref, rec.ctypes.data_as(C.c_void_p), MEM_HOST),
              "tick_ensemble")
        return rec

    # ------------------------------------------------------------------ diagnostics
    def eval_trig(self, x):
        x = np.ascontiguousarray(x, np.float32)
        s = np.empty_like(x)
        c = np.empty_like(x)
        check(load().fmskf_eval_trig(self.h, x.ctypes.data_as(C.c_void_p),
                                     s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p),
                                     x.size, MEM_HOST), "eval_trig")
        return s, c


def ensemble_combine(n_state: int, records) -> tuple[np.ndarray, np.ndarray]:
    """Fold per-rank records in rank order -> (mean [n], covariance packed [n(n+1)/2])."""
    recs = np.ascontiguousarray(records, np.float64)
    nrec = recs.shape[0] if recs.ndim == 2 else 1
    mean = np.empty(n_state, np.float64)
    cov = np.empty(n_state * (n_state + 1) // 2, np.float64)
    check(load().fmskf_ensemble_combine(n_state, recs.ctypes.data_as(C.c_void_p), nrec,
                                        mean.ctypes.data_as(C.c_void_p),
                                        cov.ctypes.data_as(C.c_void_p)), "ensemble_combine")
    return mean, cov


def shard_span(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Rank `rank`'s contiguous robot range [lo, hi) of `n_total` over `world` ranks, the
    remainder on the first ranks (bench.py's sharding): shards differ by at
    most one robot and rank order is robot order, so the rank-order fold of the records is
    the fold of the unsharded fleet."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError(f"shard_span: n_total {n_total}, world {world}, rank {rank}")
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def rccl_library() -> str:
    """the file libfmskf resolved RCCL from ("" before its first communicator call)"""
    v = load().fmskf_rccl_library()
    return v.decode() if v else ""


def comm_unique_id() -> bytes:
    """fmskf_comm_unique_id (rank 0): 128 bytes to hand to every rank's comm_init"""
    b = (C.c_uint8 * 128)()
    check(load().fmskf_comm_unique_id(b), "comm_unique_id")
    return bytes(b)


def default_config(model="kf6", n=1) -> Config:
    """Model defaults (pure host call, no GPU needed)."""
    cfg = Config()
    m = MODEL_NAMES[model] if isinstance(model, str) else int(model)
    check(load().fmskf_config_init(C.byref(cfg), m, int(n)), "config_init")
    return cfg


__all__ = ["Engine", "ensemble_combine", "default_config", "comm_unique_id", "VEHICLE_INFO_DTYPE", "MODEL_RS", "MODEL_KF6", "MODEL_EKF9",
           "MODEL_KF12D", "TRIG_TABLE512", "TRIG_LIBM", "_lib"]
