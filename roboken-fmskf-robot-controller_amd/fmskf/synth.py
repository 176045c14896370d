"""Synthetic WT901 IMU + C610/M2006 wheel-encoder traffic for N robots.

No datasets exist for this path (the reference ships none), so tests and the
bench drive the engine with trajectories generated here: per robot a commanded
body velocity inside the firmware's limits (|v| <= 400 mm/s planar,
VD_task_main.cpp:26; yaw rate within +-pi rad/s), slowly modulated, integrated
at 1 kHz; the sensors are then quantised exactly as the devices report them:

* WT901 registers: int16, angle/32768*180 deg, gyro/32768*2000 deg/s, acc/32768*16 g
  (imu_if_wt901c.cpp:96-99), frames 0x51/0x52/0x53/0x59 of 11 bytes with the
  8-bit sum (wit_c_sdk.c:77-83,148-161), 44 B per 10 ms (teraterm/wt901ttl_change_config.ttl:4).
* wheels: mecanum inverse kinematics (VD_vehicle_controller.cpp:113-118) x gear 36,
  13-bit encoder angle mod 8192, int16 rpm, reversed BR/FR motors (VD_task_main.cpp:75-78).
"""
from __future__ import annotations

import numpy as np

SEED = 0x464D534B  # "FMSK"

PI_F = np.float32(3.14159265358979)
RPM_TO_RADPS = np.float32(np.float32(2.0 * np.float32(3.1415926)) / np.float32(60.0))
WHEEL_R = 37.5
WHEEL_L = 13.08148
SQRTF2 = 1.41421356
GEAR = 36.0
MOTOR_DIR = np.array([1, 1, -1, -1], np.int64)


def wt901_frame(ftype: int, words) -> bytes:
    """One 11-byte WT901 NORMAL-protocol frame: 0x55, type, 4 little-endian words, sum."""
    w = [int(x) & 0xFFFF for x in words]
    body = bytes([0x55, ftype & 0xFF] + [b for x in w for b in (x & 0xFF, x >> 8)])
    return body + bytes([sum(body) & 0xFF])


def vdir_to_mdir(vx, vy, vth):
    """VEHICLE_CTRL::conv_Vdir_to_Mdir (VD_vehicle_controller.cpp:113-118), float64."""
    k = SQRTF2 * WHEEL_L * 4.0
    return np.stack([(vx - vy - k * vth) / WHEEL_R, (vx + vy - k * vth) / WHEEL_R,
                     (vx - vy + k * vth) / WHEEL_R, (vx + vy + k * vth) / WHEEL_R], axis=-1)


def _i16(x):
    return np.clip(np.rint(x), -32768, 32767).astype(np.int16)


def _robot_params(rng, n):
    """Per-robot commanded motion: body velocity (|v| <= 400 mm/s), yaw rate, initial heading,
    modulation phase"""
    v = rng.uniform(-400.0, 400.0, (2, n))
    nrm = np.maximum(1.0, np.hypot(v[0], v[1]) / 400.0)
    v = v / nrm
    w = rng.uniform(-np.pi, np.pi, n)
    th0 = rng.uniform(-np.pi, np.pi, n)
    ph = rng.uniform(0, 2 * np.pi, n)
    return v, w, th0, ph


def trajectory_chunks(n: int, ticks: int, chunk: int = 1000, seed: int = SEED, dt: float = 1e-3,
                      noise: bool = True):
    """A long trace of n robots generated `chunk` ticks at a time (memory bounded): yields
    (t0, Trajectory of ticks t0 .. t0 + chunk - 1).  The robots' motion continues across chunks;
    each chunk draws its sensor noise from its own seeded stream."""
    params = _robot_params(np.random.default_rng(seed), n)
    carry = None
    for k, t0 in enumerate(range(0, ticks, chunk)):
        tr = Trajectory(n, min(chunk, ticks - t0), dt=dt, noise=noise, t0=t0, params=params,
                        carry=carry, rng=np.random.default_rng([seed, k]))
        carry = (tr.px[-1], tr.py[-1], tr.angle_sum[-1])
        yield t0, tr


class Trajectory:
    """Ground truth + sensor readings of n robots over `ticks` 1 kHz ticks.

    Arrays are tick-major: [T, N] (and [T, N, 4] per wheel)."""

    def __init__(self, n: int, ticks: int, seed: int = SEED, dt: float = 1e-3, noise: bool = True,
                 t0: int = 0, params=None, carry=None, rng=None):
        # t0 / params / carry / rng: one chunk of a longer trace (trajectory_chunks); the
        # defaults give the whole trace at once (the committed fixtures depend on that path)
        rng = np.random.default_rng(seed) if rng is None else rng
        self.n, self.ticks, self.dt = n, ticks, dt
        v, w, th0, ph = _robot_params(rng, n) if params is None else params
        t = (t0 + np.arange(ticks))[:, None] * dt
        mod = 1.0 + 0.3 * np.sin(2 * np.pi * 0.5 * t + ph[None, :])
        self.vbx = v[0][None, :] * mod            # body mm/s
        self.vby = v[1][None, :] * mod
        self.w = np.broadcast_to(w[None, :], (ticks, n)).copy()   # rad/s
        th = th0[None, :] + np.cumsum(self.w * dt, axis=0) - self.w * dt + self.w * (dt * t0)
        self.th = (th + np.pi) % (2 * np.pi) - np.pi              # [-pi, pi)
        c, s = np.cos(self.th), np.sin(self.th)
        self.vx_w = (self.vbx * c - self.vby * s) * 1e-3           # world m/s
        self.vy_w = (self.vbx * s + self.vby * c) * 1e-3
        px0, py0, sum0 = (0.0, 0.0, 0) if carry is None else carry
        self.px = np.cumsum(self.vx_w * dt, axis=0) + px0
        self.py = np.cumsum(self.vy_w * dt, axis=0) + py0
        # wheels: output rad/s -> motor rad/s -> rpm; encoder counts (motor shaft, 8192/rev)
        mdir = vdir_to_mdir(self.vbx, self.vby, self.w)            # [T, N, 4] wheel rad/s
        motor_radps = mdir * GEAR
        nz = (lambda sd, shape: rng.normal(0.0, sd, shape)) if noise else (lambda sd, shape: 0.0)
        self.rpm = _i16(motor_radps / float(RPM_TO_RADPS) + nz(2.0, motor_radps.shape))
        counts = motor_radps * dt * 8192.0 / (2 * np.pi)
        self.angle_sum = np.cumsum(np.rint(counts + nz(2.0, counts.shape)), axis=0).astype(np.int64) + sum0
        # IMU registers (native sensor frame; yaw == heading)
        yaw_deg = np.degrees(self.th) + nz(0.05, self.th.shape)
        self.reg_yaw = _i16(yaw_deg / 180.0 * 32768.0)
        self.reg_gz = _i16(np.degrees(self.w) / 2000.0 * 32768.0 + nz(3.0, self.w.shape))
        acc = rng.normal(0.0, 0.02, (2, ticks, n)) if noise else np.zeros((2, ticks, n))
        self.reg_ax = _i16(acc[0] / 16.0 * 32768.0)
        self.reg_ay = _i16(acc[1] / 16.0 * 32768.0)

    # -- values as IMU_IF::Data publishes them (float32, imu_if_wt901c.cpp:96-121)
    def yaw_deg(self):
        return (self.reg_yaw.astype(np.float32) / np.float32(32768.0) * np.float32(180.0)).astype(np.float32)

    def gyro_z_dps(self):
        g = self.reg_gz.astype(np.float32) / np.float32(32768.0) * np.float32(2000.0)
        return (-g).astype(np.float32)  # published z gyro is sign-flipped (:113)

    def kf6_inputs(self):
        """(yaw_deg [T,N], gyro_z_dps [T,N], rpm [T,N,4])"""
        return self.yaw_deg(), self.gyro_z_dps(), np.ascontiguousarray(self.rpm)

    def ekf9_raw(self):
        """[T, N, 8] int16: Yaw, GZ, AX, AY registers + rpm FL BL BR FR"""
        return np.ascontiguousarray(np.concatenate(
            [self.reg_yaw[..., None], self.reg_gz[..., None], self.reg_ax[..., None],
             self.reg_ay[..., None], self.rpm], axis=-1).astype(np.int16))

    def rs_inputs(self):
        """(yaw_deg [T,N], angle_sum [T,4,N], rpm [T,N,4])"""
        return self.yaw_deg(), np.ascontiguousarray(self.angle_sum.transpose(0, 2, 1)), \
            np.ascontiguousarray(self.rpm)

    def kf12d_z(self, seed: int = SEED + 12):
        """[T, 8, N] float64: theta, omega, vx_w, vy_w, arm tip tx, ty, tz, tvz."""
        rng = np.random.default_rng(seed)
        T, n = self.th.shape
        t = np.arange(T)[:, None] * self.dt
        f = rng.uniform(0.2, 1.0, n)[None, :]
        tip = np.stack([0.30 + 0.05 * np.sin(2 * np.pi * f * t), 0.05 * np.cos(2 * np.pi * f * t),
                        0.20 + 0.10 * np.sin(np.pi * f * t)], axis=1)
        tvz = 0.10 * np.pi * f * np.cos(np.pi * f * t)
        z = np.stack([np.radians(self.yaw_deg().astype(np.float64)), self.w, self.vx_w, self.vy_w,
                      tip[:, 0], tip[:, 1], tip[:, 2], tvz], axis=1)
        return np.ascontiguousarray(z + rng.normal(0, 1e-4, z.shape))

    # -- raw device traffic
    def wt901_poll_bytes(self, tick: int, i: int) -> bytes:
        """The 44 bytes one 10 ms IMU poll drains for robot i at `tick` (acc, gyro, angle, quat)."""
        yaw = int(self.reg_yaw[tick, i])
        half = np.radians(yaw / 32768.0 * 180.0) / 2.0
        q = [int(np.rint(np.cos(half) * 32767)), 0, 0, int(np.rint(np.sin(half) * 32767))]
        return (wt901_frame(0x51, [self.reg_ax[tick, i], self.reg_ay[tick, i], 2048, 2500]) +
                wt901_frame(0x52, [0, 0, self.reg_gz[tick, i], 0]) +
                wt901_frame(0x53, [0, 0, yaw, 0x1234]) +
                wt901_frame(0x59, q))

    def wt901_poll_rows(self, tick: int, stride: int = 48):
        """wt901_poll_bytes for every robot at once: ([N, stride] uint8 rows, [N] uint32 lengths)."""
        n = self.n
        yaw = self.reg_yaw[tick].astype(np.int64)
        half = np.radians(yaw / 32768.0 * 180.0) / 2.0
        z = np.zeros(n, np.int64)
        words = [(0x51, [self.reg_ax[tick].astype(np.int64), self.reg_ay[tick].astype(np.int64), z + 2048, z + 2500]),
                 (0x52, [z, z, self.reg_gz[tick].astype(np.int64), z]),
                 (0x53, [z, z, yaw, z + 0x1234]),
                 (0x59, [np.rint(np.cos(half) * 32767).astype(np.int64), z, z,
                         np.rint(np.sin(half) * 32767).astype(np.int64)])]
        rows = np.zeros((n, stride), np.uint8)
        for f, (ftype, w) in enumerate(words):
            fr = rows[:, 11 * f: 11 * f + 11]
            fr[:, 0] = 0x55
            fr[:, 1] = ftype
            for k, v in enumerate(w):
                u = v & 0xFFFF
                fr[:, 2 + 2 * k] = (u & 0xFF).astype(np.uint8)
                fr[:, 3 + 2 * k] = (u >> 8).astype(np.uint8)
            fr[:, 10] = (fr[:, :10].astype(np.int64).sum(axis=1) & 0xFF).astype(np.uint8)
        return rows, np.full(n, 44, np.uint32)

    def can_frames(self, tick: int):
        """([N,4,8] uint8 C610 payloads, [N,4] int16 stamps) for one 1 ms tick."""
        n = self.n
        internal = self.angle_sum[tick]  # [N,4] cumulative motor counts
        sensor_ang = np.mod(internal * MOTOR_DIR[None, :], 8192).astype(np.int64)
        sensor_rpm = self.rpm[tick].astype(np.int64) * MOTOR_DIR[None, :]
        curr = np.zeros((n, 4), np.int64) + 100
        fr = np.zeros((n, 4, 8), np.uint8)
        for k, v in enumerate((sensor_ang, sensor_rpm, curr)):
            u = np.asarray(v, np.int64) & 0xFFFF
            fr[:, :, 2 * k] = (u >> 8).astype(np.uint8)
            fr[:, :, 2 * k + 1] = (u & 0xFF).astype(np.uint8)
        stamps = np.full((n, 4), ((tick + 1) * 1000 + np.arange(4)[None, :] * 7) & 0x7FFF, np.int16)
        return fr, stamps


def kf6_ring_torch(n: int, ticks: int, seed: int = SEED, device="cuda"):
    """Bench input ring generated directly in HBM (same sensor model as Trajectory,
    vectorised in torch float64 on the GPU; generation is not timed).

    Returns (yaw_deg [T,N] f32, gyro_z_dps [T,N] f32, rpm [T,N,4] i16)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f64 = torch.float64
    v = (torch.rand(2, n, generator=g, device=device, dtype=f64) * 800.0 - 400.0)
    nrm = torch.clamp(torch.hypot(v[0], v[1]) / 400.0, min=1.0)
    v = v / nrm
    w = (torch.rand(n, generator=g, device=device, dtype=f64) * 2 - 1) * np.pi
    th0 = (torch.rand(n, generator=g, device=device, dtype=f64) * 2 - 1) * np.pi
    ph = torch.rand(n, generator=g, device=device, dtype=f64) * 2 * np.pi
    yaw = torch.empty(ticks, n, dtype=torch.float32, device=device)
    gz = torch.empty(ticks, n, dtype=torch.float32, device=device)
    rpm = torch.empty(ticks, n, 4, dtype=torch.int16, device=device)
    k = SQRTF2 * WHEEL_L * 4.0
    for t in range(ticks):
        tt = t * 1e-3
        mod = 1.0 + 0.3 * torch.sin(2 * np.pi * 0.5 * tt + ph)
        vbx, vby = v[0] * mod, v[1] * mod
        th = torch.remainder(th0 + w * tt + np.pi, 2 * np.pi) - np.pi
        ryaw = torch.clamp(torch.round((torch.rad2deg(th) + 0.05 * torch.randn(n, generator=g, device=device, dtype=f64)) / 180.0 * 32768.0), -32768, 32767)
        yaw[t] = (ryaw.float() / 32768.0 * 180.0)
        rgz = torch.clamp(torch.round(torch.rad2deg(w) / 2000.0 * 32768.0 + 3.0 * torch.randn(n, generator=g, device=device, dtype=f64)), -32768, 32767)
        gz[t] = -(rgz.float() / 32768.0 * 2000.0)
        m = torch.stack([vbx - vby - k * w, vbx + vby - k * w, vbx - vby + k * w, vbx + vby + k * w], -1) / WHEEL_R
        r = m * GEAR / float(RPM_TO_RADPS) + 2.0 * torch.randn(n, 4, generator=g, device=device, dtype=f64)
        rpm[t] = torch.clamp(torch.round(r), -32768, 32767).to(torch.int16)
    return yaw.contiguous(), gz.contiguous(), rpm.contiguous()
