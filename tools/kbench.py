"""Kernel micro-benchmark: time one model's fused tick kernel at a given N with HIP
events (tick-only loop, no ensemble), for A/B sweeps of kernel variants.

  FMSKF_KF6_VARIANT=3 python tools/kbench.py --model kf6 --n 1048576
prints one JSON line: {"model", "n", "variant", "ms_per_tick", "algo_GBps", ...}
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "roboken-fmskf-robot-controller_amd")]

# SURVEY.md 8(d) algorithmic bytes (RS: theta is overwritten, never read); --comp: KF6 272
BYTES = {"kf6": 232, "rs": 140, "ekf9": 448, "kf12d": 1504}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="kf6")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=300)
    ap.add_argument("--ring", type=int, default=16)
    ap.add_argument("--many", type=int, default=0, help="ticks per launch (tick_many)")
    ap.add_argument("--packed", action="store_true", help="KF6: fmskf_kf6_record inputs")
    ap.add_argument("--pad", type=int, default=0, help="input plane pitch padding (elements)")
    ap.add_argument("--can-desync", action="store_true",
                    help="--op can: one masked tick before timing (robots' ring heads out of step)")
    ap.add_argument("--op", choices=["tick", "predict", "correct", "ensemble", "tick_ensemble", "ens_async", "control", "can_tx", "wt901", "can", "pipeline", "pipeline_graph", "isr", "isr_graph", "isr_can", "can_isr", "isr_can_graph", "can_isr_graph"], default="tick")
    ap.add_argument("--trig", choices=["table512", "libm"], default="table512")
    ap.add_argument("--host", choices=["", "pageable", "pinned"], default="",
                    help="KF6 tick with host-resident inputs staged over PCIe per call")
    ap.add_argument("--valid", action="store_true", help="a validity mask per tick (9 in 10 robots valid)")
    ap.add_argument("--comp", action="store_true", help="KF6 with FMSKF_CFG_COMP_POS (compensated positions)")
    ap.add_argument("--comm", action="store_true",
                    help="--op ens_async: a world-1 RCCL communicator on the handle (fmskf_comm_init)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import fmskf
    from fmskf.synth import kf6_ring_torch

    dev = torch.device("cuda", 0)
    n, R = args.n, max(args.ring, args.many)  # tick_many reads `many` ticks of the ring
    e = fmskf.Engine(args.model, n, trig=fmskf.TRIG_LIBM if args.trig == "libm" else fmskf.TRIG_TABLE512,
                     flags=fmskf.CFG_COMP_POS if args.comp else 0)
    if args.comp:
        BYTES["kf6"], BYTES["ekf9"] = 272, 488
    st = torch.cuda.current_stream()
    e.set_stream(st)
    yaw, gz, rpm = kf6_ring_torch(n, R, device=dev)
    if args.pad:  # input planes at a padded per-tick pitch, each array's base staggered
        def padded(t, k):
            T = t.shape[0]
            w = (n + args.pad) * t[0].numel() // n
            buf = torch.empty(T * w + k * 4096, dtype=t.dtype, device=dev)
            v = buf[k * 4096:].view(T, w)[:, : t[0].numel()]
            v.copy_(t.reshape(T, -1))
            return v.view(t.shape)
        yaw, gz, rpm = padded(yaw, 1), padded(gz, 2), padded(rpm, 3)
    if args.model == "kf6" and args.packed:  # 16-byte fmskf_kf6_record inputs
        rec = fmskf.kf6_records(yaw, gz, rpm)
        preps = [e.prepare(kf6_rec=rec[r]) for r in range(R)]
        many = dict(kf6_rec=rec)
    elif args.model == "kf6":
        preps = [e.prepare(yaw_deg=yaw[r], gyro_z_dps=gz[r], rpm=rpm[r]) for r in range(R)]
        many = dict(yaw_deg=yaw, gyro_z_dps=gz, rpm=rpm)
    elif args.model == "rs":
        # --pad: the [4][N] encoder-sum planes at a padded pitch (fmskf_tick_inputs.angle_sum_pitch)
        sums = torch.cumsum(torch.randint(-20, 20, (R, 4, n + args.pad), device=dev, dtype=torch.int64), 0)
        preps = [e.prepare(yaw_deg=yaw[r], angle_sum=sums[r], rpm=rpm[r]) for r in range(R)]
        many = dict(yaw_deg=yaw, angle_sum=sums, rpm=rpm)
    elif args.model == "ekf9":
        raw = torch.cat([torch.round(yaw / 180.0 * 32768).to(torch.int16)[..., None],
                         torch.round(-gz / 2000.0 * 32768).to(torch.int16)[..., None],
                         torch.zeros(R, n, 2, dtype=torch.int16, device=dev), rpm], -1).contiguous()
        preps = [e.prepare(raw=raw[r]) for r in range(R)]
        many = dict(raw=raw)
    else:
        z = torch.zeros(R, 8, n, dtype=torch.float64, device=dev)
        z[:, 0] = torch.deg2rad(yaw.double())
        z[:, 1] = -torch.deg2rad(gz.double())
        preps = [e.prepare(z=z[r]) for r in range(R)]
        many = dict(z=z)
    if args.valid:  # every tick's prepared inputs carry a [N] u8 validity mask
        vm = (torch.rand(R, n, device=dev) < 0.9).to(torch.uint8)
        kws = [dict(kf6_rec=rec[r]) if args.model == "kf6" and args.packed else
               dict(yaw_deg=yaw[r], gyro_z_dps=gz[r], rpm=rpm[r]) if args.model == "kf6" else
               dict(raw=raw[r]) if args.model == "ekf9" else dict(z=z[r]) for r in range(R)]
        preps = [e.prepare(valid=vm[r], **kws[r]) for r in range(R)]
    if args.host:
        return bench_host(args, e, n, yaw, gz, rpm)
    if args.op in ("pipeline", "pipeline_graph", "isr", "isr_graph", "isr_can", "can_isr", "isr_can_graph",
                   "can_isr_graph"):
        return bench_pipeline(args, e, n, yaw, gz, rpm, dev, st)
    if args.op in ("control", "can_tx", "wt901", "can"):
        return bench_io(args, e, n, R, dev, rpm, st)
    tick = getattr(fmskf.load(), "fmskf_" + ("tick" if args.op in ("ensemble", "tick_ensemble", "ens_async") else args.op))
    for k in range(20):
        e.tick_prepared(preps[k % R], tick)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if args.op == "tick_ensemble":  # fmskf_tick_ensemble: the tick with its record (+ fold)
        rec = torch.empty(e.ensemble_record_len(), dtype=torch.float64, device=dev)
        e.tick_ensemble_prepared(preps[0], rec)
        torch.cuda.synchronize()
        ev0.record(st)
        for k in range(args.ticks):
            e.tick_ensemble_prepared(preps[k % R], rec)
        ev1.record(st)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / args.ticks
        print(json.dumps({"model": args.model, "n": n, "op": "tick_ensemble", "ms_per_tick": ms,
                          "steps_per_s": n / (ms * 1e-3)}), flush=True)
        return
    if args.op == "ens_async":  # a record every tick: plain ticks, sync fused record, async begin/end
        import time
        rec = torch.empty(e.ensemble_record_len(), dtype=torch.float64, device=dev)
        res = {"model": args.model, "n": n, "op": "ens_async"}

        evs = [torch.cuda.Event() for _ in range(4)]  # hipEventDisableTiming, system-scope release
        import ctypes  # the library's kind of event: hipEventDisableTiming | hipEventDisableSystemFence
        hip = ctypes.CDLL("libamdhip64.so")
        nf = [ctypes.c_void_p() for _ in range(4)]
        for v in nf:
            assert hip.hipEventCreateWithFlags(ctypes.byref(v), ctypes.c_uint(0x2 | 0x20000000)) == 0
        sp = ctypes.c_void_p(st.cuda_stream)

        def loop(kind, ticks):
            pend = 0
            for k in range(ticks):
                if kind == "tick":
                    e.tick_prepared(preps[k % R], tick)
                elif kind == "tick_ev":  # the cost of a system-scope event behind every tick
                    e.tick_prepared(preps[k % R], tick)
                    evs[k % 4].record(st)
                    if k >= 2:
                        evs[(k - 2) % 4].synchronize()
                elif kind == "tick_ev3":  # the same, collected three ticks late
                    e.tick_prepared(preps[k % R], tick)
                    evs[k % 4].record(st)
                    if k >= 3:
                        evs[(k - 3) % 4].synchronize()
                elif kind == "tick_evnf":  # an event without the system-scope release per tick
                    e.tick_prepared(preps[k % R], tick)
                    hip.hipEventRecord(nf[k % 4], sp)
                    if k >= 2:
                        hip.hipEventSynchronize(nf[(k - 2) % 4])
                elif kind == "sync":
                    e.tick_ensemble_prepared(preps[k % R], rec)
                else:  # async: results collected two (async) or three (async3) events late
                    e.tick_ensemble_begin(preps[k % R])
                    pend += 1
                    if pend == (4 if kind == "async3" else 3):
                        e.ensemble_end()
                        pend -= 1
            while pend:
                e.ensemble_end()
                pend -= 1
        if args.comm:  # the real RCCL at world 1: the side-stream exchange of every result
            e.comm_init(fmskf.comm_unique_id(), 0, 1)
            res["comm"] = fmskf.rccl_library()
        for kind in ("tick", "tick_ev", "tick_ev3", "tick_evnf", "sync", "async", "async3") * 2:
            loop(kind, 8)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loop(kind, args.ticks)
            t1 = time.perf_counter()  # the host's submission of every call (and the result waits)
            torch.cuda.synchronize()
            res[kind + "_us"] = min(res.get(kind + "_us", 1e9), (time.perf_counter() - t0) * 1e6 / args.ticks)
            res[kind + "_host_us"] = min(res.get(kind + "_host_us", 1e9), (t1 - t0) * 1e6 / args.ticks)
        # the bench's K = 16 region shape: 20 ticks, one event at tick 10, its result collected
        # at the end (end() then synchronize, or synchronize then end()), against 20 plain ticks
        def region(kind):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(20):
                if kind != "plain" and k == 10:
                    e.tick_ensemble_begin(preps[k % R])
                else:
                    e.tick_prepared(preps[k % R], tick)
            if kind == "end_first":
                e.ensemble_end()
            torch.cuda.synchronize()
            if kind == "sync_first":
                e.ensemble_end()
            return (time.perf_counter() - t0) * 1e6 / 20
        for kind in ("plain", "end_first", "sync_first"):
            ts = sorted(region(kind) for _ in range(9))
            res["region20_" + kind + "_us"] = [round(ts[0], 2), round(ts[4], 2)]
        print(json.dumps(res), flush=True)
        return
    if args.op == "ensemble":  # the ensemble record reduction alone (partial + fold)
        rec = torch.empty(e.ensemble_record_len(), dtype=torch.float64, device=dev)
        e.ensemble_partial(rec)
        torch.cuda.synchronize()
        ev0.record(st)
        for _ in range(args.ticks):
            e.ensemble_partial(rec)
        ev1.record(st)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / args.ticks
        print(json.dumps({"model": args.model, "n": n, "op": "ensemble", "ms_per_call": ms,
                          "x_GBps": e.nx * e.elem * n / (ms * 1e-3) / 1e9}), flush=True)
        return
    if args.many:
        reps = max(1, args.ticks // args.many)
        sub = {k: v[: args.many] for k, v in many.items()}
        e.tick_many(args.many, **sub)
        torch.cuda.synchronize()
        ev0.record(st)
        for _ in range(reps):
            e.tick_many(args.many, **sub)
        ev1.record(st)
        torch.cuda.synchronize()
        ms_tick = ev0.elapsed_time(ev1) / (reps * args.many)
    else:
        ev0.record(st)
        for k in range(args.ticks):
            e.tick_prepared(preps[k % R], tick)
        ev1.record(st)
        torch.cuda.synchronize()
        ms_tick = ev0.elapsed_time(ev1) / args.ticks
    x, P = e.get_state()
    ok = bool(np.isfinite(x).all() and (P is None or np.isfinite(P).all()))
    print(json.dumps({"model": args.model, "n": n, "variant": os.environ.get("FMSKF_KF6_VARIANT", "0"),
                      "valid_mask": args.valid,
                      "op": args.op, "trig": args.trig, "many": args.many, "ms_per_tick": ms_tick,
                      "steps_per_s": n / (ms_tick * 1e-3),
                      "algo_GBps": BYTES[args.model] * n / (ms_tick * 1e-3) / 1e9, "finite": ok}),
          flush=True)


def bench_host(args, e, n, yaw, gz, rpm):
    """PCIe-inclusive rate: every tick's 16 B/robot of inputs start in host memory (--op isr:
    the fused ISR, its 0x200 frames returned to host memory every tick)."""
    import numpy as np
    import torch
    R = yaw.shape[0]
    pin = args.host == "pinned"
    hy, hg, hr = (t.cpu().pin_memory() if pin else t.cpu() for t in (yaw, gz, rpm))
    hy, hg, hr = (t.numpy() for t in (hy, hg, hr))
    if args.op == "isr":  # the host-fed firmware ISR: inputs from host, 0x200 frames back to host
        e.set_power(None)
        vel = np.zeros((3, n), np.float32)
        vel[0] = 150.0
        e.set_target_vel(vel, np.full((3, n), 1000.0, np.float32), np.full((3, n), 10000.0, np.float32))
        step = lambda k: e.isr_tick(yaw_deg=hy[k % R], gyro_z_dps=hg[k % R], rpm=hr[k % R])  # noqa: E731
    else:
        step = lambda k: e.tick(yaw_deg=hy[k % R], gyro_z_dps=hg[k % R], rpm=hr[k % R])  # noqa: E731
    for k in range(5):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.ticks):
        step(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.ticks
    print(json.dumps({"model": args.model, "n": n, "op": args.op, "host_inputs": args.host,
                      "ms_per_tick": dt * 1e3, "steps_per_s": n / dt,
                      "pcie_GBps": 16 * n / dt / 1e9}), flush=True)


def bench_pipeline(args, e, n, yaw, gz, rpm, dev, st):
    """The firmware ISR per tick -- estimator tick, wheel loops, 0x200 frames -- as three
    launches, or replayed as one HIP graph (fmskf_graph_*); launch-bound at small N."""
    import torch
    st = torch.cuda.Stream()  # graph capture needs a real stream, not the null stream
    torch.cuda.set_stream(st)
    e.set_stream(st)
    e.set_power(None)
    vel = torch.zeros((3, n), device=dev)
    vel[0] = 150.0
    e.set_target_vel(vel, torch.full((3, n), 1000.0, device=dev), torch.full((3, n), 10000.0, device=dev))
    dy, dg, dr = yaw[0].clone(), gz[0].clone(), rpm[0].clone()
    # EKF9 reads the raw WT901 words (+ rpm) instead of yaw / gyro planes
    draw = torch.cat([torch.round(dy / 180.0 * 32768).to(torch.int16)[..., None],
                      torch.round(-dg / 2000.0 * 32768).to(torch.int16)[..., None],
                      torch.zeros(n, 2, dtype=torch.int16, device=dev), dr], -1).contiguous()
    fr = torch.empty((n, 8), dtype=torch.uint8, device=dev)

    # isr_can: fmskf_isr_tick_can (the tick's CAN RX fused into the KF6 ISR); can_isr: the same
    # work as fmskf_ingest_can + fmskf_isr_tick
    cf = torch.randint(0, 256, (n, 4, 8), dtype=torch.uint8, device=dev)
    cs = (torch.arange(4, device=dev, dtype=torch.int16) * 250).expand(n, 4).contiguous()

    def direct():
        imu = dict(yaw_deg=dy) if args.model == "rs" else dict(raw=draw) if args.model == "ekf9" else \
            dict(yaw_deg=dy, gyro_z_dps=dg)
        if args.op.startswith("isr_can"):
            e.isr_tick_can(cf, cs, out=fr, **imu)
            return
        if args.op.startswith("can_isr"):
            e.ingest_can(cf, cs)
            e.isr_tick(out=fr, **imu)
            return
        if args.op.startswith("isr"):  # fmskf_isr_tick: one fused kernel for RS, KF6 and EKF9
            if args.model == "ekf9":
                e.isr_tick(out=fr, raw=draw, rpm=dr)
            else:
                e.isr_tick(out=fr, yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
            return
        e.tick(yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
        e.control(dr)
        e.can_tx(fr)
    if args.op.endswith("_graph"):
        e.graph_begin()
        direct()
        e.graph_end()
        run = lambda: e.graph_launch(1)  # noqa: E731
    else:
        run = direct
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(st)
    for _ in range(args.ticks):
        run()
    ev1.record(st)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.ticks
    ms = ev0.elapsed_time(ev1) / args.ticks
    print(json.dumps({"model": args.model, "n": n, "op": args.op, "ms_per_tick": ms,
                      "host_ms_per_tick": wall * 1e3, "robot_ticks_per_s": n / (ms * 1e-3)}), flush=True)


def bench_io(args, e, n, R, dev, rpm, st):
    """The rows either side of the tick: control step (+TX frame), WT901 and CAN ingest."""
    import numpy as np
    import torch
    from fmskf.synth import wt901_frame
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.Generator(device="cpu").manual_seed(7)
    if args.op in ("control", "can_tx"):
        e.set_power(None)
        vel = torch.stack([torch.rand(n, generator=g) * 800 - 400, torch.rand(n, generator=g) * 800 - 400,
                           torch.rand(n, generator=g) * 6 - 3]).to(dev)
        acl = torch.tensor([[1000.0], [1000.0], [30.0]], device=dev).expand(3, n).contiguous()
        jrk = torch.tensor([[10000.0], [10000.0], [300.0]], device=dev).expand(3, n).contiguous()
        e.set_target_vel(vel, acl, jrk)
        frames = torch.empty((n, 8), dtype=torch.uint8, device=dev)
        run = (lambda k: e.control(rpm[k % R])) if args.op == "control" else (lambda k: e.can_tx(frames))
        # control: power 1 + interpolators 3x12 + FF_PI_D 4x4 read, rpm 8 read; writes
        # interpolator dt/v/a 3x3, FF_PI_D 4x6, vel_tgt 3, currents 8 (power on)
        bpr = (1 + 4 * 33 + 4 * 12 + 8 + 8 + 4 * 9 + 4 * 12 + 8 + 8) if args.op == "control" else 16  # round 6: 297 B
    elif args.op == "wt901":
        # one 10 ms poll per robot: acc, gyro, angle, quaternion frames (44 B), ring of R polls
        stride = 48
        rng = np.random.default_rng(1)
        polls = []
        for r in range(min(R, 8)):
            base = bytearray()
            for t in (0x51, 0x52, 0x53, 0x59):
                base += wt901_frame(t, rng.integers(0, 65536, 4))
            row = np.zeros(stride, np.uint8)
            row[:44] = np.frombuffer(bytes(base), np.uint8)
            polls.append(torch.from_numpy(np.tile(row, (n, 1))).to(dev))
        lens = torch.full((n,), 44, dtype=torch.int32, device=dev)
        run = lambda k: e.ingest_wt901(polls[k % len(polls)], lens)  # noqa: E731
        # the standard poll (bench.py PATH_BYTES): row 48 + len 4, parser window / count / flags r+w,
        # error, 15 registers, magnetometer + q_init read, Data page written
        bpr = 48 + 4 + 2 + 2 + 4 + 24 + 4  # round 6: 88 B (13 registers only in the row / Yaw-GZ words, no magnetometer)
    else:  # can
        rng = np.random.default_rng(2)
        fr = [torch.from_numpy(rng.integers(0, 256, (n, 4, 8)).astype(np.uint8)).to(dev) for _ in range(4)]
        stp = [torch.from_numpy((np.arange(4)[None, :] * 250 + k * 1000 + np.zeros((n, 1))).astype(np.int16)).to(dev)
               for k in range(4)]
        run = lambda k: e.ingest_can(fr[k % 4], stp[k % 4])  # noqa: E731
        if args.can_desync:  # one masked tick first: random robots' Status ring heads fall out of step
            e.ingest_can(fr[0], stp[0], torch.from_numpy(rng.integers(0, 16, n).astype(np.uint8)).to(dev))
        # per wheel: frame 8 + stamp 2 in; micro, angle (2 + 2), IIR y / x (4 + 4) and the int64
        # sum read and written; rpm, curr, the previous angle (2 + 2 + 2) written
        bpr = 4 * (10 + (2 + 2 + 2 + 2 + 4 + 4) + (2 + 2 + 4 + 4) + 2 + 2)  # round 6: 168 B
    for k in range(10):
        run(k)
    torch.cuda.synchronize()
    ev0.record(st)
    for k in range(args.ticks):
        run(k)
    ev1.record(st)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / args.ticks
    print(json.dumps({"model": args.model, "n": n, "op": args.op, "ms_per_call": ms,
                      "robots_per_s": n / (ms * 1e-3), "bytes_per_robot": bpr,
                      "algo_GBps": bpr * n / (ms * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
