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

BYTES = {"kf6": 232, "rs": 144, "ekf9": 448, "kf12d": 1504}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="kf6")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=300)
    ap.add_argument("--ring", type=int, default=16)
    ap.add_argument("--many", type=int, default=0, help="ticks per launch (tick_many)")
    ap.add_argument("--op", choices=["tick", "predict", "correct", "ensemble"], default="tick")
    ap.add_argument("--trig", choices=["table512", "libm"], default="table512")
    args = ap.parse_args()
    import numpy as np
    import torch
    import fmskf
    from fmskf.synth import kf6_ring_torch

    dev = torch.device("cuda", 0)
    n, R = args.n, max(args.ring, args.many)  # tick_many reads `many` ticks of the ring
    e = fmskf.Engine(args.model, n, trig=fmskf.TRIG_LIBM if args.trig == "libm" else fmskf.TRIG_TABLE512)
    st = torch.cuda.current_stream()
    e.set_stream(st)
    yaw, gz, rpm = kf6_ring_torch(n, R, device=dev)
    if args.model == "kf6":
        preps = [e.prepare(yaw_deg=yaw[r], gyro_z_dps=gz[r], rpm=rpm[r]) for r in range(R)]
        many = dict(yaw_deg=yaw, gyro_z_dps=gz, rpm=rpm)
    elif args.model == "rs":
        sums = torch.cumsum(torch.randint(-20, 20, (R, 4, n), device=dev, dtype=torch.int64), 0)
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
    tick = getattr(fmskf.load(), "fmskf_" + ("tick" if args.op == "ensemble" else args.op))
    for k in range(20):
        e.tick_prepared(preps[k % R], tick)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
                      "op": args.op, "trig": args.trig, "many": args.many, "ms_per_tick": ms_tick,
                      "steps_per_s": n / (ms_tick * 1e-3),
                      "algo_GBps": BYTES[args.model] * n / (ms_tick * 1e-3) / 1e9, "finite": ok}),
          flush=True)


if __name__ == "__main__":
    main()
