#!/usr/bin/env python3
"""Headline benchmark: KF predict+update steps/s (whole node), 6-state fp32.

A step is one instance-tick (one correct + one predict of one filter); one timed
iteration ("tick") is one fused fmskf_tick launch over all instances of a GPU.
Workload (BASELINE.json configs[1] / SURVEY.md 8(d) cfg 2): 2^20 independent
6-state fp32 KF instances per GPU, inputs (IMU yaw + gyro z + 4 wheel rpm = 16 B
per instance-tick, one fmskf_kf6_record per robot; --inputs planes feeds the three
SoA planes instead) pre-generated into an HBM ring of 64 ticks (not timed).  Every
`--ensemble-every` ticks each rank reduces its ensemble mean/covariance record and,
for N > 1, all-gathers it over RCCL (the cfg 4 collective).  Weak scaling: per-GPU
work is fixed as N grows.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "roboken-fmskf-robot-controller_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "KF predict+update steps/s (whole node), 6-state fp32, at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes per instance-tick: x r+w 2*6*4, packed P r+w 2*21*4, input 16
BYTES_PER_STEP = {"kf6": 2 * 6 * 4 + 2 * 21 * 4 + 16}


EVENT_WINDOWS = 3


def event_ms(stream, run, ticks: int, prequeue: int = 8, windows: int = EVENT_WINDOWS) -> float:
    """GPU time per call of `run(k)`: the median over `windows` back-to-back windows of `ticks`
    calls, each between two HIP events on `stream` (the stream the kernels run on).  `prequeue`
    calls are queued before the first event, so the GPU is already busy when it is recorded and
    the host's launch lag at the start stays outside the timed span (round 4 recorded the first
    event on an idle stream: the average then exceeded the step itself); the median keeps one
    window that a host hiccup left the GPU idle in (a round-5 world-1 run: 40.7 us against
    37.0 us on the next measurement) out of the figure.  k runs on without a gap, so a
    prequeue and window that are multiples of 10 keep a 10-tick cycle aligned."""
    import torch
    for k in range(prequeue):
        run(k)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(windows + 1)]
    ev[0].record(stream)
    k = prequeue
    for w in range(windows):
        for _ in range(ticks):
            run(k)
            k += 1
        ev[w + 1].record(stream)
    torch.cuda.synchronize()
    per = sorted(ev[w].elapsed_time(ev[w + 1]) / ticks for w in range(windows))
    return per[len(per) // 2]


def mall_regime(state_and_input_bytes: float) -> str:
    """'hbm+mall' while one launch's state and inputs fit the 256 MiB Infinity Cache (MALL), so
    part of the traffic is served there; 'hbm' once they stream from HBM.  The headline passes
    124 B x N (the KF6 state read plus the 16-byte record); the other lines half their
    algorithmic bytes (every state byte is read once and written once)"""
    return "hbm+mall" if state_and_input_bytes <= (256 << 20) else "hbm"


def traffic_of(entry):
    """(PMC bytes per launch, where they came from) of a profiles/pmc_traffic*.json entry"""
    if not isinstance(entry, dict) or "hbm_bytes_per_launch" not in entry:
        return None, None
    src = entry.get("source") or {}
    what = f"{src.get('round', '?')} rocprofv3 FETCH_SIZE + WRITE_SIZE passes of {src.get('kernel', entry.get('kernel'))}"
    if src.get("committed_as"):
        what += " (" + ", ".join(src["committed_as"]) + ")"
    return entry["hbm_bytes_per_launch"], what


def scaling_diag(per_rank, exch_per_rank, value: float, ms_per_step: float, tick_ms_max: float) -> dict:
    """Why an N > 1 line's value is what it is.  per_rank: (rank, robots, plain-tick kernel ms) of
    every rank, measured with no collective in flight; exch_per_rank: every rank's side-stream
    exchange times (ms) of the timed region's ensemble events (fmskf_ensemble_exchange_ms).
    scaling_self = value / the sum of the ranks' plain-tick rates: 1.0 is perfect weak scaling of
    the kernels themselves; what is missing went to launch gaps, the ensemble ticks' record
    epilogue, the barrier and the exchange."""
    rates = [nr / (ms * 1e-3) for _, nr, ms in per_rank]
    kms = [ms for _, _, ms in per_rank]
    diag = {"tick_kernel_ms_min": min(kms), "tick_kernel_ms_max": max(kms), "tick_kernel_ms_per_rank": kms,
            "rank_local_rate_sum": sum(rates), "scaling_self": value / sum(rates),
            "ms_per_step_over_tick_kernel": ms_per_step / tick_ms_max}
    allx = [v for r in exch_per_rank for v in (r or [])]
    diag["exchange_ms"] = None if not allx else {
        "what": "side stream: ncclAllGather of the 28-double record + copy of the gathered records to "
                "pinned host memory (fmskf_ensemble_exchange_ms)",
        "events_per_rank": max(len(r or []) for r in exch_per_rank), "mean": sum(allx) / len(allx),
        "max_over_ranks": max(allx), "per_rank_max": [max(r) if r else None for r in exch_per_rank]}
    return diag


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def launcher_cmd(argv, env) -> list[str] | None:
    """`--gpus N > 1` without a launcher around us (no WORLD_SIZE in the environment): the
    torch.distributed.run command that runs this same bench as N ranks, one per GPU (None when
    no spawn is needed).  The parent never imports torch or touches a GPU; it starts the
    launcher as a child process and exits with its status (no exec of a GPU process)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    if a.gpus <= 1 or "WORLD_SIZE" in env:
        return None
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def cpu_share() -> dict:
    """What the CPU baseline may use on this host: the process's CPU affinity and the OpenMP
    thread count (OMP_NUM_THREADS; the GPU pool sets 16, each GPU's share of the host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return {"affinity_cpus": aff, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "host_cpus": os.cpu_count()}


def cpu_model() -> str:
    """The host CPU's model string (/proc/cpuinfo, as lscpu prints it)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(yaw, gz, rpm, sample_s: float):
    """The same KF6 tick on this host's CPU cores, on a bounded sample (the first 2^18 robots of
    the bench's inputs).  `value` is the tuned port (oracle/cpu_port.c: the tick specialised for
    KF6, the robots of a block in AVX-512 / AVX2 lanes, OpenMP threads over blocks, the oracle's
    operation order -- bitwise the checker's, verified on the sample here); `value_checker` is
    the generic one-robot-at-a-time oracle the tests check against.  Also the reference-semantics
    RS tick (the firmware ISR's arithmetic, VD_vehicle_controller.cpp:11-51) through the same
    port.  All on the process's OpenMP threads and on one thread."""
    import numpy as np
    import fmskf
    from oracle import oracle as orc
    n = yaw.shape[1]
    T = yaw.shape[0]
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]))
    threads = orc.max_threads()
    p0 = np.float32(np.array(cfg.p0[:21]))

    def rate(fn, budget):
        x = np.zeros((6, n), np.float32)
        P = np.repeat(p0[:, None], n, 1).copy()
        ticks = 0
        t0 = time.perf_counter()
        while True:
            fn(x, P, ticks % T)
            ticks += 1
            el = time.perf_counter() - t0
            if el >= budget and ticks >= 3:
                return n * ticks / el, ticks, el

    port = lambda nt: (lambda x, P, t: orc.port_kf6_tick(x, P, yaw[t], gz[t], rpm[t], prm, nthreads=nt))  # noqa: E731
    chk = lambda nt: (lambda x, P, t: orc.kf6_tick(x, P, yaw[t], gz[t], rpm[t], None, prm, nthreads=nt))  # noqa: E731
    # the port against the checker on the sample: three ticks from the same start, bit for bit
    xs = [np.zeros((6, n), np.float32) for _ in range(2)]
    Ps = [np.repeat(p0[:, None], n, 1).copy() for _ in range(2)]
    for t in range(3):
        port(threads)(xs[0], Ps[0], t)
        chk(threads)(xs[1], Ps[1], t)
    same = bool(np.array_equal(xs[0].view(np.uint32), xs[1].view(np.uint32)) and
                np.array_equal(Ps[0].view(np.uint32), Ps[1].view(np.uint32)))
    v, ticks, el = rate(port(threads), sample_s * 0.45)
    v1, t1, e1 = rate(port(1), max(1.5, sample_s * 0.15))
    vc, tc, ec = rate(chk(threads), max(1.5, sample_s * 0.15))
    # the reference-semantics tick (RS): encoder sums drifting by a few counts per tick
    sums = np.cumsum(np.random.default_rng(5).integers(-40, 40, (T, 4, n)), 0).astype(np.int64)
    pos, vel, prev = np.zeros((3, n), np.float32), np.zeros((3, n), np.float32), np.zeros((4, n), np.int64)
    rs = {}
    for label, nt, budget in (("all", threads, sample_s * 0.15), ("one", 1, max(1.0, sample_s * 0.1))):
        k, t0 = 0, time.perf_counter()
        while True:
            orc.port_rs_tick(pos, vel, prev, yaw[k % T], sums[k % T], rpm[k % T], nthreads=nt)
            k += 1
            el_rs = time.perf_counter() - t0
            if el_rs >= budget and k >= 3:
                break
        rs[label] = n * k / el_rs
    share = cpu_share()
    isa = orc.port().isa
    return {
        "value": v, "unit": "steps/s", "cores": threads, "kind": "port",
        "variant": f"tuned port: oracle/cpu_port.c, -march=x86-64-{isa} "
                   f"({'AVX-512' if isa == 'v4' else 'AVX2'}), robots in SIMD lanes, OpenMP over blocks",
        "bitexact_vs_checker": same,
        "cores_why": f"OpenMP threads = omp_get_max_threads() = {threads} (OMP_NUM_THREADS="
                     f"{share['omp_num_threads_env']}: the pool's per-GPU CPU share); process affinity "
                     f"{share['affinity_cpus']} of {share['host_cpus']} host CPUs",
        **share,
        "sample": f"{n} instances x {ticks} ticks ({el:.1f} s) of the same fused KF6 tick through the tuned "
                  f"port on {threads} threads; 1 thread {t1} ticks ({e1:.1f} s); the checker "
                  f"(oracle/fmskf_oracle.c orc_kf6_tick, generic n-state, one robot at a time, -O3 "
                  f"-march=x86-64-v3) {tc} ticks ({ec:.1f} s) on {threads} threads",
        "cpu_model": cpu_model(),
        "value_1core": v1,
        "value_checker": vc,
        "rs_tick": {"steps_per_s": rs["all"], "steps_per_s_1core": rs["one"],
                    "what": "reference-semantics tick (correct + odometry predict, VD_vehicle_controller.cpp:"
                            "11-51) through oracle/cpu_port.c port_rs_tick, bitwise orc_rs_tick"},
    }


def parity_sample(eng, applied, yaw, gz, rpm, trig, seed=0, k=2048):
    """The bench engine's state after every tick it ran (`applied`: the ring index of each, in
    order) against the oracle's restatement of the same sequence on k sampled robots (the first,
    the last and k - 2 seeded random ones): bit-exact or not.  Test infrastructure used as the
    checker after the timed regions, never inside them."""
    import numpy as np
    import fmskf
    from oracle import oracle as orc
    n = eng.n
    rng = np.random.default_rng(1234 + seed)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, max(0, k - 2))]))
    ti = __import__("torch").from_numpy(idx).to(yaw.device)
    ys = yaw[:, ti].cpu().numpy()
    gs = gz[:, ti].cpu().numpy()
    rs = np.ascontiguousarray(rpm[:, ti].cpu().numpy())
    cfg = fmskf.default_config("kf6", n)
    prm = orc.kf6_params(cfg.dt, np.array(cfg.q[:21]), np.array(cfg.r[:10]),
                         orc.TRIG_LIBM if trig == fmskf.TRIG_LIBM else orc.TRIG_TABLE512)
    m = idx.size
    xo = np.zeros((6, m), np.float32)
    Po = np.repeat(np.float32(np.array(cfg.p0[:21]))[:, None], m, 1).copy()
    for r in applied:
        orc.kf6_tick(xo, Po, np.ascontiguousarray(ys[r]), np.ascontiguousarray(gs[r]),
                     np.ascontiguousarray(rs[r]), None, prm, nthreads=0)
    x, P = eng.get_state()
    bad = ~(np.all(x[:, idx].view(np.uint32) == xo.view(np.uint32), axis=0) &
            np.all(P[:, idx].view(np.uint32) == Po.view(np.uint32), axis=0))
    return {"robots": int(m), "ticks": len(applied), "mismatched_robots": int(bad.sum()),
            "bitexact": not bool(bad.any()), "against": "oracle/fmskf_oracle.c orc_kf6_tick"}


def secondary_configs(dev, stream, ticks: int, trig):
    """BASELINE.json configs[2] (EKF9 2^22), configs[4] (KF12D fp64 2^20) and the cache-busting
    cfg 2 at 2^24: each model's single-tick kernel, back to back, HIP events
    on the stream it runs on; one line each with kernel_ms and its HBM roofline."""
    import torch
    import fmskf
    from fmskf.synth import SEED, kf6_ring_torch
    out = {}
    # HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE, calibrated on same-width
    # patterns (tools/pmc_traffic.py secondary; profiles/pmc_traffic_secondary.json)
    # (the 2^20 COMP line is calibrated like the path rows: profiles/pmc_traffic_paths.json)
    sec_traffic = {}
    for tname in ("pmc_traffic_secondary.json", "pmc_traffic_paths.json"):
        tpath = os.path.join(ROOT, "profiles", tname)
        if os.path.exists(tpath):
            try:
                sec_traffic.update({k: (*traffic_of(v), f"profiles/{tname}") for k, v in json.load(open(tpath)).items()
                                    if traffic_of(v)[0] is not None})
            except Exception:
                pass
    # algorithmic bytes per robot-tick as SURVEY.md 8(d) prices them (x and P read and written +
    # the inputs): EKF9 448 (its compensated heading's hidden low-part row, 8 B more read and
    # written, is reported beside it as `bytes_with_hidden_rows`), KF12D 1504, KF6 232; with
    # FMSKF_CFG_COMP_POS (the position low parts: 5 rows read and written, 40 B) KF6 272, EKF9 488
    specs = [("cfg3_ekf9_2p22", "ekf9", 1 << 22, 448, 456, 0), ("cfg5_kf12d_2p20", "kf12d", 1 << 20, 1504, None, 0),
             ("cfg2_kf6_2p24", "kf6", 1 << 24, 232, None, 0),
             ("cfg2_kf6_comp_pos_2p20", "kf6", 1 << 20, 272, None, fmskf.CFG_COMP_POS),
             ("cfg3_ekf9_comp_pos_2p22", "ekf9", 1 << 22, 488, 496, fmskf.CFG_COMP_POS)]
    R = 4
    for key, model, n, bps, bps_hidden, flags in specs:
        e = fmskf.Engine(model, n, device=dev.index, trig=trig, flags=flags)
        e.set_stream(stream)
        yaw, gz, rpm = kf6_ring_torch(n, R, seed=SEED ^ 7, device=dev)
        if model == "kf6":
            rec = fmskf.kf6_records(yaw, gz, rpm)
            preps = [e.prepare(kf6_rec=rec[r]) for r in range(R)]
            keep = (rec,)
        elif model == "ekf9":
            raw = torch.cat([torch.round(yaw / 180.0 * 32768).clamp(-32768, 32767).to(torch.int16)[..., None],
                             torch.round(-gz / 2000.0 * 32768).clamp(-32768, 32767).to(torch.int16)[..., None],
                             torch.zeros(R, n, 2, dtype=torch.int16, device=dev), rpm], -1).contiguous()
            preps = [e.prepare(raw=raw[r]) for r in range(R)]
            keep = (raw,)
        else:
            z = torch.zeros(R, 8, n, dtype=torch.float64, device=dev)
            z[:, 0] = torch.deg2rad(yaw.double())
            z[:, 1] = -torch.deg2rad(gz.double())
            z[:, 2] = 0.3
            z[:, 4] = 0.5
            preps = [e.prepare(z=z[r]) for r in range(R)]
            keep = (z,)
        del yaw, gz, rpm
        for k in range(3):
            e.tick_prepared(preps[k % R])
        torch.cuda.synchronize()
        ms = event_ms(stream, lambda k: e.tick_prepared(preps[k % R]), ticks)
        cnt = e.get_counters()
        e.close()
        del preps, keep
        torch.cuda.empty_cache()
        gbps = bps * n / (ms * 1e-3) / 1e9
        out[key] = {"model": model, "instances": n, "steps_per_s": n / (ms * 1e-3), "kernel_ms": ms,
                    "ticks": ticks, "nonfinite_instances": int(cnt[0]),
                    "roofline": {"bound": "hbm", "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                 "frac": gbps / HBM_PEAK_GBPS, "regime": mall_regime(bps * n / 2),
                                 "traffic": sec_traffic.get(key, (None,))[0],
                                 "traffic_source": (f"{sec_traffic[key][2]}: {sec_traffic[key][1]}"
                                                    if key in sec_traffic else None),
                                 "bytes_per_step": bps}}
        if flags:
            out[key]["config_flags"] = "FMSKF_CFG_COMP_POS"
        if bps_hidden:
            g2 = bps_hidden * n / (ms * 1e-3) / 1e9
            out[key]["roofline"]["bytes_with_hidden_rows"] = {"bytes_per_step": bps_hidden, "achieved": g2,
                                                              "frac": g2 / HBM_PEAK_GBPS}
    out["cfg4_shard_kf6_2p21"] = cfg4_shard(dev, stream, max(ticks, 32), trig)
    return out


# the WT901 standard poll's bytes (PATH_BYTES wt901_ingest_2p20) and the C610 RX of four wheels
# (can_ingest_2p20)
WT901_POLL_BYTES = 48 + 4 + 2 + 2 + 4 + 24 + 4
CAN_RX_BYTES = 4 * (10 + (2 + 2 + 2 + 2 + 4 + 4) + (2 + 2 + 4 + 4) + 2 + 2)
# the vehicle control step (control_step_2p20): power 1, interpolators 132 (every field but the
# acceleration, which update() writes before it reads it), FF_PI_D integral / LPF 48, the last
# step's rpm 8 (FF_PI_D now_val is formed from it), rpm 8 read; interpolator time / speed / accel
# 36, FF_PI_D 48, the rpm 8 and the currents 8 written (369 before round 6, with vel_tgt and
# FF_PI_D now_tgt / now_ctrl stored by every step and now_val as four floats)
CTRL_STEP_BYTES = 1 + 132 + 48 + 8 + 8 + 36 + 48 + 8 + 8
# algorithmic bytes per robot of the rows either side of the tick
PATH_BYTES = {
    # RS tick: pos (x, y) 8 r + (x, y, th) 12 w -- theta is overwritten by the correct, so it is
    # never read --, prev 32 r+w, sums 32, yaw 4, rpm 8 in, vel 12 out (the same bytes with the
    # sums at a padded pitch, or read from the ingested motor / IMU state)
    "rs_tick_2p20": 140,
    "rs_tick_2p20_padded_sums": 140,
    "rs_tick_2p20_device_state": 140,
    # WT901 standard poll: row 48 + len 4, the parser count and update flags 2 r, flags and error
    # 2 w, 2 registers 4 w (TEMP, VERSION: of the other thirteen the poll writes, eleven live in
    # the snapshot row and GZ / Yaw in the Yaw / GZ dword, round 6), the snapshot row 24 w (the
    # words updateData reads but the magnetometer's, which the standard poll does not carry and
    # the snapshot takes from sReg: round 6; the Data page is formed at readout), the Yaw / GZ
    # words 4 w (what the tick reads as its yaw and gyro z); the parser window is empty
    # before and after such a poll, so its words are neither read nor written (round 4: 197 B,
    # with the window words, q_init read and the 64-byte page written; round 5: 132 B, the 15
    # registers written to sReg as well as to the row; round 6: 110 B with GZ / Yaw in sReg and
    # the yaw / gyro z floats, then 102, then 88 without the magnetometer read and row words)
    "wt901_ingest_2p20": WT901_POLL_BYTES,
    # CAN RX, per wheel: frame 8 + stamp 2 in; micro, angle, previous angle, previous stamp, IIR
    # output y and the low word of the int64 sum read; the new stamp and angle (over the older
    # history slots: the current ones become the previous ones where they lie, round 6), IIR y and
    # the sum's low word written (round 6: the high word only on a carry across 2^32); rpm and curr
    # written (the speed is the IIR state y; Status's dlt is formed at readout from the angle and
    # the previous one; the IIR input state x is formed from the previous frame's angle and stamp
    # (round 5: 224 -> 216 B; round 6: 216 -> 184 -> 168 B))
    "can_ingest_2p20": CAN_RX_BYTES,
    # control step: power 1, interpolators 132, FF_PI_D 48 + 8, rpm 8 r; 36 + 48 + 8 + 8 w (round 6: the
    # outputs nothing reads back -- vel_tgt 12, FF_PI_D now_tgt / now_ctrl 32 -- formed on demand)
    "control_step_2p20": CTRL_STEP_BYTES,
    # fused KF6 ISR: the tick's 232 + the control step's CTRL_STEP_BYTES without its rpm read (the tick
    # loads it once) + the 8-byte 0x200 frame
    "isr_kf6_2p20": 232 + CTRL_STEP_BYTES - 8 + 8,
    # the firmware loop per tick on device-resident state: CAN RX, the fused KF6 ISR reading the
    # ingested Yaw / GZ words (one dword for the record's two floats, round 6) and wheel rpm, and
    # every 10th tick the WT901 poll
    "firmware_loop_kf6_2p20": CAN_RX_BYTES + (232 + CTRL_STEP_BYTES - 8 + 8) - 4 + WT901_POLL_BYTES / 10,
    # fmskf_isr_tick_can alone (the tick's CAN RX fused into the KF6 ISR, yaw / gyro planes): the
    # CAN row's 184 + the ISR's 601 without its rpm read
    "isr_can_kf6_2p20": CAN_RX_BYTES + (232 + CTRL_STEP_BYTES - 8 + 8) - 8,
    # the EKF9 ISR (k_isr_ekf9, round 5): the EKF9 tick's 448 (cfg 3's count; + 8 B with the
    # heading's hidden low-part row) + the control step's CTRL_STEP_BYTES (its own rpm plane: the tick reads
    # the raw record) + the 0x200 frame
    "isr_ekf9_2p20": 448 + CTRL_STEP_BYTES + 8,
    # with the tick's CAN RX fused in (fmskf_isr_tick_can): the CAN row's 184, the control step's
    # rpm no longer read back
    "isr_can_ekf9_2p20": CAN_RX_BYTES + (448 + CTRL_STEP_BYTES + 8) - 8,
    # the reference-semantics ISR (k_isr_rs) on the ingested motor state: the RS tick's 140 + the
    # control step's 369 without its rpm read (the tick loads it once) + the 0x200 frame
    "isr_rs_2p20": 140 + CTRL_STEP_BYTES - 8 + 8,
    # with the tick's CAN RX fused in: the CAN row's 184, the rpm and the four sums no longer read
    # back (the CAN lane hands them over in registers), and (round 6) the previous sums neither
    # read nor written while they equal the motor state's stored sums (k_isr_rs PS: 64 B)
    "isr_can_rs_2p20": CAN_RX_BYTES + (140 + CTRL_STEP_BYTES - 8 + 8) - 8 - 32 - 64,
    # the reference-semantics firmware loop (VD_task_main.cpp:366-372 with its CAN RX and IMU
    # tasks) on the fused call: CAN RX + the RS ISR in one kernel, a WT901 poll every 10th tick
    "firmware_loop_rs_fused_2p20": CAN_RX_BYTES + (140 + CTRL_STEP_BYTES - 8 + 8) - 8 - 32 - 64 + WT901_POLL_BYTES / 10,
    # the same loop with the CAN RX fused into the ISR (fmskf_isr_tick_can): the ISR no longer
    # reads the rpm plane back (the CAN lane hands it over in registers); everything else stays
    "firmware_loop_kf6_fused_2p20": CAN_RX_BYTES + (232 + CTRL_STEP_BYTES - 8 + 8) - 8 - 4 + WT901_POLL_BYTES / 10,
}


def path_rows(dev, stream, ticks: int, trig):
    """The reference-semantics tick and the rows either side of the
    tick (8(f) 1-3) at 2^20 robots, each its kernel back to back between HIP events on the
    stream it runs on: WT901 ingest of the standard 10 ms poll, C610 CAN RX, the vehicle control
    step and the fused KF6 firmware ISR (tick + control + 0x200 frame); kernel_ms and roofline
    each (bytes: PATH_BYTES)."""
    import numpy as np
    import torch
    import fmskf
    from fmskf.synth import SEED, kf6_ring_torch, wt901_frame
    n, R = 1 << 20, 4
    yaw, gz, rpm = kf6_ring_torch(n, R, seed=SEED ^ 11, device=dev)
    out = {}
    # memory-side bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the same
    # kernels at 2^20 (tools/pmc_traffic.py paths; profiles/pmc_traffic_paths.json)
    path_traffic = {}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic_paths.json")
    if os.path.exists(tpath):
        try:
            path_traffic = {k: traffic_of(v) for k, v in json.load(open(tpath)).items()
                            if traffic_of(v)[0] is not None}
        except Exception:
            path_traffic = {}

    def timed(key, run, e):
        for k in range(3):
            run(k)
        torch.cuda.synchronize()
        # the prequeued calls keep the loop's own k sequence (the firmware loop's WT901 poll
        # every 10th tick), so a multiple of 10 is queued ahead
        ms = event_ms(stream, run, ticks, prequeue=10)
        gbps = PATH_BYTES[key] * n / (ms * 1e-3) / 1e9
        tr = path_traffic.get(key, (None, None))
        out[key] = {"instances": n, "kernel_ms": ms, "robots_per_s": n / (ms * 1e-3), "ticks": ticks,
                    "roofline": {"bound": "hbm", "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                 "frac": gbps / HBM_PEAK_GBPS, "bytes_per_step": PATH_BYTES[key],
                                 "regime": mall_regime(PATH_BYTES[key] * n / 2),
                                 "traffic": tr[0],
                                 "traffic_source": f"profiles/pmc_traffic_paths.json: {tr[1]}" if tr[1] else None}}
        e.close()

    e = fmskf.Engine("rs", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    sums = torch.cumsum(torch.randint(-20, 20, (R, 4, n + 512), device=dev, dtype=torch.int64), 0)
    # the caller's [4][N] sum planes at the power-of-two stride N, and at a padded pitch
    # (fmskf_tick_inputs.angle_sum_pitch = N + 512)
    dense = sums[:, :, :n].contiguous()
    preps = [e.prepare(yaw_deg=yaw[r], angle_sum=dense[r], rpm=rpm[r]) for r in range(R)]
    timed("rs_tick_2p20", lambda k: e.tick_prepared(preps[k % R]), e)
    e = fmskf.Engine("rs", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    preps = [e.prepare(yaw_deg=yaw[r], angle_sum=sums[r], rpm=rpm[r]) for r in range(R)]
    timed("rs_tick_2p20_padded_sums", lambda k: e.tick_prepared(preps[k % R]), e)
    del preps, sums, dense
    # the firmware pipeline's form: every input from the device-resident ingest state (yaw from
    # the IMU Data page, sums and rpm from the motor state at its padded pitch)
    e = fmskf.Engine("rs", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    e.ingest_can(torch.zeros((n, 4, 8), dtype=torch.uint8, device=dev),
                 torch.zeros((n, 4), dtype=torch.int16, device=dev))
    e.ingest_wt901(torch.zeros((n, 48), dtype=torch.uint8, device=dev),
                   torch.zeros(n, dtype=torch.int32, device=dev))
    prep0 = e.prepare()
    timed("rs_tick_2p20_device_state", lambda k: e.tick_prepared(prep0), e)
    del prep0

    e = fmskf.Engine("kf6", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    rng = np.random.default_rng(SEED)
    polls = []
    for _ in range(R):
        b = b"".join(wt901_frame(t, rng.integers(0, 65536, 4)) for t in (0x51, 0x52, 0x53, 0x59))
        row = np.zeros(48, np.uint8)
        row[:44] = np.frombuffer(b, np.uint8)
        polls.append(torch.from_numpy(np.tile(row, (n, 1))).to(dev))
    lens = torch.full((n,), 44, dtype=torch.int32, device=dev)
    timed("wt901_ingest_2p20", lambda k: e.ingest_wt901(polls[k % R], lens), e)
    del polls

    e = fmskf.Engine("rs", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    frames = [torch.from_numpy(rng.integers(0, 256, (n, 4, 8)).astype(np.uint8)).to(dev) for _ in range(R)]
    stamps = [torch.from_numpy((np.arange(4)[None, :] * 250 + k * 1000 + np.zeros((n, 1))).astype(np.int16)).to(dev)
              for k in range(R)]
    timed("can_ingest_2p20", lambda k: e.ingest_can(frames[k % R], stamps[k % R]), e)

    def driven(model):
        en = fmskf.Engine(model, n, device=dev.index, trig=trig)
        en.set_stream(stream)
        en.set_power(None)
        g = torch.Generator(device="cpu").manual_seed(7)
        vel = torch.stack([torch.rand(n, generator=g) * 800 - 400, torch.rand(n, generator=g) * 800 - 400,
                           torch.rand(n, generator=g) * 6 - 3]).to(dev)
        en.set_target_vel(vel, torch.tensor([[1000.0], [1000.0], [30.0]], device=dev).expand(3, n).contiguous(),
                          torch.tensor([[10000.0], [10000.0], [300.0]], device=dev).expand(3, n).contiguous())
        return en

    e = driven("kf6")
    timed("control_step_2p20", lambda k: e.control(rpm[k % R]), e)
    e = driven("kf6")
    fr = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    timed("isr_kf6_2p20", lambda k: e.isr_tick(out=fr, yaw_deg=yaw[k % R], gyro_z_dps=gz[k % R], rpm=rpm[k % R]), e)
    e = driven("ekf9")
    raw = torch.cat([torch.round(yaw / 180.0 * 32768).to(torch.int16)[..., None],
                     torch.round(-gz / 2000.0 * 32768).to(torch.int16)[..., None],
                     torch.zeros(R, n, 2, dtype=torch.int16, device=dev), rpm], -1).contiguous()
    timed("isr_ekf9_2p20", lambda k: e.isr_tick(out=fr, raw=raw[k % R], rpm=rpm[k % R]), e)
    e = driven("ekf9")
    timed("isr_can_ekf9_2p20", lambda k: e.isr_tick_can(frames[k % R], stamps[k % R], out=fr, raw=raw[k % R]), e)
    del raw
    e = driven("rs")
    e.ingest_can(frames[0], stamps[0])
    timed("isr_rs_2p20", lambda k: e.isr_tick(out=fr, yaw_deg=yaw[k % R]), e)
    e = driven("rs")
    timed("isr_can_rs_2p20", lambda k: e.isr_tick_can(frames[k % R], stamps[k % R], out=fr, yaw_deg=yaw[k % R]), e)
    e = driven("kf6")
    timed("isr_can_kf6_2p20", lambda k: e.isr_tick_can(frames[k % R], stamps[k % R], out=fr, yaw_deg=yaw[k % R],
                                                       gyro_z_dps=gz[k % R]), e)
    # the whole firmware loop (VDT::can_tx_routine_intr with the CAN RX and IMU tasks feeding it):
    # four C610 frames per robot every tick, a WT901 poll every 10th tick, the fused ISR on the
    # ingested state; time per tick over a multiple of 10 ticks
    e = driven("kf6")
    poll = torch.from_numpy(np.tile(np.frombuffer(b"".join(
        wt901_frame(t, rng.integers(0, 65536, 4)) for t in (0x51, 0x52, 0x53, 0x59)) + bytes(4), np.uint8),
        (n, 1))).to(dev)

    def loop(k):
        e.ingest_can(frames[k % R], stamps[k % R])
        if k % 10 == 0:
            e.ingest_wt901(poll, lens, latch_qinit=(k == 0))
        e.isr_tick(out=fr)
    timed("firmware_loop_kf6_2p20", loop, e)
    e = driven("kf6")

    def loop_fused(k):
        if k % 10 == 0:
            e.ingest_wt901(poll, lens, latch_qinit=(k == 0))
        e.isr_tick_can(frames[k % R], stamps[k % R], out=fr)
    timed("firmware_loop_kf6_fused_2p20", loop_fused, e)
    e = driven("rs")

    def loop_rs(k):
        if k % 10 == 0:
            e.ingest_wt901(poll, lens, latch_qinit=(k == 0))
        e.isr_tick_can(frames[k % R], stamps[k % R], out=fr)
    timed("firmware_loop_rs_fused_2p20", loop_rs, e)
    del yaw, gz, rpm, fr, frames, stamps, poll
    torch.cuda.empty_cache()
    return out


def cfg4_shard(dev, stream, ticks: int, trig):
    """BASELINE.json configs[3] on one GPU: its 2^21-robot per-GPU shard of the 16M fleet, the
    tick alone, with the asynchronous ensemble record every 16th tick and every tick (K = 16
    and K = 1, SURVEY.md 8(d) cfg 4: fmskf_tick_ensemble_begin, each result collected two
    events late, as the headline does); HIP events on the tick stream, no collective (that is
    the N > 1 bench run's).  Fed the SoA input planes: the record-fed kernel instantiation stays the
    headline's alone, so a rocprofv3 --stats summary of the bench keeps its 2^20 average."""
    import torch
    import fmskf
    from fmskf.synth import SEED, kf6_ring_torch
    n, R = 1 << 21, 8
    e = fmskf.Engine("kf6", n, device=dev.index, trig=trig)
    e.set_stream(stream)
    yaw, gz, rpm = kf6_ring_torch(n, R, seed=SEED ^ 4, device=dev)
    preps = [e.prepare(yaw_deg=yaw[r], gyro_z_dps=gz[r], rpm=rpm[r]) for r in range(R)]
    out_rec = torch.empty(e.ensemble_record_len(), dtype=torch.float64, device=dev)

    def run(every):
        pending = 0
        for k in range(ticks):
            if every and (k + 1) % every == 0:
                e.tick_ensemble_begin(preps[k % R])
                pending += 1
                if pending == 3:
                    e.ensemble_end()
                    pending -= 1
            else:
                e.tick_prepared(preps[k % R])
        for _ in range(pending):
            e.ensemble_end()

    res = {"instances": n, "ticks": ticks, "inputs": "planes"}
    for label, every in (("tick_only", 0), ("ensemble_every_16", 16), ("ensemble_every_1", 1)):
        run(every)  # warm-up: every kernel of this sequence loaded
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        run(every)
        ev1.record(stream)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / ticks
        res[label] = {"ms_per_step": ms, "steps_per_s": n / (ms * 1e-3)}
    gbps = 232 * n / (res["tick_only"]["ms_per_step"] * 1e-3) / 1e9
    res["roofline"] = {"bound": "hbm", "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                       "frac": gbps / HBM_PEAK_GBPS, "bytes_per_step": 232}
    e.ensemble_partial(out_rec)  # the record of the final state (sanity: every robot counted)
    res["ensemble_count"] = float(out_rec[0].item())
    e.close()
    del preps, yaw, gz, rpm
    torch.cuda.empty_cache()
    return res


def main():
    cmd = launcher_cmd(sys.argv[1:], os.environ)
    if cmd is not None:  # --gpus N > 1 with no launcher: run the N ranks as a child
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        print(f"bench: --gpus {cmd[4].split('=')[1]} without a launcher: {' '.join(cmd[1:9])} ...",
              file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd, env=env).returncode)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--n-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--n-total", type=int, default=0,
                    help="strong scaling: this many robots over all ranks (contiguous shards, the "
                         "remainder on the first ranks) instead of --n-per-gpu per rank")
    ap.add_argument("--ring", type=int, default=64)
    ap.add_argument("--ensemble-every", type=int, default=16)
    ap.add_argument("--trig", choices=["table512", "libm"], default="table512")
    ap.add_argument("--cpu-sample-s", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="skip the fused multi-tick figure")
    ap.add_argument("--gather", choices=["auto", "async", "stream", "native"], default="auto",
                    help="N > 1: native (the default with RCCL): libfmskf's own communicator "
                         "(fmskf_comm_init), fmskf_tick_ensemble_begin / fmskf_ensemble_end -- the "
                         "fused record, its fold carried by the next record's tick kernel (or run ahead of "
                         "the next plain tick), ncclAllGather + copy-out on the handle's side stream "
                         "overlapping the next ticks, the path C callers bind; async / stream: "
                         "torch.distributed all-gather on RCCL's stream or in the tick stream "
                         "(auto = native, or async under gloo / --same-device)")
    ap.add_argument("--ensemble", choices=["fused", "separate"], default="fused",
                    help="ensemble ticks: fmskf_tick_ensemble (the tick kernel writes the record) or "
                         "fmskf_tick + fmskf_ensemble_partial")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the cfg 3 / cfg 5 / 2^24 single-GPU kernel lines")
    ap.add_argument("--secondary-ticks", type=int, default=20)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend (gloo: test rehearsal of the N > 1 path, the "
                         "records staged through host memory)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing N > 1 on a one-GPU box; not a scaling run)")
    ap.add_argument("--check-ensemble", action="store_true",
                    help="after the timed region: the gathered record vs each rank's stand-alone "
                         "record of the same state (reported as ensemble_check)")
    ap.add_argument("--inputs", choices=["records", "planes"], default="records",
                    help="16-byte fmskf_kf6_record per robot (one load per lane) or yaw/gyro/rpm planes")
    ap.add_argument("--cfg4-16m", action="store_true",
                    help="also run BASELINE configs[3] (2^24 robots over the ranks) at world 1 "
                         "(at world > 1 it always runs, reported as cfg4_16M)")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the cfg4_16M block")
    ap.add_argument("--cfg4-steps", type=int, default=64)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import fmskf
    from fmskf.synth import SEED, kf6_ring_torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # a torch.distributed.run launch (RANK set) always builds the RCCL group, also at N=1,
    # so the collective path is the one measured whenever the launcher is used
    distributed = world > 1 or "RANK" in os.environ
    gloo = args.backend == "gloo"
    if distributed:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if distributed:
            if gloo:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])

    def all_gather(out, inp, async_op=False):
        """all-gather of device tensors (gloo: staged through host memory, synchronous)"""
        if not gloo:
            return dist.all_gather_into_tensor(out, inp, async_op=async_op)
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)
        return None

    def max_over_ranks(vals):
        t = torch.tensor(vals, dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.tolist()]

    if args.n_total > 0:  # SURVEY 8(d) cfg 4 strong scaling: the same 2^24 total at every N
        lo, hi = fmskf.shard_span(args.n_total, world, rank)
        n = hi - lo
        n_global = args.n_total
    else:
        n = args.n_per_gpu
        n_global = n * world
    R = args.ring
    stream = torch.cuda.current_stream()
    trig = fmskf.TRIG_LIBM if args.trig == "libm" else fmskf.TRIG_TABLE512
    eng = fmskf.Engine("kf6", n, device=local, trig=trig)
    eng.set_stream(stream)
    yaw, gz, rpm = kf6_ring_torch(n, R, seed=SEED ^ 2 ^ (rank << 8), device=dev)
    planes = [eng.prepare(yaw_deg=yaw[r], gyro_z_dps=gz[r], rpm=rpm[r]) for r in range(R)]
    if args.inputs == "records":
        krec = fmskf.kf6_records(yaw, gz, rpm)  # [R][N] 16-byte records (same values)
        prepared = [eng.prepare(kf6_rec=krec[r]) for r in range(R)]
        many_in = dict(kf6_rec=krec)
    else:
        krec = None
        prepared = planes
        many_in = dict(yaw_deg=yaw, gyro_z_dps=gz, rpm=rpm)
    tick_fn = fmskf.load().fmskf_tick
    rec_len = eng.ensemble_record_len()
    rec = torch.empty(rec_len, dtype=torch.float64, device=dev)
    n_events = max(1, (2 * args.steps + args.warmup) // max(1, args.ensemble_every) + 3)
    # one record and one gather slot per ensemble event: the all-gather runs asynchronously
    # on RCCL's stream (ordered after the record by RCCL's stream dependency) while the next
    # ticks proceed; pending gathers are joined before the timed region closes
    recs = torch.zeros(n_events, rec_len, dtype=torch.float64, device=dev)
    gathered = torch.zeros(n_events, world, rec_len, dtype=torch.float64, device=dev)
    ev_count = [0]
    pending = []

    if args.gather == "auto":
        args.gather = "async" if (gloo or args.same_device) else "native"
    def native_comm(e):
        """the handle's own RCCL communicator: rank 0's unique id reaches the others over the
        torch.distributed group, then fmskf_comm_init on every rank.  Returns every rank's error
        (empty when every communicator came up): all ranks learn the same list over torch's own
        group, so on any failure they all measure with torch's all-gather instead, and the line
        says why -- a failure is reported, never silent."""
        err, uid = None, [None]
        if rank == 0:
            try:
                uid = [fmskf.comm_unique_id()]
            except Exception as ex:  # noqa: BLE001
                err = f"rank 0: fmskf_comm_unique_id: {ex}"
        dist.broadcast_object_list(uid, src=0)
        if err is None and uid[0] is None:
            err = f"rank {rank}: no communicator id from rank 0"
        elif err is None:
            try:
                e.comm_init(uid[0], rank, world)
            except Exception as ex:  # noqa: BLE001
                err = f"rank {rank}: fmskf_comm_init: {ex}"
        errs = [None] * world
        dist.all_gather_object(errs, err)
        return [x for x in errs if x]

    rccl = None
    gather_fallback = None
    if args.gather == "native" and distributed:
        # the handle's own RCCL communicator: rank 0's unique id reaches the others over the
        # torch.distributed group (without a launcher there is no communicator: the fold writes
        # this GPU's record straight into the handle's pinned result slot)
        errs = native_comm(eng)
        if errs:
            gather_fallback = {"from": "native", "to": "async", "errors": errs}
            print(f"bench: fmskf_comm_init failed ({errs[0]}); measuring with --gather async", file=sys.stderr)
            args.gather = "async"
        else:
            # what RCCL itself reports (ncclCommCount / ncclCommUserRank), from every rank: a
            # one-rank communicator inside an N-process job would show here
            cw, cr = eng.comm_info()
            seen = [None] * world
            dist.all_gather_object(seen, (cw, cr))
            rccl = {"ranks": cw, "user_ranks": sorted(r for _, r in seen), "sizes": sorted({w for w, _ in seen}),
                    "library": fmskf.rccl_library()}
    native_stats = [None]
    native_pending = [0]
    exch_ms = []  # side-stream all-gather + copy-out time of every collected native result
    # ring index of every tick applied to `eng`, in order: the post-timing parity replay
    applied = []

    def tick(r, src=None):
        eng.tick_prepared((src or prepared)[r], tick_fn)
        applied.append(r)

    def native_collect(keep):
        """fmskf_ensemble_end_count of the oldest pending events until `keep` remain (the robots
        the gathered records count and how many records were folded are kept with the result)"""
        while native_pending[0] > keep:
            native_stats[0] = eng.ensemble_end_count()
            native_pending[0] -= 1
            xms = eng.ensemble_exchange_ms()  # -1 without a communicator (no side-stream gather)
            if xms >= 0:
                exch_ms.append(xms)

    def ens_event(k):
        """one ensemble event after tick k: record (fused into the tick, or a separate pass),
        then this rank's share of the all-gather"""
        e = ev_count[0] % n_events
        if args.gather == "native":
            # fused tick + record; its fold rides in the next record's tick kernel (or runs ahead
            # of the next plain tick), the all-gather and copy-out on the handle's side stream;
            # results are collected two events late (they finished while later ticks ran), so
            # the host never waits behind the tick stream
            eng.tick_ensemble_begin(prepared[k % R])
            applied.append(k % R)
            native_pending[0] += 1
            native_collect(2)
        else:
            # without a process group the "gather" is the identity: the record is written in
            # place into its gather slot
            dst = recs[e] if distributed else gathered[e][0]
            if args.ensemble == "fused":
                eng.tick_ensemble_prepared(prepared[k % R], dst)
                applied.append(k % R)
            else:
                tick(k % R)
                eng.ensemble_partial(dst)
            if distributed and (args.gather == "stream" or gloo):
                all_gather(gathered[e].view(-1), recs[e])
            elif distributed:
                pending.append(all_gather(gathered[e].view(-1), recs[e], async_op=True))
        ev_count[0] += 1

    def step(k):
        if args.ensemble_every > 0 and (k + 1) % args.ensemble_every == 0:
            ens_event(k)
        else:
            tick(k % R)

    def run_cfg4_16m():
        n_total = 1 << 24
        lo4, hi4 = fmskf.shard_span(n_total, world, rank)
        n4, R4 = hi4 - lo4, 8
        e4 = fmskf.Engine("kf6", n4, device=local, trig=trig)
        e4.set_stream(stream)
        y4, g4, r4 = kf6_ring_torch(n4, R4, seed=SEED ^ 0x16 ^ (rank << 8), device=dev)
        rec4 = fmskf.kf6_records(y4, g4, r4)
        del y4, g4, r4
        p4 = [e4.prepare(kf6_rec=rec4[r]) for r in range(R4)]
        native4 = args.gather == "native"
        info = None
        if native4 and distributed:
            errs4 = native_comm(e4)
            if errs4:  # every rank falls back together (torch's all-gather)
                native4 = False
            else:
                info = e4.comm_info()
        rb = torch.empty(e4.ensemble_record_len(), dtype=torch.float64, device=dev)
        gb = torch.empty(world, e4.ensemble_record_len(), dtype=torch.float64, device=dev)
        pend, last = [0], [None]

        def collect(keep):
            while pend[0] > keep:
                last[0] = e4.ensemble_end_count()
                pend[0] -= 1

        def run(every, ticks):
            for k in range(ticks):
                if (k + 1) % every:
                    e4.tick_prepared(p4[k % R4])
                elif native4:
                    e4.tick_ensemble_begin(p4[k % R4])
                    pend[0] += 1
                    collect(2)
                else:
                    e4.tick_ensemble_prepared(p4[k % R4], rb)
                    if distributed:
                        all_gather(gb.view(-1), rb)
                    else:
                        gb[0].copy_(rb)
            collect(0)

        res = {"instances_total": n_total, "instances_this_rank": n4, "n_gpus": world, "scaling": "strong",
               "inputs": "records", "gather": args.gather if native4 or args.gather != "native" else "async"}
        if not native4 and args.gather == "native":
            res["gather_fallback"] = errs4
        for label, every in (("ensemble_every_16", 16), ("ensemble_every_1", 1)):
            run(every, 2 * every + 6)  # warm-up: every kernel and result slot of this sequence
            torch.cuda.synchronize()
            barrier()
            torch.cuda.synchronize()
            ta = time.perf_counter()
            run(every, args.cfg4_steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - ta
            barrier()
            if distributed:
                el = max_over_ranks([el])[0]
            res[label] = {"steps_per_s": n_total * args.cfg4_steps / el, "ms_per_step": el * 1e3 / args.cfg4_steps,
                          "ticks": args.cfg4_steps}
        if native4:
            res["gathered_count"], res["records_folded"] = last[0][2], last[0][3]
        else:
            res["gathered_count"], res["records_folded"] = float(gb[:, 0].sum().item()), world
        if info is not None:
            res["rccl_ranks"], res["rccl_rank"] = info
        e4.close()
        del p4, rec4, rb, gb
        torch.cuda.empty_cache()
        return res

    def join():
        native_collect(0)
        while pending:
            pending.pop().wait()  # the current stream waits for the collective

    for k in range(args.warmup):
        step(k)
    # every path the timed region runs has run once before it (kernels load lazily on their
    # first launch: ~2 ms for the ensemble kernels, measured inside the timed region in round 1)
    if args.ensemble_every > 0 and (args.warmup < args.ensemble_every or args.warmup == 0):
        ens_event(args.warmup)
    if args.ensemble_every > 0 and args.gather == "native":
        # the handle's four result slots each come into use once before the timed region
        # (first record / wait of a slot's events), collected both ways: two events late and
        # the newest one by itself (its fold stand-alone)
        for j in range(5):
            ens_event(args.warmup + 1 + j)
        join()
        ens_event(args.warmup + 6)
    join()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # exactly the K timed ticks, wall clock between the two synchronisations (no event
    # record inside: its host call would delay the first launch)
    exch_ms.clear()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    t_sub = time.perf_counter()
    join()
    t_join = time.perf_counter()
    timed_exch = list(exch_ms)  # the exchanges of the timed region's ensemble events
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    # where the host spent the timed region (diagnostic): submitting the K steps, collecting
    # the pending ensemble results, the final synchronise
    host_split = {"submit_ms": (t_sub - t0) * 1e3, "join_ms": (t_join - t_sub) * 1e3,
                  "sync_ms": (t1 - t_join) * 1e3}
    # the same K-step sequence once more between HIP events on the tick stream: the GPU-side
    # duration of the timed region's work on the tick stream (diagnostic; `value` is the wall
    # clock above).  The second event is recorded before the pending results are collected:
    # that collection is a host wait on the side stream, and recording after it counted the
    # tick stream's idle time behind the wait (up to 3% of the span on a 20-step region)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for k in range(args.warmup + args.steps, args.warmup + 2 * args.steps):
        step(k)
    ev1.record(stream)
    join()
    torch.cuda.synchronize()
    region_ms = ev0.elapsed_time(ev1)

    # the tick kernel's own average launch duration (the roofline's denominator): the median of
    # three windows of KT >= 200 more back-to-back plain ticks on the kernel's stream, no
    # ensemble kernel and no collective in flight, 8 ticks queued before the first HIP event
    # (rocprofv3's per-kernel average for the same command: profiles/)
    KT = max(200, args.steps)
    tick_ms = event_ms(stream, lambda k: tick(k % R), KT)
    # secondary: the same tick fed the three input planes (when the headline uses records)
    planes_ms = tick_ms
    if args.inputs == "records":
        planes_ms = event_ms(stream, lambda k: tick(k % R, planes), KT)
    local_tick_ms = tick_ms
    per_rank = None
    if distributed:
        # each rank's own plain-tick time (min / max over ranks) and the rate it implies: a
        # scaling curve below world x that rate comes from outside the tick (launch, barrier,
        # the exchange), and the line says so (`scaling_diag`)
        seen = [None] * world
        dist.all_gather_object(seen, (rank, n, local_tick_ms))
        per_rank = sorted(seen)
        elapsed, region_ms, tick_ms, planes_ms = max_over_ranks([elapsed, region_ms, tick_ms, planes_ms])
    kern_avg_ms = tick_ms

    total_steps = n_global * args.steps
    value = total_steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # cfg 4 also reports K = 1: the ensemble record (and its all-gather for
    # N > 1) after every tick, over 256 more ticks -- a secondary figure, not `value`
    k1 = None
    if args.ensemble_every > 0:
        k1_steps = 256  # the drain of the last pending results at the end is amortized over 256 ticks
        barrier()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for k in range(k1_steps):
            # begin every tick, each result collected two ticks later (three: the same 2.68-2.69e10,
            # three alternating pairs on one box)
            if args.gather == "native":
                eng.tick_ensemble_begin(prepared[k % R])
                applied.append(k % R)
                native_pending[0] += 1
                native_collect(2)
                continue
            if args.ensemble == "fused":
                eng.tick_ensemble_prepared(prepared[k % R], rec)
                applied.append(k % R)
            else:
                tick(k % R)
                eng.ensemble_partial(rec)
            if distributed:
                all_gather(gathered[0].view(-1), rec)
        native_collect(0)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        k1_el = tb - ta
        if distributed:
            k1_el = max_over_ranks([k1_el])[0]
        k1 = {"steps_per_s": n_global * k1_steps / k1_el, "ms_per_step": k1_el * 1e3 / k1_steps,
              "ticks": k1_steps}

    # BASELINE configs[3] in the same invocation (SURVEY.md 8(d) cfg 4): 2^24 robots over the
    # ranks (contiguous shards, strong scaling), records, the ensemble record every 16th tick and
    # every tick, each result gathered over the ranks -- libfmskf's own communicator in the
    # native path -- and collected two events late; wall clock between barriers, max over ranks
    cfg4 = None
    if (world > 1 or args.cfg4_16m) and not args.no_cfg4:
        cfg4 = run_cfg4_16m()

    # ensemble sanity (outside the timed region): fold the last gathered records in rank order
    last = gathered[(ev_count[0] - 1) % n_events].cpu().numpy() if ev_count[0] else None
    ens = None
    if args.gather == "native" and native_stats[0] is not None:
        # the count is the gathered records' own (the sum of their count rows), not n_global
        mean, cov, cnt, nrec = native_stats[0]
        ens = {"count": cnt, "records_folded": nrec, "mean_theta": float(mean[2]), "var_vx": float(cov[9])}
    elif last is not None:
        mean, cov = fmskf.ensemble_combine(6, last)
        ens = {"count": float(last[:, 0].sum()), "mean_theta": float(mean[2]),
               "var_vx": float(cov[9])}
    counters = eng.get_counters()

    # --check-ensemble: one more ensemble event through the measured path (fused record or
    # separate partial, then the gather), against each rank's stand-alone record of the same
    # state folded the same way: max relative difference of mean and covariance
    ens_check = None
    if args.check_ensemble and args.ensemble_every > 0:
        k = args.warmup + 2 * args.steps
        e = ev_count[0] % n_events
        ens_event(k)
        join()
        torch.cuda.synchronize()
        own = torch.from_numpy(eng.ensemble_partial()).to(dev)
        allown = torch.zeros(world, rec_len, dtype=torch.float64, device=dev)
        if distributed:
            all_gather(allown.view(-1), own)
        else:
            allown[0].copy_(own)
        mr, cr = fmskf.ensemble_combine(6, allown.cpu().numpy())
        if args.gather == "native":
            mg, cg = native_stats[0][:2]
        else:
            mg, cg = fmskf.ensemble_combine(6, gathered[e].cpu().numpy())
        import numpy as np
        rel = lambda a, b: float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))  # noqa: E731
        ens_check = {"mean_max_rel": rel(mg, mr), "cov_max_rel": rel(cg, cr),
                     "count": float(allown[:, 0].sum().item())}

    # secondary figure: the same ring replayed by one fused multi-tick launch per ring pass
    fused = None
    if not args.no_fused:
        e2 = fmskf.Engine("kf6", n, device=local, trig=trig)
        e2.set_stream(stream)
        e2.tick_many(R, **many_in)
        torch.cuda.synchronize()
        reps = max(1, args.steps // R)
        ta = time.perf_counter()
        for _ in range(reps):
            e2.tick_many(R, **many_in)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        fused = {"ticks_per_launch": R, "steps_per_s_per_gpu": n * R * reps / (tb - ta),
                 "input_bytes_per_step": 16}
        e2.close()

    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("n_instances") == n and tj.get("kernel", "").startswith("k_kf6") and \
                    tj.get("inputs", "planes") == args.inputs:
                traffic, traffic_src = traffic_of(tj)
                traffic_src = f"profiles/pmc_traffic.json: {traffic_src}"
        except Exception:
            traffic, traffic_src = None, None

    bpl = BYTES_PER_STEP["kf6"] * n  # algorithmic bytes per launch (one tick of one GPU)
    achieved = bpl / (kern_avg_ms * 1e-3) / 1e9
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.n_total > 0 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: WT901 yaw/gyro-z + 4 wheel rpm per robot (fmskf.synth), 64-tick HBM ring"
                + (", one 16-byte fmskf_kf6_record per robot-tick" if krec is not None else ", SoA planes"),
        "config": {
            "workload": ("cfg2: 2^20 independent 6-state fp32 KF instances per GPU" if args.n_total <= 0 else
                         f"cfg4 strong scaling: {n_global} independent 6-state fp32 KF instances over "
                         f"{world} GPU(s)") +
                        ", fused correct+predict per tick (fmskf_tick; every ensemble_every-th tick "
                        + ("fmskf_tick_ensemble_begin: the tick kernel also writes the ensemble record, "
                           "its fold carried by the next tick, libfmskf's ncclAllGather + copy-out on a side "
                           "stream, fmskf_ensemble_end two events later)" if args.gather == "native" else
                           "fmskf_tick_ensemble, which also writes the ensemble record; torch "
                           "all-gather)"),
            "instances_per_gpu": n,
            "global_instances": n_global,
            "trig": args.trig,
            "inputs": args.inputs,
            "ensemble_every": args.ensemble_every,
            "ensemble": args.ensemble,
            "gather": args.gather,
            # the library libfmskf's communicator resolves (a rehearsal names its stand-in)
            "rccl_library": rccl["library"] if rccl is not None else None,
            "parallelism": f"instance-sharded x{world}" + (
                (", RCCL all-gather of ensemble records" if not gloo else ", gloo all-gather of ensemble records")
                if world > 1 else "") + (" (rehearsal: every rank on cuda:0)" if args.same_device else ""),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            # the PMC bytes are not collected inside this run (rocprofv3 counter passes need runs
            # of their own): the committed profile they come from
            "traffic_source": traffic_src,
            "bytes_per_step": BYTES_PER_STEP["kf6"],
            "kernel_ms": kern_avg_ms,
            # the launcher's choice (kernels_kf6.hip launch_o): 2 robots per lane while the
            # state and one tick's inputs (124 B per robot) fit the 256 MiB Infinity Cache
            "kernel": ("k_kf6p<4, 2, " if n * 124 <= (256 << 20) else "k_kf6t<4, ") +
                      "Opt<TABLE512, UPD, PRED, SMALL, !VALID" + (", REC>>" if krec is not None else ">>"),
            "timed_region_ms_per_step": region_ms / args.steps,
            "kernel_ms_plane_inputs": planes_ms,
            "kernel_ticks_timed": KT, "kernel_windows": EVENT_WINDOWS,  # kernel_ms: the median window
            # 124 B per robot (the state read + the 16-byte record) against the 256 MiB
            # Infinity Cache: at 2^20 the state stays MALL-resident between ticks, so `achieved`
            # is HBM + MALL; secondary.cfg2_kf6_2p24 is the HBM-only figure
            "regime": mall_regime(124 * n),
        },
        "timed_region_host": host_split,
        "cpu_baseline": None,
        "fused_replay": fused,
        "ensemble_every_1": k1,
        "ensemble": ens,
        "nonfinite_instances": int(counters[0]),
    }
    if ens_check is not None:
        out["ensemble_check"] = ens_check
    if gather_fallback is not None:
        out["gather_fallback"] = gather_fallback
    if per_rank is not None:
        # why the N > 1 value is what it is: each rank's plain tick alone (no collective in flight)
        # against the whole job's rate, and what the ensemble exchange cost on the side stream
        xs = [None] * world
        dist.all_gather_object(xs, timed_exch)
        diag = scaling_diag(per_rank, xs, value, ms_per_step, tick_ms)
        out["scaling_diag"] = diag
    if rccl is not None:
        # the communicator libfmskf's asynchronous exchange ran over, as RCCL reports it
        out["rccl_ranks"] = rccl["ranks"]
        out["rccl"] = rccl
    if cfg4 is not None:
        out["cfg4_16M"] = cfg4
    # post-timing parity (outside every timed region): the measured engine's state against the
    # oracle's restatement of the same tick sequence on sampled robots, bit for bit
    par = parity_sample(eng, applied, yaw, gz, rpm, trig, seed=rank)
    if distributed:
        bad, = max_over_ranks([float(par["mismatched_robots"])])
        par["mismatched_robots_max_over_ranks"] = int(bad)
        par["bitexact"] = bad == 0
    out["parity_sampled"] = par
    eng.close()
    del prepared, planes, krec, many_in
    if not args.no_secondary and world == 1:  # single-GPU configs: one line at N=1
        torch.cuda.empty_cache()
        out["secondary"] = secondary_configs(dev, stream, args.secondary_ticks, trig)
        out["path_rows"] = path_rows(dev, stream, -(-max(args.secondary_ticks, 20) // 10) * 10, trig)
    # the CPU baseline on rank 0 after every timed region (at N > 1 the other ranks wait at
    # the final barrier): the same KF6 tick on a bounded 2^18-robot sample
    if rank == 0 and not args.no_cpu_baseline:
        import numpy as np
        y = np.ascontiguousarray(yaw[:8, : 1 << 18].cpu().numpy())
        g = np.ascontiguousarray(gz[:8, : 1 << 18].cpu().numpy())
        r = np.ascontiguousarray(rpm[:8, : 1 << 18].cpu().numpy())
        cb = cpu_baseline(y, g, r, args.cpu_sample_s)
        cb["gpu_over_cpu"] = value / cb["value"]  # the driver-timed value, not the kernel time
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
