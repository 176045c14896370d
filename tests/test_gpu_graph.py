"""A per-tick call sequence captured into a HIP graph (fmskf_graph_*) replays bit-identically
to the same calls made one by one; the graph reads whatever the fixed input buffers hold at
replay time, like the firmware's ISR reading the latest sensor values."""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu


def test_graph_replay_matches_direct_calls():
    import torch
    n, T = 4099, 30
    tr = Trajectory(n, T, seed=71)
    yaw, gz, rpm = tr.kf6_inputs()
    st = torch.cuda.Stream()
    vel = np.zeros((3, n), np.float32)
    vel[0] = 150.0
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    with torch.cuda.stream(st), Engine("kf6", n) as a, Engine("kf6", n) as b:
        for e in (a, b):
            e.set_stream(st)
            e.set_power(None)
            e.set_target_vel(vel, acl, jrk)
        dy = torch.empty(n, dtype=torch.float32, device="cuda")
        dg = torch.empty(n, dtype=torch.float32, device="cuda")
        dr = torch.empty((n, 4), dtype=torch.int16, device="cuda")
        fa = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
        fb = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
        # capture: estimator tick + wheel loops + 0x200 frames, all device pointers
        b.graph_begin()
        b.tick(yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
        b.control(dr)
        b.can_tx(fb)
        b.graph_end()
        for t in range(T):
            dy.copy_(torch.from_numpy(yaw[t]))
            dg.copy_(torch.from_numpy(gz[t]))
            dr.copy_(torch.from_numpy(rpm[t]))
            a.tick(yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
            a.control(dr)
            a.can_tx(fa)
            b.graph_launch(1)
        st.synchronize()
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32))
        np.testing.assert_array_equal(Pa.view(np.uint32), Pb.view(np.uint32))
        np.testing.assert_array_equal(a.get_ctrl()["curr"], b.get_ctrl()["curr"])
        assert torch.equal(fa, fb)


@pytest.mark.parametrize("n", [4099, 65536])
def test_graph_isr_tick_kf6_fused(n):
    """KF6 fmskf_isr_tick (the fused one-kernel ISR, k_isr_kf6) captured with device input
    planes and a device frame buffer: each replay equals a direct isr_tick and the three-call
    tick + control + can_tx sequence, state and frames bit for bit."""
    import torch
    T = 16
    tr = Trajectory(n, T, seed=73)
    yaw, gz, rpm = tr.kf6_inputs()
    st = torch.cuda.Stream()
    vel = np.zeros((3, n), np.float32)
    vel[2] = 0.8
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    with torch.cuda.stream(st), Engine("kf6", n) as a, Engine("kf6", n) as b, Engine("kf6", n) as c:
        for e in (a, b, c):
            e.set_stream(st)
            e.set_power(None)
            e.set_target_vel(vel, acl, jrk)
        dy = torch.empty(n, dtype=torch.float32, device="cuda")
        dg = torch.empty(n, dtype=torch.float32, device="cuda")
        dr = torch.empty((n, 4), dtype=torch.int16, device="cuda")
        fa, fb, fc = (torch.empty((n, 8), dtype=torch.uint8, device="cuda") for _ in range(3))
        b.graph_begin()
        b.isr_tick(out=fb, yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
        b.graph_end()
        for t in range(T):
            dy.copy_(torch.from_numpy(yaw[t]))
            dg.copy_(torch.from_numpy(gz[t]))
            dr.copy_(torch.from_numpy(rpm[t]))
            a.tick(yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
            a.control(dr)
            a.can_tx(fa)
            b.graph_launch(1)
            c.isr_tick(out=fc, yaw_deg=dy, gyro_z_dps=dg, rpm=dr)
            st.synchronize()
            assert torch.equal(fa, fb), f"tick {t}: graph frames"
            assert torch.equal(fa, fc), f"tick {t}: direct isr frames"
        xa, Pa = a.get_state()
        for e in (b, c):
            x, P = e.get_state()
            np.testing.assert_array_equal(xa.view(np.uint32), x.view(np.uint32))
            np.testing.assert_array_equal(Pa.view(np.uint32), P.view(np.uint32))
            np.testing.assert_array_equal(a.get_ctrl()["curr"], e.get_ctrl()["curr"])


def test_graph_isr_tick_can_kf6():
    """fmskf_isr_tick_can (the tick's CAN RX fused into the KF6 ISR) captured with device CAN
    buffers, input planes and frame buffer: each replay equals direct ingest_can + isr_tick,
    frames, state and the motor state bit for bit."""
    import torch
    n, T = 4099, 12
    tr = Trajectory(n, T, seed=79)
    yaw, gz, _ = tr.kf6_inputs()
    st = torch.cuda.Stream()
    vel = np.zeros((3, n), np.float32)
    vel[0] = 150.0
    acl = np.full((3, n), 1000.0, np.float32)
    jrk = np.full((3, n), 10000.0, np.float32)
    with torch.cuda.stream(st), Engine("kf6", n) as a, Engine("kf6", n) as b:
        for e in (a, b):
            e.set_stream(st)
            e.set_power(None)
            e.set_target_vel(vel, acl, jrk)
        dy = torch.empty(n, dtype=torch.float32, device="cuda")
        dg = torch.empty(n, dtype=torch.float32, device="cuda")
        df = torch.empty((n, 4, 8), dtype=torch.uint8, device="cuda")
        ds = torch.empty((n, 4), dtype=torch.int16, device="cuda")
        fa, fb = (torch.empty((n, 8), dtype=torch.uint8, device="cuda") for _ in range(2))
        b.graph_begin()
        b.isr_tick_can(df, ds, out=fb, yaw_deg=dy, gyro_z_dps=dg)
        b.graph_end()
        for t in range(T):
            f, s = tr.can_frames(t)
            df.copy_(torch.from_numpy(np.ascontiguousarray(f)))
            ds.copy_(torch.from_numpy(np.ascontiguousarray(s)))
            dy.copy_(torch.from_numpy(yaw[t]))
            dg.copy_(torch.from_numpy(gz[t]))
            a.ingest_can(df, ds)
            a.isr_tick(out=fa, yaw_deg=dy, gyro_z_dps=dg)
            b.graph_launch(1)
            st.synchronize()
            assert torch.equal(fa, fb), f"tick {t}: graph frames"
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32))
        np.testing.assert_array_equal(Pa.view(np.uint32), Pb.view(np.uint32))
        ma, mb = a.get_motors(), b.get_motors()
        for k in ma:
            np.testing.assert_array_equal(ma[k], mb[k], err_msg=k)
        # the Status fields, incl. the stamps and dlt from the two history slots (round 6: each
        # replay of the one-call graph starts from the order the capture began with)
        sa, sb = a.get_motor_status(), b.get_motor_status()
        for k in sa:
            np.testing.assert_array_equal(np.asarray(sa[k]).view(np.uint8), np.asarray(sb[k]).view(np.uint8), err_msg=k)


def test_graph_errors():
    with Engine("kf6", 64) as e:
        with pytest.raises(fmskf.FmskfError):
            e.graph_begin()            # null stream: capture refused
        with pytest.raises(fmskf.FmskfError):
            e.graph_launch(1)          # nothing captured


@pytest.mark.parametrize("model", ["kf6", "ekf9"])
def test_graph_captures_tick_ensemble(model):
    """fmskf_tick_ensemble captured as the first record of a fresh handle: the shift vector is
    taken by fmskf_graph_begin before the capture (a launch inside a capture would only be
    recorded), so every replay's record equals the record of the same call made directly."""
    import torch
    n, T = 5003, 4
    tr = Trajectory(n, T, seed=74)
    st = torch.cuda.Stream()
    if model == "kf6":
        yaw, gz, rpm = tr.kf6_inputs()
        src = [dict(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t]) for t in range(T)]
    else:
        raw = tr.ekf9_raw()
        src = [dict(raw=raw[t]) for t in range(T)]
    with torch.cuda.stream(st), Engine(model, n) as a, Engine(model, n) as b:
        for e in (a, b):
            e.set_stream(st)
        dev = {k: torch.empty(v.shape, dtype=getattr(torch, str(v.dtype)), device="cuda")
               for k, v in src[0].items()}
        rb = torch.empty(b.ensemble_record_len(), dtype=torch.float64, device="cuda")
        b.graph_begin()
        b.tick_ensemble(out=rb, **dev)
        b.graph_end()
        for t in range(T):
            for k, v in src[t].items():
                dev[k].copy_(torch.from_numpy(v))
            ra = a.tick_ensemble(**dev)
            b.graph_launch()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(ra, rb.cpu().numpy())
        xa, _ = a.get_state()
        xb, _ = b.get_state()
    np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32))


def test_async_ensemble_pending_across_capture():
    """A pending asynchronous result whose fold has not been queued yet (the newest event) stays
    pending across a capture: plain ticks captured in the graph do not fold it (the replay would
    fold whatever the slot holds then), fmskf_ensemble_end refuses inside the capture, and after
    it the result equals the synchronous record of the same state, bit for bit."""
    import torch
    n, T = 4099, 3
    tr = Trajectory(n, T, seed=75)
    yaw, gz, rpm = tr.kf6_inputs()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st), Engine("kf6", n) as a, Engine("kf6", n) as b:
        for e in (a, b):
            e.set_stream(st)
        want = fmskf.ensemble_combine(6, a.tick_ensemble(yaw_deg=yaw[0], gyro_z_dps=gz[0], rpm=rpm[0])[None, :])
        b.tick_ensemble_begin(yaw_deg=yaw[0], gyro_z_dps=gz[0], rpm=rpm[0])
        dev = [torch.from_numpy(np.ascontiguousarray(v[1])).cuda() for v in (yaw, gz, rpm)]
        torch.cuda.synchronize()
        b.graph_begin()
        b.tick(yaw_deg=dev[0], gyro_z_dps=dev[1], rpm=dev[2])
        with pytest.raises(fmskf.FmskfError):
            b.ensemble_end()                      # the newest fold would be captured, not run
        b.graph_end()
        got = b.ensemble_end()
        b.graph_launch()
        a.tick(yaw_deg=yaw[1], gyro_z_dps=gz[1], rpm=rpm[1])
        torch.cuda.synchronize()
        xa, _ = a.get_state()
        xb, _ = b.get_state()
    np.testing.assert_array_equal(want[0], got[0])
    np.testing.assert_array_equal(want[1], got[1])
    np.testing.assert_array_equal(xa.view(np.uint32), xb.view(np.uint32))
