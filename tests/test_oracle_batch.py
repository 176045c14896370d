"""The oracle's batched IMU and CAN ingest (orc_wt901_update_batch, orc_can_ingest_batch: the
per-instance restatements in a C loop) equal the per-instance oracle objects on the same
traffic, and fmskf.synth's vectorised poll rows equal its per-robot poll bytes.  The fleet-size
long-horizon GPU test (tests/test_gpu_long.py) relies on both."""
import numpy as np

from fmskf.synth import Trajectory


def test_poll_rows_equal_poll_bytes():
    tr = Trajectory(53, 21, seed=8)
    for t in (0, 10, 20):
        rows, lens = tr.wt901_poll_rows(t)
        assert rows.shape == (53, 48) and (lens == 44).all()
        for i in range(53):
            b = np.frombuffer(tr.wt901_poll_bytes(t, i), np.uint8)
            np.testing.assert_array_equal(rows[i, :44], b)
            assert not rows[i, 44:].any()


def test_batched_ingest_equals_instances(orc):
    n, T = 41, 40
    tr = Trajectory(n, T, seed=9)
    wb, mb = orc.Wt901Batch(n), orc.MotorBatch(n)
    imus = [orc.Wt901(0x51) for _ in range(n)]
    mot = [[orc.M2006(d) for d in (1, 1, -1, -1)] for _ in range(n)]
    rng = np.random.default_rng(3)
    for t in range(T):
        fr, st = tr.can_frames(t)
        fr = fr.copy()
        fr[rng.random((n, 4)) < 0.1] ^= 0x5A          # corrupted payloads
        mb.rx(fr, st)
        for i in range(n):
            for w in range(4):
                mot[i][w].rx(fr[i, w], int(st[i, w]))
        if t % 10 == 0:
            rows, lens = tr.wt901_poll_rows(t)
            rows[::7, 13] ^= 0xFF                      # a bad checksum in some polls
            lens[::5] = 30                             # torn polls
            wb.update(rows, lens, latch_qinit=(t == 0))
            for i in range(n):
                imus[i].update(rows[i, :lens[i]], latch_qinit=(t == 0))
    np.testing.assert_array_equal(wb.data.view(np.uint32), np.stack([m.data for m in imus], 1).view(np.uint32))
    np.testing.assert_array_equal(wb.is_error, np.array([m.is_error for m in imus], np.uint8))
    for f in ("angle_sum", "rpm", "curr", "micro", "angle", "head", "speed_radps", "iir_prev_y"):
        got = mb.field(f)
        want = np.array([[getattr(mot[i][w].s, f) for w in range(4)] for i in range(n)]).astype(got.dtype)
        np.testing.assert_array_equal(got, want, err_msg=f)
