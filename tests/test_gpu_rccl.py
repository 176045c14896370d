"""The native multi-GPU ensemble path (fmskf_comm_init / fmskf_ensemble_stats): an RCCL
communicator owned by the handle.  One GPU on the test box -> world size 1: the record goes
through ncclAllGather on the handle's stream and must fold to exactly what the host combine
of the device partial gives; without a communicator the same call covers this handle alone.
(World > 1 on one GPU: tests/test_gpu_rccl_multirank.py, through the loopback stand-in; RCCL
itself at N > 1: bench.py on the driver's node.)"""
import numpy as np
import pytest

import fmskf
from fmskf import Engine
from fmskf.synth import Trajectory

pytestmark = pytest.mark.gpu


def test_ensemble_stats_over_rccl_world1(orc):
    n, T = 50_001, 10
    tr = Trajectory(n, T, seed=61)
    yaw, gz, rpm = tr.kf6_inputs()
    with Engine("kf6", n) as e:
        for t in range(T):
            e.tick(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
        m0, c0 = e.ensemble_stats()                    # no communicator: this handle
        uid = fmskf.comm_unique_id()
        assert len(uid) == 128
        with pytest.raises(fmskf.FmskfError):
            e.comm_info()                              # no communicator yet
        e.comm_init(uid, 0, 1)
        assert e.comm_info() == (1, 0)                 # ncclCommCount / ncclCommUserRank
        assert "librccl" in fmskf.rccl_library()       # the real RCCL, not a stand-in
        m1, c1 = e.ensemble_stats()                    # through ncclAllGather
        rec = e.ensemble_partial()
        x, _ = e.get_state()
    mh, ch = fmskf.ensemble_combine(6, rec[None, :])
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(m1, mh)
    np.testing.assert_array_equal(c1, ch)
    # against the oracle's two-pass moments of the same state
    mo, co = orc.ens_finalize(6, orc.ens_partial(x))
    np.testing.assert_allclose(m1, mo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(c1, co, rtol=1e-9, atol=1e-15)


def test_comm_init_rejects_bad_rank():
    with Engine("kf6", 16) as e:
        with pytest.raises(fmskf.FmskfError):
            e.comm_init(b"\0" * 128, 2, 2)


@pytest.mark.parametrize("model", ["kf6", "ekf9", "kf12d"])
def test_sharded_handles_fold_to_the_whole_fleet(model):
    """Weak-scaling shards in one process: the fleet split over three handles (one per GPU in
    a multi-GPU process; here all on device 0), each handle's ensemble record, folded with
    fmskf_ensemble_combine in shard order, equals the statistics of one handle holding every
    robot (1e-12 relative) and of numpy on the same states."""
    import fmskf
    from fmskf import Engine
    rng = np.random.default_rng(11)
    sizes = [1000, 257, 4096]
    n = sum(sizes)
    with Engine(model, n) as whole:
        x = (rng.normal(size=(whole.nx, n)) * 0.5 + 2.0).astype(whole.dtype)
        whole.set_state(x, None)
        mw, cw = fmskf.ensemble_combine(whole.nx, whole.ensemble_partial()[None, :])
    recs, lo = [], 0
    for sz in sizes:
        with Engine(model, sz) as e:
            e.set_state(np.ascontiguousarray(x[:, lo:lo + sz]), None)
            recs.append(e.ensemble_partial())
        lo += sz
    ms, cs = fmskf.ensemble_combine(x.shape[0], np.stack(recs))
    np.testing.assert_allclose(ms, mw, rtol=1e-12)
    np.testing.assert_allclose(cs, cw, rtol=1e-10, atol=1e-14)
    ref = np.cov(x.astype(np.float64))
    packed = np.array([ref[i, j] for i in range(x.shape[0]) for j in range(i + 1)])
    np.testing.assert_allclose(cs, packed, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(ms, x.astype(np.float64).mean(axis=1), rtol=1e-12)


def _ens_inputs(model, n, T, seed):
    tr = Trajectory(n, T, seed=seed)
    if model == "kf6":
        yaw, gz, rpm = tr.kf6_inputs()
        return lambda t: dict(yaw_deg=yaw[t], gyro_z_dps=gz[t], rpm=rpm[t])
    if model == "ekf9":
        raw = tr.ekf9_raw()
        return lambda t: dict(raw=raw[t])
    if model == "kf12d":
        z = tr.kf12d_z()
        return lambda t: dict(z=np.ascontiguousarray(z[t]))
    ryaw, sums, rrpm = tr.rs_inputs()
    return lambda t: dict(yaw_deg=ryaw[t], angle_sum=np.ascontiguousarray(sums[t]), rpm=rrpm[t])


@pytest.mark.parametrize("model,n,every,comm", [("kf6", 70001, 1, True), ("kf6", 1 << 20, 3, False),
                                                ("kf6", (1 << 21) + 200_000, 1, False),
                                                ("ekf9", (1 << 21) + 100_000, 1, False),
                                                ("ekf9", 5001, 2, True), ("kf12d", 3001, 1, False),
                                                ("rs", 4097, 1, True)])
def test_async_ensemble_matches_sync(model, n, every, comm):
    """fmskf_tick_ensemble_begin / fmskf_ensemble_end (event k's fold carried by extra blocks at
    the front of event k + 1's tick grid -- including the 8974-record KF6 and 8583-record EKF9
    folds of the one-robot-per-lane kernels past the Infinity Cache -- or stand-alone: ahead of
    a plain tick, for the last event and for the non-fused RS record; the all-gather and
    copy-out on the side stream; results collected two events late, so three are
    pending at every begin with every = 1) against the synchronous fmskf_tick_ensemble of a twin
    handle on the same inputs: the states stay bit-identical and every (mean, cov) equals the
    fold of the synchronous record bit for bit, with and without a (world-1) RCCL communicator
    (which exchanges nothing: its result takes the one-GPU path)."""
    T = 9
    kw = _ens_inputs(model, n, T, seed=63)
    with Engine(model, n) as a, Engine(model, n) as b:
        if comm:
            b.comm_init(fmskf.comm_unique_id(), 0, 1)
        want, got, pending = [], [], 0
        for t in range(T):
            if (t + 1) % every == 0:
                want.append(fmskf.ensemble_combine(a.nx, a.tick_ensemble(**kw(t))[None, :]))
                b.tick_ensemble_begin(**kw(t))
                pending += 1
                if pending == 3:
                    got.append(b.ensemble_end())
                    pending -= 1
            else:
                a.tick(**kw(t))
                b.tick(**kw(t))
        while pending:
            got.append(b.ensemble_end())
            pending -= 1
        # the side stream's all-gather + copy-out time of the last collected result: -1 without
        # a communicator and with a world-1 one (round 6: a one-rank all-gather is the identity, so
        # the fold writes the pinned slot itself; world > 1: tests/test_gpu_rccl_multirank.py)
        xms = b.ensemble_exchange_ms()
        assert xms == -1.0, xms
        with pytest.raises(fmskf.FmskfError):
            b.ensemble_end()                               # nothing pending
        xa, Pa = a.get_state()
        xb, Pb = b.get_state()
        # the stand-alone asynchronous record of the current state (no tick)
        b.ensemble_begin()
        ms, cs = b.ensemble_end()
        mp, cp = fmskf.ensemble_combine(b.nx, b.ensemble_partial()[None, :])
    np.testing.assert_array_equal(xa.view(np.uint8), xb.view(np.uint8))
    if Pa is not None:
        np.testing.assert_array_equal(Pa.view(np.uint8), Pb.view(np.uint8))
    assert len(got) == len(want) == T // every
    for (mw, cw), (mg, cg) in zip(want, got):
        np.testing.assert_array_equal(mw, mg)
        np.testing.assert_array_equal(cw, cg)
    np.testing.assert_array_equal(ms, mp)
    np.testing.assert_array_equal(cs, cp)


def test_async_ensemble_limits():
    with Engine("kf6", 1000) as e:
        for _ in range(4):
            e.ensemble_begin()
        with pytest.raises(fmskf.FmskfError):
            e.ensemble_begin()                              # a fifth pending begin
        for _ in range(4):
            e.ensemble_end()
        e.ensemble_begin()                                  # the slots are reusable
        m, c = e.ensemble_end()
    assert np.all(m == 0.0) and np.all(c == 0.0)            # zero state: zero moments


def test_async_ensemble_across_reset():
    """Results begun before a reset fold with the shift of the state they recorded: retaking
    the shift first queues the pending fold (stream-ordered ahead of the rewrite), so the
    pending result and the next one both equal the synchronous records of the same states."""
    n = 3001
    rng = np.random.default_rng(8)
    with Engine("ekf9", n) as a, Engine("ekf9", n) as b:
        x1 = (rng.normal(size=(9, n)) + 2.0).astype(np.float32)
        for e in (a, b):
            e.set_state(x1, None)
        b.ensemble_begin()
        want1 = fmskf.ensemble_combine(9, a.ensemble_partial()[None, :])
        x2 = (rng.normal(size=(9, n)) * 3.0 - 1.0).astype(np.float32)
        for e in (a, b):
            e.reset()
            e.set_state(x2, None)
        b.ensemble_begin()
        want2 = fmskf.ensemble_combine(9, a.ensemble_partial()[None, :])
        got1, got2 = b.ensemble_end(), b.ensemble_end()
    for w, g in ((want1, got1), (want2, got2)):
        np.testing.assert_array_equal(w[0], g[0])
        np.testing.assert_array_equal(w[1], g[1])
