"""The native multi-GPU ensemble path (fmskf_comm_init / fmskf_ensemble_stats): an RCCL
communicator owned by the handle.  One GPU on the test box -> world size 1: the record goes
through ncclAllGather on the handle's stream and must fold to exactly what the host combine
of the device partial gives; without a communicator the same call covers this handle alone.
(N > 1 is exercised by bench.py under torch.distributed at round end.)"""
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
        e.comm_init(uid, 0, 1)
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
