import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "roboken-fmskf-robot-controller_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden_wt901():
    d = np.load(os.path.join(ROOT, "tests", "golden", "wt901_ref.npz"))
    return {k: d[k] for k in d.files}


def iter_golden_streams(g):
    """Yield (read_reg_index, kind, polls[list of bytes], regs [P,144], cbs [P][list])."""
    off_b = 0
    off_p = 0
    off_cb = 0
    for s, np_ in enumerate(g["n_polls"]):
        polls, regs, cbs = [], [], []
        for k in range(int(np_)):
            L = int(g["poll_len"][off_p])
            polls.append(bytes(g["bytes"][off_b:off_b + L]))
            off_b += L
            regs.append(g["regs"][off_p])
            c = int(g["cb_count"][off_p])
            cbs.append(list(zip(g["cb_reg"][off_cb:off_cb + c].tolist(),
                                g["cb_num"][off_cb:off_cb + c].tolist())))
            off_cb += c
            off_p += 1
        yield int(g["read_reg_index"][s]), str(g["kind"][s]), polls, np.stack(regs), cbs
