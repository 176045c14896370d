"""One rank of tests/test_gpu_rccl_multirank.py: a handle with its own communicator (libfmskf's
fmskf_comm_init, over the loopback RCCL stand-in named by FMSKF_RCCL_LIBRARY, so several ranks
share the test box's one GPU), ticking its own shard of the fleet.  No torch: the process loads
libfmskf and, through it, the stand-in, never torch's RCCL.

    rccl_rank_worker.py MODEL RANK WORLD N T EVERY ID_FILE OUT.npz

Writes every asynchronous result (fmskf_tick_ensemble_begin / fmskf_ensemble_end), the local
record of the same tick from a twin handle without a communicator (fmskf_tick_ensemble), the
synchronous fmskf_ensemble_stats and a stand-alone fmskf_ensemble_begin / end at the end."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "roboken-fmskf-robot-controller_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fmskf  # noqa: E402
from fmskf import Engine  # noqa: E402
from test_gpu_rccl import _ens_inputs  # noqa: E402


def main():
    model, rank, world, n, T, every, id_file, out = sys.argv[1:9]
    rank, world, n, T, every = int(rank), int(world), int(n), int(T), int(every)
    if rank == 0:
        uid = fmskf.comm_unique_id()
        with open(id_file + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(id_file + ".tmp", id_file)
    else:
        t_end = time.time() + 60
        while not os.path.exists(id_file):
            if time.time() > t_end:
                raise SystemExit("no communicator id from rank 0")
            time.sleep(0.05)
        with open(id_file, "rb") as f:
            uid = f.read()
    kw = _ens_inputs(model, n, T, seed=100 + rank)
    local, got = [], []
    with Engine(model, n) as a, Engine(model, n) as b:
        b.comm_init(uid, rank, world)
        info = b.comm_info()  # (world, rank) as the communicator itself reports them
        counts, xms = [], []
        pending = 0
        for t in range(T):
            if (t + 1) % every == 0:
                local.append(a.tick_ensemble(**kw(t)))
                b.tick_ensemble_begin(**kw(t))
                pending += 1
                if pending == 3:
                    m_, c_, cnt, nrec = b.ensemble_end_count()
                    got.append((m_, c_))
                    counts.append((cnt, nrec))
                    xms.append(b.ensemble_exchange_ms())
                    pending -= 1
            else:
                a.tick(**kw(t))
                b.tick(**kw(t))
        while pending:
            m_, c_, cnt, nrec = b.ensemble_end_count()
            got.append((m_, c_))
            counts.append((cnt, nrec))
            xms.append(b.ensemble_exchange_ms())
            pending -= 1
        ms, cs = b.ensemble_stats()              # synchronous: partial, ncclAllGather, fold
        b.ensemble_begin()                       # asynchronous stand-alone record
        ma, ca = b.ensemble_end()
        final = a.ensemble_partial()
        xa, _ = a.get_state()
        xb, _ = b.get_state()
    np.savez(out, local=np.stack(local), got_mean=np.stack([g[0] for g in got]),
             got_cov=np.stack([g[1] for g in got]), sync_mean=ms, sync_cov=cs, alone_mean=ma,
             alone_cov=ca, final=final, comm_info=np.array(info), counts=np.array(counts), exchange_ms=np.array(xms),
             rccl_library=np.array(fmskf.rccl_library()), same_state=np.array(np.array_equal(xa.view(np.uint8), xb.view(np.uint8))))


if __name__ == "__main__":
    main()
