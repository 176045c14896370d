"""fmskf -- MI355X-native batched IMU + mecanum-odometry state estimation.

Host-side mirror of the C ABI in include/fmskf.h (libfmskf.so, HIP kernels for
gfx950).  See DESIGN.md for the hot path, its boundary and the data layout.
"""
from ._lib import (ABI_VERSION, CFG_COMP_POS, MEM_DEVICE, MEM_HOST, MODEL_EKF9, MODEL_KF6, MODEL_KF12D,
                   MODEL_RS, TRIG_LIBM, TRIG_TABLE512, FmskfError, load)
from .engine import (KF6_RECORD_DTYPE, Engine, comm_unique_id, default_config, ensemble_combine,
                     kf6_records, rccl_library, shard_span)

__all__ = ["Engine", "default_config", "ensemble_combine", "FmskfError", "load", "ABI_VERSION",
           "MEM_HOST", "MEM_DEVICE", "MODEL_RS", "MODEL_KF6", "MODEL_EKF9", "MODEL_KF12D",
           "TRIG_TABLE512", "TRIG_LIBM", "KF6_RECORD_DTYPE", "kf6_records", "shard_span",
           "CFG_COMP_POS", "rccl_library"]
