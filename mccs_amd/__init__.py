"""mccs_amd — MI355X-native allreduce reduction path of mCCS.

Layers:
  include/mccs_devcomm.h   layout-identical device ABI (reference devcomm.h)
  include/mccs_hip.h       C-ABI of libmccs_hip.so
  mccs_amd/csrc/           gfx950 HIP kernels + C++ host runtime
  mccs_amd/*.py            ctypes face mirroring libmccs (src/libmccs)
"""
from ._lib import DataType, MccsError, RedOp, load  # noqa: F401
from .reduce import get_tune, reduce, reduce_copy, tune, tune_grid  # noqa: F401

__version__ = "0.1.0"
