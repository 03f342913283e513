"""fedtree_amd -- MI355X-native batch Paillier engine behind FedTree's HE interface.

The compute path is libfthe.so (hand-scheduled gfx950 Montgomery kernels +
HIP glue kernels, C ABI in include/fthe.h).  This package is the host-side
mirror of the reference's operator interface (Paillier / Paillier_GPU,
GHPair, Server/Party HE methods); see fedtree_amd/paillier.py.
"""
from ._lib import FtheError, LIB_PATH, load  # noqa: F401

__all__ = ["FtheError", "LIB_PATH", "load", "paillier"]


def __getattr__(name):
    if name == "paillier":
        from . import paillier
        return paillier
    raise AttributeError(name)
