"""mignn -- MI355X-native (gfx950) GNN message-passing engine behind the
Caesar3142/GNN-BFS-RANS `FlowGNN.forward` API.

The compute lives in `libmignn.so` (HIP kernels, C ABI in include/mignn.h);
this package mirrors the reference's Python surface on top of it.
"""

from .data import Batch, Data  # noqa: F401
from .gnn_model import FlowGNN, FlowGNNSurrogate  # noqa: F401

__all__ = ["FlowGNN", "FlowGNNSurrogate", "Data", "Batch"]
