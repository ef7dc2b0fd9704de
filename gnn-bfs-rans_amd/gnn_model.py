"""Drop-in module: `from gnn_model import FlowGNN, FlowGNNSurrogate` resolves
to the MI355X engine when `gnn-bfs-rans_amd/` is on sys.path ahead of the
reference (reference module: gnn_model.py)."""

from mignn.gnn_model import FlowGNN, FlowGNNSurrogate  # noqa: F401
