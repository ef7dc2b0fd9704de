"""Drop-in module: `from graph_constructor import GraphConstructor` resolves to
the device mesh -> graph builder when `gnn-bfs-rans_amd/` is on sys.path ahead
of the reference (reference module: graph_constructor.py)."""

from mignn.graph import GraphConstructor  # noqa: F401
