"""Drop-in module: `from openfoam_loader import OpenFOAMLoader` resolves to the
native reader when `gnn-bfs-rans_amd/` is on sys.path ahead of the reference
(reference module: openfoam_loader.py)."""

from mignn.openfoam_loader import OpenFOAMLoader  # noqa: F401
