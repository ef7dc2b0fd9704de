"""Drop-in module: `from normalization import FieldNormalizer` resolves to the
device float64 normaliser when `gnn-bfs-rans_amd/` is on sys.path ahead of the
reference (reference module: normalization.py)."""

from mignn.normalization import FieldNormalizer, WeightedMSELoss  # noqa: F401
