"""Minimal graph containers with the `torch_geometric.data` surface the
reference scripts use (graph_constructor.py:262-267, train.py:9, :155):
`Data(x, edge_index, edge_attr, y, num_nodes)`, attribute access,
`.to(device)`, `num_nodes` / `num_edges`, and `Batch.from_data_list`
(node-offset concatenation + `batch` vector).  PyG is not available on the
MI355X boxes, so the engine ships its own.
"""

from __future__ import annotations

from typing import List, Optional

import torch


class Data:
    def __init__(self, x: Optional[torch.Tensor] = None, edge_index: Optional[torch.Tensor] = None,
                 edge_attr: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None,
                 num_nodes: Optional[int] = None, **kwargs):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.y = y
        self._num_nodes = num_nodes
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        if self._num_nodes is not None:
            return int(self._num_nodes)
        if self.x is not None:
            return int(self.x.shape[0])
        if self.edge_index is not None and self.edge_index.numel() > 0:
            return int(self.edge_index.max()) + 1
        return 0

    @num_nodes.setter
    def num_nodes(self, n):
        self._num_nodes = n

    @property
    def num_edges(self) -> int:
        return 0 if self.edge_index is None else int(self.edge_index.shape[1])

    def keys(self) -> List[str]:
        return [k for k, v in self.__dict__.items() if not k.startswith("_") and v is not None]

    def __getitem__(self, key):
        return getattr(self, key)

    def to(self, device, non_blocking: bool = False) -> "Data":
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            out.__dict__[k] = v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v
        return out

    def __repr__(self) -> str:
        parts = []
        for k in self.keys():
            v = getattr(self, k)
            parts.append(f"{k}={list(v.shape)}" if torch.is_tensor(v) else f"{k}={v}")
        return f"{self.__class__.__name__}({', '.join(parts)})"


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list: List[Data]) -> "Batch":
        xs, eis, eas, ys, bs = [], [], [], [], []
        offset = 0
        for i, d in enumerate(data_list):
            n = d.num_nodes
            if d.x is not None:
                xs.append(d.x)
            if d.edge_index is not None:
                eis.append(d.edge_index + offset)
            if d.edge_attr is not None:
                eas.append(d.edge_attr)
            if d.y is not None:
                ys.append(d.y)
            bs.append(torch.full((n,), i, dtype=torch.long))
            offset += n
        cat = lambda ts: torch.cat(ts, 0) if ts else None  # noqa: E731
        b = cls(x=cat(xs), edge_index=torch.cat(eis, 1) if eis else None, edge_attr=cat(eas),
                y=cat(ys), num_nodes=offset)
        b.batch = torch.cat(bs) if bs else None
        b.num_graphs = len(data_list)
        return b
