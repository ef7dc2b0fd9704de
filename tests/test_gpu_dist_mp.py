"""The multi-process shard route: FlowGNNShard through
DistExchange in separate processes -- k-slab ranges, column order, the window
GCN kernel, layer 1 from layer 0's row codes with the ghost codes in the
halo -- against the unsharded forward on the same mesh.  The ranks share
cuda:0 of a one-GPU box under gloo (tests/mp_shard_worker.py); the in-process
shard tests (test_gpu_dist.py) cover the same layers through LocalExchange."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, **env):
    port = str(_free_port())
    procs = []
    for r in range(world):
        e = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port, HSA_ENABLE_IPC_MODE_LEGACY="0",
                 **{k: str(v) for k, v in env.items()})
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_shard_worker.py")],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, err = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, err))
    for rc, o, err in outs:
        assert rc == 0, f"rank exited {rc}: {err[-2000:]}"
    line = [ln for ln in outs[0][1].splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


@pytest.mark.parametrize("world,H", [(2, 128), (3, 128), (2, 64)])
def test_multiprocess_shards_match_unsharded(world, H):
    r = _run(world, MP_GRID="48,40,12", MP_H=H, MP_LAYERS=4, MP_TYPE="GCN")
    print(r)
    assert r["route"]["window"], r
    assert r["route"]["codes"] == (H == 128), r
    assert all(g == 2 * 48 * 40 for g in r["n_ghost"]), r       # k-slabs: two halo planes
    assert r["device_errors"] == [0] * world
    assert not any(r["nondeterministic"])
    for e, s in zip(r["max_err"], r["scale"]):
        assert e <= 2e-6 * s, r
