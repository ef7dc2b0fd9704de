"""Generate tests/golden/foam_case.npz: the bytes of the reference's OpenFOAM
case files (data, not source) that the reader tests parse -- the polyMesh
(points, faces, owner, neighbour, boundary) and the fields of time 282 --
stored as compressed uint8 arrays under "<relative path>".  The expected
parse results are the reference loader's outputs already held in mesh.npz
(make_mesh_fixture.py).  Runs only in the build container (/root/reference).

Usage:  python tests/golden/make_foam_fixture.py
"""

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CASE = "/root/reference/OpenFOAM-data"
FILES = [f"constant/polyMesh/{n}" for n in ("points", "faces", "owner", "neighbour", "boundary")]
FILES += [f"282/{n}" for n in ("U", "p", "k", "epsilon", "nut")]


def main():
    out = {}
    for rel in FILES:
        with open(os.path.join(CASE, rel), "rb") as f:
            out[rel] = np.frombuffer(f.read(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "foam_case.npz"), **out)


if __name__ == "__main__":
    main()
