"""Writes a small synthetic vessel data set in the format get_vessels reads
(setupGeometry.f90:585-627): res/edges.dat (two 1-based node indices per line),
res/nodes.dat (x y z per line, in the reference's 10-um units: it multiplies by res = 0.001 cm)
and res/radii.dat (one radius per node, same units), plus vessels.toml beside them.

The reference does not ship these files, so the data are build-defined:
a random tree over a 320 x 180 x 260 unit box (the .32 x .18 x .26 cm dermis box of :650),
radii 0.5-3 units (5-30 um). The text mixes the list-directed forms a Fortran `read(u, *)`
accepts (blank and comma separators, a `d` exponent, a value on the next line), so the C++
front end's reader is checked against the Fortran runtime's (tests/test_fortran_binding.py).

    python tests/golden/make_vessel_data.py OUTDIR [N_NODES] [SEED] [--extra-edges K]
"""
from __future__ import annotations

import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def vessel_tree(n_nodes: int = 40, seed: int = 7, extra_edges: int = 0):
    """(edges (E, 2) 1-based, nodes (N, 3), radii (N,)): a random tree (E = N - 1) grown from a
    root, plus `extra_edges` edges between random nodes (so E >= N and every node is read)."""
    rng = np.random.Generator(np.random.Philox(seed))
    ext = np.array([320.0, 180.0, 260.0])
    nodes = [rng.uniform(0.2 * ext, 0.8 * ext)]
    edges = []
    for i in range(1, n_nodes):
        parent = int(rng.integers(0, i))
        step = rng.normal(size=3)
        step = step / np.linalg.norm(step) * rng.uniform(8.0, 40.0)
        nodes.append(np.clip(nodes[parent] + step, 1.0, ext - 1.0))
        edges.append((parent + 1, i + 1))
    for _ in range(extra_edges):
        a, b = rng.integers(1, n_nodes + 1, size=2)
        edges.append((int(a), int(b)))
    nodes = np.round(np.array(nodes), 3)
    radii = np.round(rng.uniform(0.5, 3.0, size=n_nodes), 4)
    return np.array(edges, dtype=np.int64), nodes, radii


def write_vessel_data(outdir, n_nodes: int = 40, seed: int = 7, extra_edges: int = 0, toml: bool = True):
    """Write edges.dat, nodes.dat, radii.dat (and vessels.toml) into outdir; returns the
    arrays as written."""
    os.makedirs(outdir, exist_ok=True)
    edges, nodes, radii = vessel_tree(n_nodes, seed, extra_edges)
    with open(os.path.join(outdir, "edges.dat"), "w") as f:
        for i, (a, b) in enumerate(edges.tolist()):
            f.write(f"{a},{b}\n" if i % 3 == 1 else f"  {a}   {b}\n")
    with open(os.path.join(outdir, "nodes.dat"), "w") as f:
        for i, (x, y, z) in enumerate(nodes.tolist()):
            if i % 4 == 1:
                f.write(f"{x!r}, {y!r}, {z!r}\n")
            elif i % 4 == 2:
                f.write(f"{x!r} {y!r}\n{z!r}\n")   # the read continues on the next record
            elif i % 4 == 3:
                f.write(f"{repr(x).replace('e', 'd') if 'e' in repr(x) else repr(x) + 'd0'} {y!r} {z!r}   ! c\n")
            else:
                f.write(f"{x!r} {y!r} {z!r}\n")
    with open(os.path.join(outdir, "radii.dat"), "w") as f:
        for r in radii.tolist():
            f.write(f"{r!r}\n")
    if toml:
        shutil.copy(os.path.join(HERE, "res", "vessels.toml"), os.path.join(outdir, "vessels.toml"))
    return edges, nodes, radii


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    extra = int(sys.argv[sys.argv.index("--extra-edges") + 1]) if "--extra-edges" in sys.argv else 0
    if extra:
        args = [a for a in args if a != str(extra)]
    write_vessel_data(args[0], int(args[1]) if len(args) > 1 else 40, int(args[2]) if len(args) > 2 else 7, extra)
