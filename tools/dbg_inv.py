import sys; sys.path.insert(0, '.')
import numpy as np
from rsmcrt_amd.job import Job
from rsmcrt_amd import scene, abi
from rsmcrt_amd.engine import Engine
text = open("tests/golden/res/thinBarrier.toml").read()
text = (text.replace("maxNumSteps = 30000", "maxNumSteps = 3").replace("nphotons = 10000000", "nphotons = 2000")
        .replace("BoxDimensions = [0.0,2.0,2.0]", "BoxDimensions = [0.5,2.0,2.0]")
        + '\n[[detectors]]\ntype = "circle"\nID = "T"\nposition = [1.49, 0.0, 0.0]\ndirection = [1.0, 0.0, 0.0]\n'
        'radius = 1.0\nnbins = 10\nlayer = 2\ninverseTarget = 0.2\n')
open("/tmp/inv.toml", "w").write(text)
j = Job("/tmp/inv.toml", mode="inverse")
d = j.desc
sc = scene.Scene([]); sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]; sc.top = list(j.top[:d.n_top])
for fl in (abi.FLAG_PATHLENGTH, abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE, 0):
    with Engine(sc, d.grid, j.detectors) as eng:
        r = eng.run(d.source, 2000, seed=d.seed, flags=fl)
        print(fl, r.counters_dict(), r.det_bins)
        cfg = j.inverse_config()
        print(eng.inverse(d.source, cfg, 2000, j.targets(), seed=d.seed, flags=fl))
print(j.run_inverse())
