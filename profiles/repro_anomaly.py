import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "whisper-git_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import wgraph
from wgraph import synth
from oracle import oracle_c
d = synth.generate("anomaly", 5000, seed=77)
eng = wgraph.Engine(0)
eng.build(d)
eng.synchronize()
o = oracle_c.OracleLayout(d)
lane, color = eng.lanes()
print("lanes equal", lane.tobytes() == o.lane.astype(np.uint32).tobytes(), flush=True)
