import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))
sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP engine")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


def golden_names():
    """DAG goldens (tests/golden/make_golden.py); font_*.npz are SDF atlases."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith("font_"))


def load_golden(name):
    from wgraph.synth import Dag
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    d = Dag(z["oid"], z["time"], z["parent_off"], z["parent_oid"], z["flags"], z["band"])
    return d, {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def engine():
    """One HIP engine context for the whole GPU test session."""
    from wgraph import Engine
    e = Engine(0)
    yield e
    e.close()


# GPU tests run the §8(a)-(e) hot path first (layout/geometry/vertex parity,
# shards, atlas, glyph quads), then the §8(f) rows (order, search, frames,
# render), so a failure in a widening row never hides hot-path results.
_FIRST = ("test_gpu_parity", "test_gpu_shard", "test_gpu_font", "test_gpu_text")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        mod = item.module.__name__.rsplit(".", 1)[-1] if item.module else ""
        return (0, _FIRST.index(mod)) if mod in _FIRST else (1, 0)
    items.sort(key=rank)   # stable: file order is kept within each group
