"""CPU: bench.py takes the roofline's HBM traffic from the latest
profiles/<tag>_pmc.json of the workload, latest by the tag scheme
r<round><a..z, aa..az, ba..> (round, then suffix length, then suffix) —
not by file name, where r06o would sort after r06bf."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_root):
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.ROOT = tmp_root
    return b


def test_latest_pmc_by_tag_order(tmp_path):
    prof = tmp_path / "profiles"
    prof.mkdir()
    w = "some workload"
    for tag, v in (("r05h", 1), ("r06o", 2), ("r06af", 3), ("r06bf", 4), ("r06z", 5)):
        (prof / f"{tag}_pmc.json").write_text(json.dumps({"workload": w, "hbm_bytes_per_launch": v}))
    (prof / "r07_pmc.json").write_text(json.dumps({"workload": "other", "hbm_bytes_per_launch": 9}))
    (prof / "r06ca_pmc.json").write_text("not json")
    got = _bench(str(tmp_path)).pmc_traffic(None, w)
    assert got["hbm_bytes_per_launch"] == 4 and got["_file"] == os.path.join("profiles", "r06bf_pmc.json")
