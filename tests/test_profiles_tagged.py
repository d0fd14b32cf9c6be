"""The bench line's counters come from one final tree: the PMC summary
(`pmc`), the HBM traffic (`roofline.traffic`) and the rocprof kernel means
(`roofline.rocprof_source`) that bench.py reads for the north-star workload carry one round tag."""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def _tag(path):
    m = re.search(r"(r\d+[a-z0-9]*)_", os.path.basename(path))
    assert m, path
    return m.group(1)


def test_nstar_counters_share_one_tag():
    import bench
    pmc = bench.PMC_FILES["nstar"]
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
        traffic_src = json.load(fh)["source"]
    with open(os.path.join(ROOT, "profiles", bench.ROCPROF_MEANS)) as fh:
        rocprof_src = json.load(fh)["source"]
    tags = {_tag(pmc), _tag(traffic_src), _tag(rocprof_src)}
    assert len(tags) == 1, (pmc, traffic_src, rocprof_src)
    for rel in ("profiles/" + pmc, traffic_src, rocprof_src):
        assert os.path.exists(os.path.join(ROOT, rel)), rel
