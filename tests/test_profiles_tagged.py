"""The bench line's counters come from one final tree: the PMC
summaries of every workload the line reports (`pmc` of the main line and of every `secondary`),
the HBM traffic (`roofline.traffic`) and the rocprof kernel means (`roofline.rocprof_source`)
carry one round tag, and every one of them exists."""
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


def test_every_workload_has_final_tree_counters():
    import bench
    want = {"nstar", "1m", "1m_big", "100m", "10b", "200b", "lua_1m",
            "model_P8_nstar", "model_P8_200b", "model_repl8_10b"}   # every secondary and per-rank model
    assert want <= set(bench.PMC_FILES)
    tags = {_tag(f) for f in bench.PMC_FILES.values()}
    assert tags == {bench.PMC_TAG}, tags
    for w, f in bench.PMC_FILES.items():
        path = os.path.join(ROOT, "profiles", f)
        assert os.path.exists(path), path
        with open(path) as fh:
            doc = json.load(fh)
        assert doc.get(w), (f, "no kernels for workload %s" % w)

