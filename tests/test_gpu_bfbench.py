"""The C++ bench binary (redis-bloomfilter_amd/lib/bfbench, SURVEY §8 b "Callers") drives the
engine through the C ABI alone: its step runs on the GPU, finds every member of its include?
batches and reports a sane false-positive rate, in the plain and the pipelined form."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "redis-bloomfilter_amd", "lib", "bfbench")


@pytest.mark.parametrize("pipeline", ["0", "1"])
def test_bfbench_runs_through_the_c_abi(pipeline):
    out = subprocess.run([BIN, "--config", "1m", "--steps", "3", "--warmup", "1", "--pipeline", pipeline, "--host"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["false_negatives"] == 0
    assert (line["m"], line["k"]) == (9585058, 6)
    assert line["keys_per_s"] > 1e8
    assert 0.0 <= line["observed_fp_rate"] < 0.5
    assert line["host_api"]["insert_keys_per_s"] > 0
    names = set(line["kernels_ms"])
    assert ("include_hash_kernel" in names) == (pipeline == "1")
