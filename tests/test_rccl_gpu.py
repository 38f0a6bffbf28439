"""bench.py's multi-GPU data path on a real GPU (reference sub-window split,
core/sampler.cpp:55-78): torch.distributed over RCCL at world size 1, the cost deal, the timed
steps with their per-step film gather and the reassembly, in a child process started before it
uses the GPU (tests/rccl_world1.py). The 2..8-rank deal and gather are covered by the gloo tests
(test_tiles_dist.py) and the 8-rank C3 reassembly on one GPU (test_configs_gpu.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_bench_path():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_world1.py"), str(_free_port())], env=env,
                       capture_output=True, text=True, timeout=300)
    line = next((x for x in r.stdout.splitlines() if x.startswith("{")), None)
    assert r.returncode == 0 and line, "rc %d\n%s\n%s" % (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    d = json.loads(line)
    assert d["backend"] == "nccl" and d["world"] == 1 and d["film_equal"]
    assert d["skin_tiles"] > 0
