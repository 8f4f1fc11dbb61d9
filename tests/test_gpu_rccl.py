"""The strong-scaling path's collectives over RCCL (tools/rccl_probe.py) on the one-GPU box: a
one-rank RCCL communicator bound to the device as bench.py binds it for N > 1, running the
eyebox gather of an 8-way C3 split (device pack, ``dist.gather`` into rank 0's receive rows,
device assembly), the grid reduce, the two ``timed_run`` all-reduces and a barrier.  RCCL refuses
two ranks on one GPU, so this is the closest the builder's box gets to the driver's 8-GPU run:
it pins the call shapes, dtypes and buffers RCCL is given, not the transfer speed.

Tolerance: exact (the assembled grid equals the traced one bit for bit)."""
import json
import os
import socket
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_collectives_of_the_strong_scaling_path():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "rccl_probe.py")], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["backend"] == "nccl"
    assert rec["gather_equal"] and rec["reduce_equal"] and rec["all_reduce_ok"]
    assert rec["hits"] > 0
    out = os.environ.get("WGRT_RESULTS_DIR")
    if out:
        with open(os.path.join(out, "rccl_probe.json"), "w") as f:
            json.dump(rec, f, indent=1)
