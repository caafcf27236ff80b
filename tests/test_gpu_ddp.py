"""Data-parallel training paths with two real ranks (tests/ddp_check.py under torch.distributed.run, gloo, both
ranks on the one leased GPU): averaged gradients with the overlapped hash-table all-reduce, eager and graph-replayed
steps keeping the replicas identical."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _bench_default():
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    return bench.DEFAULT_PRECISION


@pytest.mark.parametrize("precision", ["fp32", _bench_default()])
def test_two_rank_training(tmp_path, precision):
    """fp32 and the benchmarked preset (its fp16 weight-gradient launches deferred into the third graph, the fp16
    panels they read made in the first two)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "ddp.json"
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(HERE, "ddp_check.py"), str(out), precision]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    ranks = "\n".join(l for l in r.stderr.splitlines() if l.startswith("[rank"))
    assert r.returncode == 0, r.stdout[-2000:] + ranks[-6000:]
    res = json.loads(out.read_text())
    print(res)
    assert res["world"] == 2
    assert res["grads_differ_across_ranks"] > 1e-3          # the ranks really trained on different rays
    assert res["grad_err"] < 1e-4, res
    assert res["pose_grad_err"] < 1e-4, res
    assert res["reduced_equal_across_ranks"]
    assert res["eager_params_equal"]
    assert res["graph_disabled"] is None
    assert res["graph_stats"]["replays"] >= 1, res
    assert res["graph_params_equal"]
    # the graph path's exchange (hash tables overlapped with the weight-gradient graph, the rest after it) averages the
    # ranks' gradients, as the eager path does
    assert res["graph_allreduces"] >= 1 and res["graph_grad_err"] < 1e-6, res
    # the hash-table regions went out early, in two stages: the radiance and background tables after the backward's
    # first phase (overlapping the SDF backward graph), the SDF table after the second (overlapping the weight
    # gradients) -- 3 tables per replayed step
    assert res["graph_overlapped_regions"] >= 3 * res["graph_stats"]["replays"], res
    assert res["graph_stage_order_ok"], res
