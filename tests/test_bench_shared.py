"""bench.py's multi-rank path as timed code (VERDICT r2 Missing #3): configs[3]
as ONE shared image whose layers are LPT-partitioned over the ranks
(trivy_amd.shard.scan_sharded inside the timed step).  Two ranks on one GPU
over gloo must produce exactly the merged per-layer results of a single-rank
run of the same image (reference: per-layer fan-out + merge,
pkg/fanal/artifact/image/image.go:201-240, pkg/fanal/analyzer/analyzer.go:422-444)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(cmd, log):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    with open(log, "w") as f:
        p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=f, timeout=240)
    assert p.returncode == 0, open(log).read()[-3000:]
    lines = [x for x in p.stdout.decode().splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout.decode()[-2000:]
    return json.loads(lines[0])


def test_shared_layer_set_is_rank_independent():
    sys.path.insert(0, ROOT)
    import bench
    from trivy_amd.shard import partition

    a = bench.shared_layer_set(5, 0.06, 5)
    assert a == bench.shared_layer_set(5, 0.03 * 2, 5)
    assert abs(sum(a) - 0.06) < 1e-9 and len(set(a)) == 5
    parts = partition([int(g * 1e9) for g in a], 2)
    assert sorted(i for p in parts for i in p) == list(range(5))


@pytest.mark.gpu
def test_bench_shared_two_ranks_gloo_equals_one_rank(tmp_path):
    common = ["--config", "3", "--shared", "--total-layers", "5", "--image-gb", "0.06", "--steps", "1",
              "--warmup", "0", "--no-cpu", "--no-parity"]
    one = _run([sys.executable, "-u", "bench.py", *common, "--dump", str(tmp_path / "one.npz")],
               str(tmp_path / "one.log"))
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                *common, "--dist-backend", "gloo", "--dump", str(tmp_path / "two.npz")], str(tmp_path / "two.log"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["layers_per_rank"] and sum(two["config"]["layers_per_rank"]) == 5
    assert min(two["config"]["layers_per_rank"]) >= 1  # both ranks analyzed layers
    a, b = np.load(tmp_path / "one.npz"), np.load(tmp_path / "two.npz")
    assert sorted(a.files) == sorted(b.files) and len(a.files) == 10
    n = 0
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k
        if k.startswith("locs"):
            n += len(a[k])
    assert n > 0 and one["counts"]["locs"] == two["counts"]["locs"] == n


@pytest.mark.gpu
def test_bench_config2_two_ranks_gloo(tmp_path):
    """The headline path's N > 1 shape (the driver's SCALE run: one rank per
    GPU, a barrier and the max over ranks around the timed steps, the whole
    job's bytes / that time), here as two ranks sharing one GPU over gloo:
    one JSON line from rank 0, n_gpus 2, the aggregate over both ranks'
    corpora, rank 0's parity properties intact."""
    common = ["--config", "2", "--gb", "1", "--steps", "2", "--warmup", "1", "--no-cpu"]
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                *common, "--dist-backend", "gloo"], str(tmp_path / "two.log"))
    assert two["n_gpus"] == 2 and two["scaling"] == "weak"
    assert abs(two["config"]["gb_per_gpu"] - 1.0) < 0.01
    # value = both ranks' bytes / the slowest rank's time
    assert abs(two["value"] - 2 * two["config"]["gb_per_gpu"] * 1e3 / two["ms_per_step"]) / two["value"] < 0.02
    p = two["parity"]
    assert p["planted_found"] == p["planted"] and p["decoys_found"] == 0 and p["spot_mismatched_files"] == 0
