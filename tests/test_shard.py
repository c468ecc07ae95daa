"""Multi-rank sharding (trivy_amd/shard.py) on the CPU:
LPT partition properties, and a world-size-2 gloo run whose merged result
equals the single-process scan.  The per-rank scanner here is the CPU oracle
(tests only); on the GPU box each rank passes its engine's Scanner.scan_batch."""
import os
import random
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from trivy_amd.shard import partition, scan_sharded

from . import corpus_gen


def test_partition_covers_and_balances():
    rng = random.Random(3)
    for n_ranks in (1, 2, 3, 8):
        sizes = [int(rng.lognormvariate(8.7, 1.6)) + 10 for _ in range(500)]
        parts = partition(sizes, n_ranks)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in p) for p in parts]
        assert max(loads) - min(loads) <= max(sizes)
        assert all(p == sorted(p) for p in parts)
    assert partition([], 4) == [[], [], [], []]
    assert partition([5, 5], 4)[2:] == [[], []]
    with pytest.raises(ValueError):
        partition([1], 0)


def _oracle_scan(batch):
    from oracle import secret_oracle as O
    sc = O.Scanner(None)
    return [sc.scan(p, d) for p, d in batch]


def _corpus():
    return corpus_gen.make_corpus(21, 24)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = _corpus()
        res = scan_sharded(_oracle_scan, files, sizes=[len(d) for _, d in files])
        if rank == 0:
            import json
            with open(out_path, "w") as f:
                json.dump(res, f, default=lambda o: o.__dict__)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_rank_gloo_merge_equals_single_process(tmp_path):
    import json
    out = str(tmp_path / "merged.json")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    merged = json.load(open(out))
    files = _corpus()
    want = json.loads(json.dumps(_oracle_scan(files), default=lambda o: o.__dict__))
    assert merged == want
    assert sum(len(r["Findings"]) for r in want) > 0


def test_world_one_is_a_plain_call():
    files = _corpus()[:6]
    assert scan_sharded(_oracle_scan, files, sizes=[len(d) for _, d in files]) == _oracle_scan(files)


@pytest.mark.gpu
def test_sharded_engine_scan_matches_batch():
    import trivy_amd.secret as S
    sc = S.new_scanner(None)
    batch = [S.ScanArgs(p, d) for p, d in _corpus()]
    assert scan_sharded(sc.scan_batch, batch) == sc.scan_batch(batch)


# --- layer sets (BASELINE configs[3]: image layers sharded across GPUs) ------

def _layers():
    from .test_gpu_layer import _layer
    return [_layer(60 + k, 30 + 7 * k) for k in range(5)]


def _oracle_layers(layers):
    from .test_gpu_layer import _oracle_layer
    return [_oracle_layer(x) for x in layers]


def _layer_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        layers = _layers()
        res = scan_sharded(_oracle_layers, layers, sizes=[len(x) for x in layers])
        if rank == 0:
            import json
            with open(out_path, "w") as f:
                json.dump(res, f, default=lambda o: o.__dict__)
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_layer_set_merge_equals_single_process(tmp_path):
    """Layers are the shard unit for an image: LPT over layer bytes, one
    analyze_layers call per rank, host merge in layer order."""
    import json
    out = str(tmp_path / "layers.json")
    mp.start_processes(_layer_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    merged = json.load(open(out))
    want = json.loads(json.dumps(_oracle_layers(_layers()), default=lambda o: o.__dict__))
    assert merged == want
    assert sum(len(s) for s, _, _ in want) > 0


@pytest.mark.gpu
def test_sharded_layer_set_matches_pipelined():
    from trivy_amd.analyzer import SecretAnalyzer
    from trivy_amd.walker import analyze_layers
    a = SecretAnalyzer()
    a.init("")
    layers = _layers()
    fn = lambda ls: analyze_layers(a, ls)  # noqa: E731
    assert scan_sharded(fn, layers, sizes=[len(x) for x in layers]) == fn(layers)
