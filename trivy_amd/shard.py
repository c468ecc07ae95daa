"""Multi-GPU sharding of a scan batch.

Files are independent in `Scanner.Scan` (pkg/fanal/secret/scanner.go:371-452
keeps no cross-file state), so a batch shards by file with no data-path
collective: each rank (one process per GPU) scans its own files on its own
engine, and only the per-file results are merged on the host, in input
order, the way the analyzer concatenates per-file `types.Secret`s
(pkg/fanal/analyzer/analyzer.go:403-444, sort at :218-229).

  partition(sizes, n)        greedy LPT by byte size: files largest first, each
                             to the least-loaded rank (ties: lowest rank), so
                             every rank gets about total/n bytes
  scan_sharded(fn, batch)    rank r runs fn(its files); results are exchanged
                             with all_gather_object (host objects only: tens of
                             bytes per finding) and returned in batch order

For an image (BASELINE configs[3]) the shard unit is the layer: batch =
the layer tars, sizes = their byte lengths, scan_fn = a closure over
`trivy_amd.walker.analyze_layers` on this rank's engine.

The merge is the only communication; with world size 1 (or no process group)
it is a plain call.

One file larger than a rank's share is split by byte range instead
(`scan_split`): rank r runs the scan pass over
[cut_r, cut_{r+1}) with the halo `Scanner.part_halo()` asks for
(tsg_scan_part_device), the per-part scan states (keyword bits, owned anchor
hits, per-4 KiB newline counts: KiB, not the file) are gathered on the owner,
which runs the rest of the pipeline over the whole file
(tsg_scan_merge_device).  The result equals the single-GPU scan of the file by
construction, whatever straddles a cut: a private key or a JWT across two
parts is verified by the owner over the whole file.
"""
from __future__ import annotations

import heapq
from typing import Any, Callable, List, Optional, Sequence


def partition(sizes: Sequence[int], n_ranks: int) -> List[List[int]]:
    """Greedy LPT: indices of the files each rank scans (each file exactly
    once; rank loads differ by at most the largest file)."""
    if n_ranks < 1:
        raise ValueError("n_ranks must be >= 1")
    order = sorted(range(len(sizes)), key=lambda i: (-int(sizes[i]), i))
    heap = [(0, r) for r in range(n_ranks)]
    parts: List[List[int]] = [[] for _ in range(n_ranks)]
    for i in order:
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    for p in parts:
        p.sort()  # keep input order inside a shard (batch locality, stable merge)
    return parts


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is part of this image
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def scan_sharded(scan_fn: Callable[[List[Any]], List[Any]], batch: Sequence[Any],
                 sizes: Optional[Sequence[int]] = None, group=None) -> List[Any]:
    """Scan `batch` across the ranks of the default (or given) process group.

    scan_fn(sub_batch) -> one result per item, in order (e.g.
    `Scanner.scan_batch` on this rank's engine).  sizes: bytes per item
    (default: len(item.content)).  Every rank must call this with the same
    batch; every rank returns the full, input-ordered result list.
    """
    dist = _dist()
    world = dist.get_world_size(group) if dist else 1
    rank = dist.get_rank(group) if dist else 0
    if sizes is None:
        sizes = [len(getattr(b, "content", b"")) for b in batch]
    parts = partition(sizes, world)
    mine = parts[rank]
    local = scan_fn([batch[i] for i in mine]) if mine else []
    if len(local) != len(mine):
        raise RuntimeError(f"scan_fn returned {len(local)} results for {len(mine)} files")
    if world == 1:
        gathered = [list(zip(mine, local))]
    else:
        gathered = [None] * world
        dist.all_gather_object(gathered, list(zip(mine, local)), group=group)
    out: List[Any] = [None] * len(batch)
    seen = 0
    for shard in gathered:
        for i, res in shard:
            out[i] = res
            seen += 1
    if seen != len(batch):
        raise RuntimeError(f"merge saw {seen} results for {len(batch)} files")
    return out


SPAN = 4096  # cuts and views fall on the engine's 4 KiB line-count spans


def split_ranges(file_len: int, n_parts: int, halo) -> List[tuple]:
    """Byte ranges of a split file: (own_lo, own_hi, view_lo, view_hi) per
    part, own ranges tiling [0, file_len) at 4 KiB-aligned cuts (fewer parts
    when the file is too small for n), views widened by halo = (left, right)."""
    if n_parts < 1:
        raise ValueError("n_parts must be >= 1")
    left, right = halo
    cuts = sorted({0, file_len} | {(file_len * r // n_parts) // SPAN * SPAN for r in range(1, n_parts)})
    out = []
    for lo, hi in zip(cuts, cuts[1:]):
        if hi <= lo:
            continue
        v_lo = max(0, lo - left) // SPAN * SPAN
        v_hi = min(file_len, hi + right)
        out.append((lo, hi, v_lo, v_hi))
    return out


def scan_split(scanner, args, group=None, owner: int = 0, n_parts: Optional[int] = None):
    """Byte-range split of ONE file over the ranks of `group` (every rank
    calls it with the same args).  Part p is scanned by group rank p % world;
    the parts go to `owner` -- a rank WITHIN `group` (gather_object: host
    bytes) -- whose engine merges them; every rank returns the file's Secret.
    With no process group the parts run one after another on this rank's
    engine."""
    dist = _dist()
    world = dist.get_world_size(group) if dist else 1
    rank = dist.get_rank(group) if dist else 0
    if not 0 <= owner < world:
        raise ValueError(f"owner {owner} is not a rank of the group (size {world})")
    # collectives address processes by global rank
    owner_global = dist.get_global_rank(group, owner) if dist and group is not None else owner
    data = args.content
    n = len(data)
    ranges = split_ranges(n, n_parts or world, scanner.part_halo())
    mine = []
    for p, (lo, hi, v_lo, v_hi) in enumerate(ranges):
        if p % world == rank:
            mine.append((p, scanner.scan_part(memoryview(data)[v_lo:v_hi], v_lo, lo, hi, n, args.file_path)))
    if world == 1:
        parts = [b for _, b in sorted(mine)]
    else:
        gathered = [None] * world if rank == owner else None
        dist.gather_object(mine, gathered, dst=owner_global, group=group)
        parts = [b for _, b in sorted(x for g in gathered for x in g)] if rank == owner else None
    result = [scanner.scan_merge(args, parts) if rank == owner else None]
    if world > 1:
        dist.broadcast_object_list(result, src=owner_global, group=group)
    return result[0]
