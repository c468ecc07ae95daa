"""The largest file the engine verifies: 2 GiB - 1 bytes (the reference scans
any size, scanner.go:371-452; the walker spools entries >= 100 MiB and still
scans them, cached_file.go:36-52).  The match search runs on 32-bit
file-relative positions with signed capture slots, so a file of 2 GiB or more
is rejected with TSG_ERR_UNSUPPORTED (never mis-scanned); that is checked too.

The file is N identical filler lines, a pad, and a tail of secrets ending at
byte 2^31 - 1, so every match sits just below 2^31 (no signed-position slip)
and the last one ends on the last byte.  Its findings are the oracle's findings
for (10 filler lines + pad + the same tail) with every line number moved by
N - 10: the filler holds no keyword and no match, and the Code lines before
the first finding are filler either way.  Checked through the whole-file
device scan and the two-part byte-range split."""
import dataclasses
import json

import numpy as np
import pytest

pytest.importorskip("trivy_amd._native")

FILLER = b"alpha bravo charlie delta echo foxtrot golf hotel india juliet lima\n"


def _tail():
    from .split_corpus import straddle_block
    rng = np.random.default_rng(3)
    return straddle_block(rng, 0)[1:] + straddle_block(rng, 1)[1:]


def _shift(findings, d):
    out = []
    for f in findings:
        f = json.loads(json.dumps(f))
        f["StartLine"] += d
        f["EndLine"] += d
        for ln in (f["Code"]["Lines"] or []):
            ln["Number"] += d
        out.append(f)
    return out


@pytest.mark.gpu
def test_gpu_largest_file_whole_and_split_and_one_more_byte_rejected():
    import trivy_amd.secret as S
    from oracle import secret_oracle as o
    from trivy_amd.shard import scan_split

    from .test_gpu_parity import _canon, _plain
    size = 2 ** 31 - 1
    t0 = _tail()
    n = (size - len(t0) - 1) // len(FILLER)
    tail = b"x" * (size - n * len(FILLER) - len(t0) - 1) + b"\n" + t0
    assert n * len(FILLER) + len(tail) == size
    arr = np.empty(size, dtype=np.uint8)
    arr[:n * len(FILLER)].reshape(n, len(FILLER))[:] = np.frombuffer(FILLER, dtype=np.uint8)
    arr[n * len(FILLER):] = np.frombuffer(tail, dtype=np.uint8)
    data = arr.tobytes()
    del arr
    print(f"[large] built {size} bytes", flush=True)
    small = o.Scanner(None).scan("big.log", FILLER * 10 + tail)
    want_f = [{k: v for k, v in dataclasses.asdict(f).items() if k not in ("Start", "End")} for f in small["Findings"]]
    assert {f["RuleID"] for f in want_f} >= {"private-key", "jwt-token", "aws-access-key-id", "github-pat"}
    want = _canon({"FilePath": "big.log", "Findings": _shift(want_f, n - 10)})
    sc = S.new_scanner(None, device=0)
    args = S.ScanArgs("big.log", data)
    got = sc.scan_batch_device([args])[0]
    print("[large] whole-file scan done", flush=True)
    assert _canon(_plain(got)) == want
    assert _canon(_plain(scan_split(sc, args, n_parts=2))) == want
    # one byte more: rejected, not mis-scanned
    import trivy_amd._native as N
    big = S.ScanArgs("big.log", data + b"\n")
    del data
    with pytest.raises(N.EngineError) as ei:
        sc.scan_batch_device([big])
    assert ei.value.code == N.TSG_ERR_UNSUPPORTED
