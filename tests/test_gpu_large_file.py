"""Files of any size (the reference scans any size, scanner.go:371-452; the
walker spools entries >= 100 MiB and still scans them, cached_file.go:36-52).
The match search runs on 32-bit file-relative positions with signed capture
slots up to 2^31 - 1 bytes; the jobs of longer files run the same kernels
instantiated on 64-bit positions and slots.

1. The last 32-bit file: N identical filler lines, a pad, and a tail of
   secrets ending at byte 2^31 - 1 (every match just below 2^31, the last one
   on the last byte).
2. A file of 2^32 + 64 MiB: blocks of secrets whose private key straddles
   byte 2^31 and byte 2^32 (its BEGIN before, its END after), with a group
   rule through the capture search (aws-secret-access-key) and one through the
   span shortcut (heroku-api-key), and a last block ending on the last byte.

Findings are the oracle's findings for each block's window (10 filler lines +
pad + block + 10 filler lines) with every line number moved by the lines
before the window: the filler holds no keyword and no match, and Code lines
reach only 2 lines past a finding.  Checked through the whole-file device scan
and the two-part byte-range split."""
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


def _block(rng, tag):
    from .split_corpus import straddle_block
    sec = bytes(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789/+"[int(x)]
                for x in rng.integers(0, 64, size=40))
    hexu = lambda k: bytes(b"0123456789ABCDEF"[int(x)] for x in rng.integers(0, 16, size=k))  # noqa: E731
    uuid = hexu(8) + b"-" + hexu(4) + b"-" + hexu(4) + b"-" + hexu(4) + b"-" + hexu(12)
    return (straddle_block(rng, tag)[1:] + b"aws_secret_access_key = \"" + sec + b"\"\n"
            + b"cfg heroku_api_key = \"" + uuid + b"\"\n")


def _layout(size, starts, blocks):
    """Segments (filler lines, pad + block) putting block i at byte starts[i]
    (the last block ends on the file's last byte); returns the segments and per
    block its oracle window and line shift."""
    segs, wins, pos, lines = [], [], 0, 0
    ends = list(starts) + [size - len(blocks[-1])]
    for i, (st, blk) in enumerate(zip(ends, blocks)):
        gap = st - pos
        a = (gap - 1) // len(FILLER) - 1
        k = gap - a * len(FILLER) - 1
        assert a >= 10 and 0 <= k < 2 * len(FILLER)
        pad = b"x" * k + b"\n"
        segs.append((a, pad + blk))
        last = i == len(blocks) - 1
        wins.append((FILLER * 10 + pad + blk + (b"" if last else FILLER * 10), lines + a - 10))
        lines += a + 1 + blk.count(b"\n")
        pos = st + len(blk)
    assert pos == size
    return segs, wins


def _build(size, segs):
    arr = np.empty(size, dtype=np.uint8)
    pos = 0
    for a, tail in segs:
        arr[pos:pos + a * len(FILLER)].reshape(a, len(FILLER))[:] = np.frombuffer(FILLER, dtype=np.uint8)
        pos += a * len(FILLER)
        arr[pos:pos + len(tail)] = np.frombuffer(tail, dtype=np.uint8)
        pos += len(tail)
    assert pos == size
    return arr


@pytest.mark.gpu
def test_gpu_file_past_4gib_whole_and_split_vs_oracle():
    import trivy_amd.secret as S
    from oracle import secret_oracle as o
    from trivy_amd.shard import scan_split

    from .test_gpu_parity import _canon, _plain
    size = (1 << 32) + (64 << 20)
    rng = np.random.default_rng(11)
    blocks = [_block(rng, t) for t in range(3)]
    # the private key's BEGIN line 40 bytes before 2^31 / 2^32, its END after
    segs, wins = _layout(size, [(1 << 31) - 40, (1 << 32) - 40], blocks)
    oracle = o.Scanner(None)
    want_f = []
    censored_nl = 0  # Scan numbers lines on the censored content: earlier blocks' censored newlines are gone
    for text, shift in wins:
        small = oracle.scan("huge.log", text, with_offsets=True)
        fs = [{k: v for k, v in dataclasses.asdict(f).items() if k not in ("Start", "End")} for f in small["Findings"]]
        assert {f["RuleID"] for f in fs} >= {"private-key", "jwt-token", "aws-access-key-id", "github-pat",
                                              "aws-secret-access-key", "heroku-api-key"}
        want_f += _shift(fs, shift - censored_nl)
        cens = np.zeros(len(text), dtype=bool)
        for f in small["Findings"]:
            cens[f.Start:f.End] = True
        censored_nl += int((np.frombuffer(text, dtype=np.uint8)[cens] == 10).sum())
    want = _canon({"FilePath": "huge.log", "Findings": want_f})
    data = _build(size, segs).tobytes()
    print(f"[large] built {size} bytes", flush=True)
    sc = S.new_scanner(None, device=0)
    args = S.ScanArgs("huge.log", data)
    got = _canon(_plain(sc.scan_batch_device([args])[0]))
    print("[large] whole-file scan done", flush=True)
    lines = [(f["RuleID"], f["StartLine"]) for f in got["Findings"]]
    assert got == want, lines
    assert _canon(_plain(scan_split(sc, args, n_parts=2))) == want


@pytest.mark.gpu
def test_gpu_largest_32bit_file_whole_and_split():
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
