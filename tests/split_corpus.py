"""Deterministic large files for the byte-range split tests.

`make_split_file(size, seed, cut_parts)` builds `size` bytes of text lines
(numpy, a few seconds for 64 MiB) and overwrites, at every cut that
`trivy_amd.shard.split_ranges` makes for each n in `cut_parts`, a block of
secrets that straddles the cut: a PEM private key, a JWT, an AWS access key
id, a GitHub token and a custom-rule secret.  One more private key runs from
64 KiB before the 2-way cut to 32 KiB after it, wider than any halo, and a
Kelvin sign sits next to every cut.  The custom rule's
keyword appears only in the file's first line, so its gate holds only when
the parts' keyword bits are OR'd.

The oracle's findings for the 64 MiB file are committed in
tests/golden/split_64mib.json (made by tools/make_split_golden.py); the GPU
test checks the file's sha256 before comparing.
"""
from __future__ import annotations

import numpy as np

SPAN = 4096

# filler vocabulary: lowercase words that hold no builtin keyword
_WORDS = [b"alpha", b"bravo", b"charlie", b"delta", b"echo", b"foxtrot", b"golf", b"hotel", b"india",
          b"juliet", b"lima", b"mike", b"november", b"oscar", b"papa", b"quebec", b"romeo", b"tango",
          b"uniform", b"victor", b"whiskey", b"xray", b"yankee", b"zulu", b"0", b"17", b"2048", b"=", b":",
          b"(", b")", b"{", b"}", b",", b";", b"value", b"count", b"index", b"name", b"data", b"path"]

CUSTOM_RULE = dict(id="split-custom", category="Custom", title="split custom", severity="HIGH",
                   regex=r"splitsecret_[0-9a-f]{24}", keywords=["triggerword"])

PEM_BODY_LINE = b"MIIEowIBAAKCAQEAu1SU1LfVLPHCozMxH2Mo4lgOEePzNm0tRgeLezV6ffAt0gunVTLw7onLRnrq0"


def _filler(rng, size):
    idx = rng.integers(0, len(_WORDS), size=size // 4 + 1024)
    toks = np.array(_WORDS, dtype=object)[idx]
    text = b" ".join(toks.tolist())
    arr = np.frombuffer(text, dtype=np.uint8).copy()[:size]
    # a newline every ~70 bytes
    nl = rng.integers(40, 100, size=size // 40 + 2).cumsum()
    arr[nl[nl < size]] = ord("\n")
    return arr


def straddle_block(rng, tag: int) -> bytes:
    body = b"\n".join([PEM_BODY_LINE] * 6)
    hexd = "".join("0123456789abcdef"[int(x)] for x in rng.integers(0, 16, size=24)).encode()
    alnum = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ234567"
    aws = b"AKIA" + bytes(alnum[int(x)] for x in rng.integers(0, 32, size=16))
    gh = b"ghp_" + bytes(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJ0123456789"[int(x)]
                         for x in rng.integers(0, 46, size=36))
    jwt = (b"eyJhbGciOiJIUzI1NiIsInR5cCI6IkpXVCJ9.eyJzdWIiOiIxMjM0NTY3ODkwIiwibmFtZSI6IkpvaG4iLCJ0Ijo"
           + str(tag).encode() + b"fQ.SflKxwRJSMeKKF2QT4fwpMeJf36POk6yJV_adQssw5c")
    return (b"\n-----BEGIN RSA PRIVATE KEY-----\n" + body + b"\n-----END RSA PRIVATE KEY-----\n"
            b"jwt = " + jwt + b"\n"
            b"aws_access_key_id = " + aws + b"\n"
            b"github = " + gh + b"\n"
            b"x = splitsecret_" + hexd + b"\n")


def cuts_for(size, parts):
    return sorted({(size * r // n) // SPAN * SPAN for n in parts for r in range(1, n)} - {0})


def make_split_file(size: int, seed: int = 7, cut_parts=(2, 3, 4)) -> bytes:
    rng = np.random.default_rng(seed)
    arr = _filler(rng, size)
    head = b"triggerword here\n"
    arr[:len(head)] = np.frombuffer(head, dtype=np.uint8)
    for i, c in enumerate(cuts_for(size, cut_parts)):
        blk = np.frombuffer(straddle_block(rng, i), dtype=np.uint8)
        # the cut falls at a different point of each block
        at = c - int(rng.integers(8, len(blk) - 8))
        arr[at:at + len(blk)] = blk
        k = "\u212a".encode()  # Kelvin sign spelling of 'k' in "key"
        kel = b"\n" + k + b"ey = value\n"
        arr[c + 2000:c + 2000 + len(kel)] = np.frombuffer(kel, dtype=np.uint8)
    if size >= (1 << 21):
        c = cuts_for(size, (2,))[0]
        span = min(size // 8, 64 << 10)
        body = (PEM_BODY_LINE + b"\n") * ((span + span // 2) // (len(PEM_BODY_LINE) + 1))
        pem = b"\n-----BEGIN OPENSSH PRIVATE KEY-----\n" + body + b"-----END OPENSSH PRIVATE KEY-----\n"
        arr[c - span:c - span + len(pem)] = np.frombuffer(pem, dtype=np.uint8)
    return arr.tobytes()
