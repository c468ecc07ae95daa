"""Per-file finding digests for full-size parity (test / bench infrastructure).

One finding hashes to XXH64 (seed 0) of the packed little-endian record
    rule u32 | start u64 | end u64 | StartLine u32 | EndLine u32 |
    xxh64(Match) u64 | n_lines u32 | per Code line: Number u32, flags u8
    (1 IsCause, 2 FirstCause, 4 LastCause), xxh64(Content) u64
and a file's digest is the sum (mod 2^64) of its findings' hashes: Scan's
final sort leaves (RuleID, Match) ties in any order (scanner.go:441-446), so
the digest is order-free.  bench_cpu/cpu_scan.cpp computes the same record in
C (`tsgb_finding_hash`) for the C++ restatement and for an engine result read
through the drop-in ABI (`tsgb_result_digest`); this module computes it from
the Python oracle's findings, independently of that C code."""
import struct

import xxhash

MASK = (1 << 64) - 1


def _enc(t: str) -> bytes:
    return t.encode("utf-8", "surrogateescape")


def finding_hash(rule: int, start: int, end: int, sl: int, el: int, match: bytes, lines) -> int:
    """lines: (Number, Content bytes, IsCause, FirstCause, LastCause) tuples."""
    b = [struct.pack("<IQQIIQI", rule, start, end, sl, el, xxhash.xxh64(match).intdigest(), len(lines))]
    for num, content, c, f, last in lines:
        b.append(struct.pack("<IBQ", num, int(c) | int(f) << 1 | int(last) << 2, xxhash.xxh64(content).intdigest()))
    return xxhash.xxh64(b"".join(b)).intdigest()


def oracle_file_digest(findings, rule_index) -> tuple[int, int]:
    """(count, digest) of one oracle Scan result (`with_offsets=True`);
    rule_index maps RuleID -> the engine's rule index (config order)."""
    d = 0
    for x in findings:
        lines = [(ln["Number"], _enc(ln["Content"]), ln["IsCause"], ln["FirstCause"], ln["LastCause"])
                 for ln in x.Code["Lines"]]
        d = (d + finding_hash(rule_index[x.RuleID], x.Start, x.End, x.StartLine, x.EndLine, _enc(x.Match),
                              lines)) & MASK
    return len(findings), d
