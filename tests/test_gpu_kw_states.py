"""Keyword states (k_scan_fast resolves keyword-only outputs itself: the
group goes to its wave's LDS queue, drained at each span's end, instead of a
k_report event; engine.hip kw_resolve, ruleset.cpp build_fast).
MatchKeywords (pkg/fanal/secret/scanner.go:169-181) must stay exact:

* CPU: the builtin ruleset's keyword states cover the short keyword-only
  keywords (jwt, lob, key: most of configs[2]'s former events);
* GPU: gate bits against the oracle's MatchKeywords on many tiny files
  (several files per 4 KiB span, keywords on file edges, split by a file
  separator, in both cases, next to bytes >= 0x80 and control bytes that
  alias letters in the scan's fold columns), on files dense enough to
  overflow a wave's queue (the overflow becomes events), and on a file of
  more than 1 MiB (read-first keyword words); and the complete findings of
  such files against the oracle's Scan."""
import ctypes
import random

import pytest

from oracle import secret_oracle as o

from . import corpus_gen

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")


def _kw_states(sc):
    ns, nk = ctypes.c_uint32(), ctypes.c_uint32()
    buf = ctypes.create_string_buffer(4096)
    N.check(N.lib.tsg_ruleset_kw_states(sc._rs.handle, ctypes.byref(ns), ctypes.byref(nk), buf, 4096))
    words = [w.decode() for w in buf.raw.split(b"\0")[: nk.value]]
    return ns.value, words


def test_builtin_keyword_states():
    sc = S.new_scanner(None)
    ns, words = _kw_states(sc)
    assert ns > 0 and {"jwt", "lob", "key"} <= set(words), (ns, words)
    # every keyword-state keyword is a keyword some rule's non-implied gate needs
    need = {k.lower() for r in sc.rules for k in r.keywords}
    assert set(words) <= need


def _tiny_files(seed, n, words):
    rng = random.Random(seed)
    alias = [0xEA, 0xCB, 0xF7, 0x0A, 0x0B, 0x1A, 0xC5, 0xE2]  # >= 0x80 / control bytes
    files = []
    for i in range(n):
        parts = []
        for _ in range(rng.randint(0, 4)):
            w = rng.choice(words)
            w = "".join(c.upper() if rng.random() < 0.3 else c for c in w).encode()
            k = rng.random()
            if k < 0.2:  # an aliasing byte in place of one letter
                j = rng.randrange(len(w))
                w = w[:j] + bytes([rng.choice(alias)]) + w[j + 1:]
            parts.append(w)
            parts.append(bytes(rng.choice(b"abc xyz_=\n\t.") for _ in range(rng.randint(0, 12))))
        body = b"".join(parts)
        if rng.random() < 0.3:  # a keyword at the very end / start of a file
            body = body + rng.choice(words).encode()
        if rng.random() < 0.3:
            body = rng.choice(words).encode() + body
        files.append((f"t/{i:05d}.txt", body))
    return files


@pytest.mark.gpu
def test_gpu_keyword_states_gates_vs_oracle():
    from .test_gpu_stress import _check_gates
    sc = S.new_scanner(None)
    _, words = _kw_states(sc)
    words = words + ["apikey", "api_key", "token", "secret"]
    files = _tiny_files(5, 4000, words)
    # split by a file separator: "jw" | "t..."
    files += [("edge/a.txt", b"xx jw"), ("edge/b.txt", b"t lo"), ("edge/c.txt", b"b ke"), ("edge/d.txt", b"y")]
    # dense: a wave's queue overflows within one span (the rest become events)
    files.append(("dense.txt", b"jwt lob key " * 4000))
    files.append(("dense_mixed.txt", b"".join(w.encode() + b" " for w in words) * 500))
    # > 1 MiB: read-first keyword words
    files.append(("big.txt", b"abc " * 300_000 + b"JwT\n" + b"zzz " * 10_000 + b"Lob"))
    files += corpus_gen.make_corpus(91, 300)
    assert _check_gates(None, files) > 0


@pytest.mark.gpu
def test_gpu_keyword_states_findings_vs_oracle():
    from .test_gpu_parity import _canon, _oracle_plain, _plain
    sc = S.new_scanner(None)
    oc = o.Scanner(None)
    _, words = _kw_states(sc)
    rng = random.Random(9)
    files = _tiny_files(6, 1500, words)
    # files whose rules need a keyword-state keyword AND hold the anchor
    jwt = "eyJhbGciOiJIUzI1NiJ9." + "eyJzdWIiOiIxMjM0NTY3ODkwIn0." + "SflKxwRJSMeKKF2QT4fwpMeJf36POk6yJV_adQssw5c"
    for i in range(300):
        kw = rng.choice(["jwt", "JWT", "Jw\xeat", "lob", "key"]).encode("latin-1")
        files.append((f"plant/{i}.txt", b"x " * rng.randint(0, 50) + kw + b" = " + jwt.encode() + b"\n"))
    got = sc.scan_batch_device([S.ScanArgs(p, d) for p, d in files])
    n = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oc.scan(p, d))
        n += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n > 100


def _many_keywords_config(tmp_path, n_rules=70, seed=17):
    """Custom rules whose keywords are short strings over a small alphabet
    (suffixes of one another: states with two outputs) and whose regex never
    holds them (so every keyword is needed by a non-implied gate): more
    keyword-only states than the scan keeps (kFastKwStates / kFastKwBits), the
    rest resolved as events."""
    from . import stress_rules
    rng = random.Random(seed)
    words = set()
    while len(words) < n_rules:
        words.add("".join(rng.choice("abcdefgh") for _ in range(rng.randint(2, 4))))
    words = sorted(words, key=lambda w: (len(w), w))
    rules = [({"id": f"kwmany-{i}", "category": "test", "title": "t", "severity": "LOW",
               "regex": r"zq[0-9]{6}", "keywords": [w]}, None) for i, w in enumerate(words)]
    path = str(tmp_path / "trivy-secret.yaml")
    stress_rules.write_config(path, rules)
    return path, words


def test_many_keywords_states_capped(tmp_path):
    path, _ = _many_keywords_config(tmp_path)
    sc = S.new_scanner(S.parse_config(path))
    ns, words = _kw_states(sc)
    assert 0 < ns <= 32 and len(words) <= 32


@pytest.mark.gpu
def test_gpu_many_keywords_gates_and_findings_vs_oracle(tmp_path):
    from .test_gpu_parity import _canon, _oracle_plain, _plain
    from .test_gpu_stress import _check_gates
    path, words = _many_keywords_config(tmp_path)
    files = _tiny_files(21, 2000, words)
    rng = random.Random(22)
    for i in range(400):
        body = " ".join(rng.choice(words) for _ in range(rng.randint(0, 6)))
        body += f" zq{rng.randrange(10**6):06d} " + " ".join(rng.choice(words) for _ in range(rng.randint(0, 3)))
        files.append((f"f/{i}.txt", body.encode()))
    files.append(("dense.txt", (" ".join(words) + " zq123456\n").encode() * 300))
    assert _check_gates(path, files) > 0
    sc = S.new_scanner(S.parse_config(path))
    oc = o.Scanner(o.parse_config(path))
    got = sc.scan_batch_device([S.ScanArgs(p, d) for p, d in files])
    n = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oc.scan(p, d))
        n += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n > 200
