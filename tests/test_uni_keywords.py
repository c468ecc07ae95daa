"""Keywords whose lowercase holds a non-ASCII rune (custom trivy-secret.yaml
rules; MatchKeywords compares strings.ToLower(keyword) with
bytes.ToLower(content), scanner.go:169-181).  The engine finds them with
k_uni_keywords around the batch's non-ASCII bytes (unicode.ToLower table
tools/gen_lower_table.py -> trivy_amd/csrc/gre_lower_table.h).

CPU: the ToLower table against Python's (Unicode 13.0) lowercase mapping and
the oracle's go_bytes_to_lower.  GPU: rules gated only by such keywords over
files spelling them in every case (and with invalid bytes, across 4 KiB
spans, keyword and match in different places) against the oracle's Scan,
through the whole-batch path and the byte-range split."""
import random
import re
import unicodedata

import pytest

from oracle import secret_oracle as o

N = pytest.importorskip("trivy_amd._native")

TABLE = "trivy_amd/csrc/gre_lower_table.h"


def _table():
    txt = open(TABLE).read()
    return {int(a, 16): int(b, 16) for a, b in re.findall(r"\{0x([0-9a-f]+), 0x([0-9a-f]+)\}", txt)}


def test_lower_table_is_go_simple_lowercase():
    t = _table()
    for cp in range(0x30000):
        if 0xD800 <= cp <= 0xDFFF or unicodedata.category(chr(cp)) == "Cn":
            continue
        want = 0x69 if cp == 0x130 else (ord(chr(cp).lower()) if len(chr(cp).lower()) == 1 else cp)
        assert t.get(cp, cp) == want, hex(cp)
    # added after Unicode 13.0 (Go 1.22 = 15.0): Vithkuqi, Glagolitic, Latin
    assert t[0x10570] == 0x10597 and t[0x2C2F] == 0x2C5F and t[0xA7C0] == 0xA7C1


KWS = ["clé", "пароль", "straße", "ΣΕΚΡΕΤ", "ǅ", "ključ"]


def _rules():
    import trivy_amd.secret as S
    return [S.Rule(id=f"uni-{i}", category="Uni", title="uni", severity="HIGH",
                   regex=r"val_[0-9a-f]{8}", keywords=[kw]) for i, kw in enumerate(KWS)] + \
        [S.Rule(id="uni-mixed", category="Uni", title="uni", severity="HIGH", regex=r"tok_[A-Z]{6}",
                keywords=["zzz", "Ключ"])]


def _spellings(rng, kw):
    forms = [kw, kw.upper(), kw.lower(), kw.title(), kw.swapcase()]
    f = rng.choice(forms)
    return "".join(c.upper() if rng.random() < 0.3 else c for c in f)


def _files(seed, n):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        parts = []
        for _ in range(rng.randint(1, 30)):
            k = rng.random()
            if k < 0.25:
                parts.append(_spellings(rng, rng.choice(KWS + ["ключ", "КЛЮЧ"])).encode())
            elif k < 0.5:
                parts.append(b"val_%08x" % rng.getrandbits(32))
            elif k < 0.6:
                parts.append(b"tok_" + bytes(rng.choice(b"ABCDEFGHIJ") for _ in range(6)))
            elif k < 0.7:
                parts.append(bytes([rng.randint(0x80, 0xFF)]))  # invalid byte next to a keyword
            elif k < 0.75:
                parts.append(b"x" * rng.randint(3000, 9000))  # push keywords across 4 KiB spans
            else:
                parts.append(rng.choice([b"alpha", b" ", b"\n", b"=", "é".encode(), "K".encode(), "ſ".encode()]))
        out.append((f"uni/f{i:04d}.txt", b"".join(parts)))
    return out


def _oracle(rules, files):
    sc = o.Scanner(None)
    sc.rules = [o.Rule(id=r.id, category=r.category, title=r.title, severity=r.severity,
                       regex=o.GoRegexp(r.regex), keywords=r.keywords) for r in rules]
    return [sc.scan(p, d) for p, d in files]


@pytest.mark.gpu
def test_gpu_non_ascii_keywords_vs_oracle():
    import trivy_amd.secret as S
    from trivy_amd.shard import scan_split

    from .test_gpu_parity import _canon, _oracle_plain, _plain
    rules = _rules()
    sc = S.new_scanner(S.Config(enable_builtin_rule_ids=["__none__"], custom_rules=rules), device=0)
    files = _files(5, 300)
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    want = _oracle(rules, files)
    n_kept = n_gated = 0
    for (p, d), g, w in zip(files, got, want):
        w = _oracle_plain(w)
        assert _canon(_plain(g)) == _canon(w), p
        n_kept += len(w["Findings"])
        n_gated += b"val_" in d and not w["Findings"]
    assert n_kept > 300 and n_gated > 5  # both outcomes of the gate occur
    # one long file through the byte-range split: keyword in one part, match in another
    big = b"".join(d for _, d in files[:120])
    args = S.ScanArgs("uni/big.txt", big)
    w = _canon(_oracle_plain(_oracle(rules, [("uni/big.txt", big)])[0]))
    assert _canon(_plain(sc.scan_batch_device([args])[0])) == w
    assert _canon(_plain(scan_split(sc, args, n_parts=5))) == w
