"""Lazy newline counts (engine.hip k_nl_cands / k_nl_spans / k_nl_check /
k_nl_tail): k_scan_fast no longer counts newlines, so the spans line numbering
reads are counted after the candidates, from each candidate file's start to
16 KiB past its last candidate, and completed when a location ends past that
bound or the span after it holds fewer than 4 newlines.  These files sit on
each of those edges -- a secret followed by a 40 KiB line (Code's lines below
lie past the bound), a secret in the file's last span, secrets far apart
(the bound moves), a long file whose only secret is at its end, a secret
right after 20 KiB of empty lines, a file of few newlines, neighbours in the
same 4 KiB spans -- and every finding (StartLine, EndLine, Match, Code) must
equal the oracle's."""
import random

import pytest

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")

TOK = b"ghp_" + b"A1b2C3d4E5f6G7h8I9j0K1l2M3n4O5p6Q7r8"  # github-pat
AWS = b"AKIA" + b"Z" * 16


def _files():
    rng = random.Random(7)
    words = [b"alpha", b"beta", b"gamma", b"delta", b"key", b"token", b"x=1", b"{", b"}"]

    def text(n, nl_every=60):
        out = bytearray()
        while len(out) < n:
            out += rng.choice(words) + (b"\n" if rng.randrange(nl_every) == 0 else b" ")
        return bytes(out[:n])

    f = []
    f.append(("long_after.txt", b"token: " + TOK + b"\n" + b"z" * 40_000 + b"\nend1\nend2\nend3\n"))
    f.append(("long_after_nonl.txt", b"a\nb\ntoken: " + TOK + b" " + b"q" * 50_000))
    f.append(("last_span.txt", text(9000) + b"\nsecret " + AWS + b"\nlast\n"))
    f.append(("far_apart.txt", b"x " + TOK + b"\n" + text(70_000) + b"\n" + AWS + b"\n" + text(3000)))
    f.append(("only_at_end.txt", text(120_000) + b"\n" + TOK))
    f.append(("empty_lines.txt", b"\n" * 20_000 + TOK + b"\n\n\n"))
    f.append(("few_newlines.txt", text(30_000, nl_every=4000) + b" " + AWS + b" " + text(30_000, nl_every=4000)))
    for i in range(12):  # small neighbours sharing spans with the above and each other
        body = text(rng.randint(10, 900)) + (b"\n" + TOK + b"\n" if i % 3 == 0 else b"")
        f.append((f"small{i}.txt", body))
    f.append(("no_secret_big.txt", text(200_000)))
    f.append(("nl_right_after.txt", TOK + b"\n"))
    f.append(("crossing.txt", text(4090) + b"\n" + TOK + b"\n" + text(5000)))
    return f


def test_lazy_newline_counts_vs_oracle():
    from .test_gpu_parity import _compare_batch
    n = _compare_batch(_files(), seed_info="lazy-lines")
    assert n >= 10


def test_lazy_newline_counts_custom_full_file_rule(tmp_path):
    """A rule without anchors runs as a full-file job: its files are counted
    whole from the candidate stage (k_nl_cands' kFullFlag)."""
    from .test_gpu_parity import _compare_batch
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text("rules:\n  - id: any-digits\n    category: t\n    title: t\n    severity: LOW\n"
                   "    regex: '[0-9]{12}'\n")
    files = _files() + [("digits.txt", b"x\n" * 5000 + b"123456789012\n" + b"y" * 30_000 + b"\nz\n")]
    assert _compare_batch(files, str(cfg), seed_info="lazy-lines-full") > 0
