"""Speculative verify jobs (engine.hip k_mark_jobs soft splits, k_chain_fix,
k_verify_redo): candidates of one (file, rule) are verified in parallel as
separate jobs, and a job whose first match starts before the previous match's
end is re-run in order -- Go's FindAll (regexp.go allMatches, scanner.go:107)
is sequential, so the result must equal the oracle's on texts built to make
the parallel jobs collide: matches that swallow later anchor hits, long lazy
matches, overlapping windows, many hits of one rule in one file.  GPU."""
import random

import pytest

from oracle import secret_oracle as O
import trivy_amd.secret as S

RULES = [
    ("span-begin", r"BEGIN[^#]*?END", ["begin"]),                          # later BEGINs inside a match
    ("greedy-eq", r"(?i)key[a-z ]{0,300}=[0-9]{3}", ["key"]),            # a match reaches over later "key"s
    ("tok", r"tk_[a-z0-9]{8}", ["tk_"]),                                  # dense, independent hits
    ("unb", r"(?:x|y)*xq[0-9]{2}", ["xq"]),                               # unbounded window (alphabet run)
]


def _yaml():
    lines = ["rules:"]
    for rid, rx, kws in RULES:
        lines += [f"  - id: {rid}", "    category: c", "    title: t", "    severity: HIGH",
                  "    regex: '" + rx.replace("'", "''") + "'", "    keywords:"]
        lines += [f"      - {k}" for k in kws]
    return "\n".join(lines) + "\n"


def _texts():
    rng = random.Random(41)
    out = []
    for i in range(60):
        parts = []
        for _ in range(rng.randint(10, 80)):
            r = rng.random()
            if r < 0.15:
                parts.append("BEGIN" + " filler" * rng.randint(0, 40))
            elif r < 0.25:
                parts.append("END")
            elif r < 0.45:
                parts.append("key" + " abc" * rng.randint(0, 30) + rng.choice(["=123", "=12", " x"]))
            elif r < 0.65:
                parts.append("tk_" + "".join(rng.choice("abc0123") for _ in range(rng.choice([7, 8, 9]))))
            elif r < 0.75:
                parts.append("".join(rng.choice("xy") for _ in range(rng.randint(0, 90))) + "xq" + str(rng.randint(0, 999)))
            else:
                parts.append("lorem ipsum " * rng.randint(1, 12))
        sep = rng.choice([" ", "\n", "  ", ";"])
        out.append((f"spec/f{i:03d}.txt", sep.join(parts).encode()))
    return out


@pytest.mark.gpu
def test_gpu_speculative_jobs_vs_oracle(tmp_path):
    from .test_gpu_parity import _canon, _oracle_plain, _plain
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(_yaml())
    sc_o = O.Scanner(O.parse_config(str(cfg)))
    sc_g = S.new_scanner(S.parse_config(str(cfg)), device=0)
    files = _texts()
    got = sc_g.scan_batch([S.ScanArgs(p, d) for p, d in files])
    per_rule = {}
    for (p, d), g in zip(files, got):
        want = _oracle_plain(sc_o.scan(p, d))
        for f in want["Findings"]:
            per_rule[f["RuleID"]] = per_rule.get(f["RuleID"], 0) + 1
        assert _canon(_plain(g)) == _canon(want), p
    assert all(per_rule.get(r[0], 0) > 20 for r in RULES), per_rule
