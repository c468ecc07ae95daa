#!/usr/bin/env python3
"""Debug helper (GPU box): oracle vs engine on one fold-spelled fuzz file and
one bench-corpus file; optional verify profile of a full bench scan."""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import secret_oracle as O  # noqa: E402
from tests import corpus_gen  # noqa: E402
import trivy_amd.secret as S  # noqa: E402
from trivy_amd import _native as N  # noqa: E402

_FOLD = {"k": ["K"], "K": ["K"], "s": ["ſ"], "S": ["ſ"], "i": ["İ"], "I": ["İ"]}


def fold_spell(rng, text, p=0.35):
    return "".join(rng.choice(_FOLD[c]) if c in _FOLD and rng.random() < p else c for c in text)


def fuzz_files():
    rng = random.Random(2026)
    tpl = corpus_gen.secret_instances(rng)
    files = []
    for i in range(500):
        lines = []
        for _ in range(rng.randint(1, 12)):
            x = rng.random()
            if x < 0.45:
                s = rng.choice(tpl)()
                lines.append(fold_spell(rng, s) if rng.random() < 0.7 else s)
            elif x < 0.6:
                kw = rng.choice(corpus_gen.KEYWORD_SPRINKLE)
                lines.append(corpus_gen.noise_line(rng) + " " + fold_spell(rng, kw, 0.6) + " " + corpus_gen.noise_line(rng))
            else:
                lines.append(corpus_gen.noise_line(rng))
        files.append((f"src/f{i}.txt", "\n".join(lines).encode("utf-8")))
    return files


def compare(path, data):
    sc = S.new_scanner(None)
    g = sc.scan_batch([S.ScanArgs(path, data)])[0]
    w = O.Scanner(None).scan(path, data, with_offsets=True)
    gs = sorted((f.RuleID, f.StartLine, f.Match) for f in g.Findings)
    ws = sorted((f.RuleID, f.StartLine, f.Match) for f in w["Findings"])
    print("== ", path, "engine", len(gs), "oracle", len(ws))
    for x in sorted(set(gs) ^ set(ws)):
        print("  ", "ENGINE-ONLY" if x in gs else "ORACLE-ONLY", x)
    for f in w["Findings"]:
        if (f.RuleID, f.StartLine, f.Match) not in gs:
            print("   oracle span", f.RuleID, f.Start, f.End, repr(data[max(0, f.Start - 40):f.End + 10]))


if __name__ == "__main__":
    files = fuzz_files()
    for p, d in files:
        if p == "src/f49.txt":
            compare(p, d)
    for seed, f, n in [(20261017, 60262, None)]:
        sizes = None
        import bench
        sizes = bench.file_sizes(seed, int(50e9))
        n = int(sizes[f])
        buf = (ctypes.c_uint8 * n)()
        N.gen.tsg_gen_file(seed, f, n, 1e-6, buf)
        compare("src00/pkg000/file%010d.txt" % f, bytes(buf))
