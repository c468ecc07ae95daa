#!/usr/bin/env python3
"""Golden fixture for the fold-special cliff test (tests/test_gpu_fold.py).

Each case is a 64 MiB file of the bench corpus (tsg_gen_file host twin,
seeded) with a few lines spliced in that spell keywords / anchor literals
with İ (U+0130), K (U+212A) or ſ (U+017F).  The expected findings come from
the CPU oracle (oracle/secret_oracle.py, ~2 min per case), so the GPU test
only regenerates the bytes and compares.  Run from the repo root:
    python3 tools/make_fold_fixture.py  > tests/golden/fold_big.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import secret_oracle as O  # noqa: E402
from trivy_amd import _native as N  # noqa: E402

from tests.fold_cases import CASES, build  # noqa: E402


def main():
    out = []
    for case in CASES:
        data = build(N, case)
        res = O.Scanner(None).scan("src/big.txt", data, with_offsets=True)
        want = sorted([f.RuleID, f.Start, f.End, f.StartLine, f.EndLine] for f in res["Findings"])
        out.append(dict(case, want=want))
        print(f"{case['name']}: {len(want)} findings", file=sys.stderr)
    json.dump({"source": "tools/make_fold_fixture.py (oracle/secret_oracle.py expectations)", "cases": out},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
