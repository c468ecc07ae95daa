"""Oracle findings for the byte-range split test file (tests/split_corpus.py):
writes tests/golden/split_64mib.json = {size, seed, sha256, findings} for the
builtin rules + tests.split_corpus.CUSTOM_RULE.  CPU only (about a minute)."""
import dataclasses
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import secret_oracle as o  # noqa: E402
from tests.split_corpus import CUSTOM_RULE, make_split_file  # noqa: E402


def oracle_scanner():
    sc = o.Scanner(None)
    r = CUSTOM_RULE
    sc.rules = list(sc.rules) + [o.Rule(id=r["id"], category=r["category"], title=r["title"], severity=r["severity"],
                                        regex=o.GoRegexp(r["regex"]), keywords=r["keywords"])]
    return sc


def main(size=64 << 20, seed=7, out=os.path.join(ROOT, "tests", "golden", "split_64mib.json")):
    data = make_split_file(size, seed)
    res = oracle_scanner().scan("logs/big.log", data)
    findings = [{k: v for k, v in dataclasses.asdict(f).items() if k not in ("Start", "End")} for f in res["Findings"]]
    doc = {"size": size, "seed": seed, "path": "logs/big.log", "sha256": hashlib.sha256(data).hexdigest(),
           "findings": findings}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    print(out, len(findings), "findings")


if __name__ == "__main__":
    main()
