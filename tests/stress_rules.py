"""configs[4] stress material (test helper): generated gitleaks-style rule sets
and corpora that exercise them.

BASELINE.json configs[4]: "1000+ generated gitleaks-style regexes forcing DFA
state explosion / NFA bit-parallel fallback, minified long-line and
binary-ish files".  The rule families mirror the shapes custom
`trivy-secret.yaml` rules take (`pkg/fanal/secret/scanner.go:28-48` Rule
fields: id, category, title, severity, regex, keywords, path,
secret-group-name, allow-rules):

* generic assignment rules: `(?i)(?:kw1|kw2)[sep]{0,20}...(?P<secret>body)(?:term|$)`
* prefixed tokens: `prefix_[0-9a-zA-Z]{n}` (literal anchor)
* gap rules: `(?i)w1.{0,5}w2[:=]\\s*([A-Za-z0-9]{20,40})`
* keyword-less rules (every file takes the full-scan path)
* explosion rules: `(?:x|y)*x(?:x|y){k}lit` -- a forward DFA over these needs
  2^k states, so the verify DFA's state cap must hand them to the VM
* path-restricted and per-rule allow-listed rules

Everything is seeded; the same (seed, n_rules) always gives the same YAML and
the same corpus.
"""
from __future__ import annotations

import random
import string

from tests import corpus_gen

_CONS = "bcdfghjklmnprstvwxz"
_VOW = "aeiou"
_SEPS = ["=", ": ", " = ", ":= ", "=> ", ": '", '="', " := \"", ":\t"]
_BODIES = [  # (regex body, generator of a matching value)
    (r"[0-9a-z]{32}", lambda r: _rs(r, string.digits + string.ascii_lowercase, 32)),
    (r"[a-f0-9]{40}", lambda r: _rs(r, "0123456789abcdef", 40)),
    (r"[a-z0-9_\-]{16,64}", lambda r: _rs(r, string.ascii_lowercase + string.digits + "_-", r.randint(16, 64))),
    (r"[A-Za-z0-9]{24}", lambda r: _rs(r, string.ascii_letters + string.digits, 24)),
    (r"[0-9]{12,18}", lambda r: _rs(r, string.digits, r.randint(12, 18))),
]


def _rs(rng, alphabet, n):
    return "".join(rng.choice(alphabet) for _ in range(n))


def _word(rng, used, lo=3, hi=5):
    while True:
        w = "".join(rng.choice(_CONS) + rng.choice(_VOW) for _ in range(rng.randint(lo, hi)))
        if w not in used:
            used.add(w)
            return w


def make_rules(seed, n_rules):
    """[(rule dict, instance generator or None)] for n_rules custom rules."""
    rng = random.Random(seed)
    used = set()
    out = []
    for i in range(n_rules):
        fam = i % 10
        rid = f"stress-{i:04d}"
        rule = {"id": rid, "category": "Stress", "title": f"stress rule {i}",
                "severity": rng.choice(["LOW", "MEDIUM", "HIGH", "CRITICAL"])}
        if fam in (0, 1, 2, 3):  # generic assignment, gitleaks shape
            k1, k2 = _word(rng, used), _word(rng, used)
            body, gen = _BODIES[rng.randrange(len(_BODIES))]
            rule["regex"] = (r"(?i)(?:" + k1 + "|" + k2 + r")(?:[0-9a-z\-_\t .]{0,20})(?:[\s|']|[\s|\"]){0,3}"
                             r"(?:=|>|:=|\|\|:|<=|=>|:)(?:'|\"|\s|=|`){0,5}(?P<secret>" + body
                             + r")(?:['|\"|\n|\s|`|;]|$)")
            rule["keywords"] = [k1, k2.upper()]
            rule["secret-group-name"] = "secret"
            inst = (lambda k1=k1, k2=k2, gen=gen: lambda r: (r.choice([k1, k2.upper(), k1.capitalize()])
                                                              + r.choice(["", "_key", ".token", " api"])
                                                              + r.choice(_SEPS) + gen(r) + r.choice(["'", '"', ";", " ", ""])))()
        elif fam in (4, 5):  # prefixed token
            p = _word(rng, used, 2, 3)
            n = rng.choice([20, 32, 36, 40])
            rule["regex"] = p + r"_[0-9a-zA-Z]{" + str(n) + "}"
            rule["keywords"] = [p + "_"]
            inst = (lambda p=p, n=n: lambda r: p + "_" + _rs(r, string.ascii_letters + string.digits, n))()
        elif fam == 6:  # .{0,5} gap between two words
            w1, w2 = _word(rng, used, 2, 3), _word(rng, used, 2, 3)
            rule["regex"] = r"(?i)" + w1 + r".{0,5}" + w2 + r"[:=]\s*([A-Za-z0-9]{20,40})"
            rule["keywords"] = [w1]
            rule["secret-group-name"] = ""
            inst = (lambda w1=w1, w2=w2: lambda r: w1.upper() + _rs(r, "-_ .x", r.randint(0, 5)) + w2 + "="
                    + _rs(r, string.ascii_letters + string.digits, r.randint(20, 40)))()
        elif fam == 7:  # keyword-less
            w = _word(rng, used, 2, 2).upper()
            rule["regex"] = r"\b" + w + r"[0-9]{12}\b"
            inst = (lambda w=w: lambda r: w + _rs(r, string.digits, 12))()
        elif fam == 8:  # explosion: needs 2^k forward DFA states
            lit = _word(rng, used, 2, 2)
            k = rng.randint(10, 14)
            rule["regex"] = r"(?:x|y)*x(?:x|y){" + str(k) + "}" + lit
            rule["keywords"] = [lit]
            inst = (lambda lit=lit, k=k: lambda r: _rs(r, "xy", r.randint(0, 6)) + "x" + _rs(r, "xy", k) + lit)()
        else:  # path-restricted, with a rule allow-list
            w = _word(rng, used)
            rule["regex"] = w + r"-[a-z0-9]{10,30}"
            rule["keywords"] = [w]
            rule["path"] = r".*\.(?:env|cfg|txt)$"
            rule["allow-rules"] = [{"id": f"{rid}-allow", "description": "dummies", "regex": "dummy"}]
            inst = (lambda w=w: lambda r: w + "-" + r.choice(["dummy", ""]) + _rs(r, string.ascii_lowercase
                                                                                    + string.digits, r.randint(10, 24)))()
        out.append((rule, inst))
    return out


def _yaml_str(s):
    return "'" + s.replace("'", "''") + "'"


def write_config(path, rules):
    """YAML for parse_config (scanner.go:272-302 shape)."""
    lines = ["rules:"]
    for r, _ in rules:
        lines.append(f"  - id: {r['id']}")
        for k in ("category", "title", "severity"):
            lines.append(f"    {k}: {_yaml_str(r[k])}")
        lines.append(f"    regex: {_yaml_str(r['regex'])}")
        if r.get("keywords"):
            lines.append("    keywords:")
            lines.extend(f"      - {_yaml_str(k)}" for k in r["keywords"])
        if "secret-group-name" in r:
            lines.append(f"    secret-group-name: {_yaml_str(r['secret-group-name'])}")
        if "path" in r:
            lines.append(f"    path: {_yaml_str(r['path'])}")
        if "allow-rules" in r:
            lines.append("    allow-rules:")
            for a in r["allow-rules"]:
                lines.append(f"      - id: {a['id']}")
                lines.append(f"        description: {_yaml_str(a['description'])}")
                lines.append(f"        regex: {_yaml_str(a['regex'])}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def make_corpus(seed, rules, n_files, long_line_bytes=200_000):
    """Text files with planted custom-rule instances (~1 per 300 B), one
    minified single-line file, and binary-ish files (bytes >= 0x80, NULs)."""
    rng = random.Random(seed)
    gens = [g for _, g in rules if g is not None]
    exts = ["env", "cfg", "txt", "js", "py", "yaml"]
    files = []
    for i in range(n_files):
        base = corpus_gen.make_file(rng, n_lines=rng.randint(1, 60)).decode("utf-8", "surrogateescape").split("\n")
        for _ in range(max(1, len(base) // 4)):
            j = rng.randrange(len(base))
            base[j] = base[j][: rng.randrange(len(base[j]) + 1)] + " " + rng.choice(gens)(rng)
        files.append((f"stress/pkg{i % 7}/f{i:05d}.{rng.choice(exts)}",
                      "\n".join(base).encode("utf-8", "surrogateescape")))
    # minified: one long line of tokens and planted instances
    parts, n = [], 0
    while n < long_line_bytes:
        t = rng.choice(gens)(rng) if rng.random() < 0.05 else _rs(rng, string.ascii_letters + "{}();=,.:'\"", rng.randint(1, 24))
        parts.append(t)
        n += len(t) + 1
    files.append(("stress/min/app.min.js", (";".join(parts)).encode()))
    for i in range(4):  # binary-ish: high bytes and NULs around planted text
        blob = bytearray(rng.randrange(256) for _ in range(rng.randint(2000, 8000)))
        for _ in range(8):
            at = rng.randrange(len(blob))
            blob[at:at] = (" " + rng.choice(gens)(rng) + "\n").encode()
        files.append((f"stress/bin/blob{i}.txt", bytes(blob)))
    return files
