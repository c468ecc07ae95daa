"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A plain-Python restatement of Trivy's secret scanner used as the *checker* for
the MI355X engine.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module; the product path
(``trivy_amd``) never does and fails loudly without its HIP library.

What it restates (reference = /root/reference, Trivy v2 snapshot):
  * Scanner.Scan / FindLocations / FindSubmatchLocations / AllowLocation /
    MatchKeywords / Blocks / censorLocation / toFinding / findLocation
    .................................. pkg/fanal/secret/scanner.go:97-537
  * Config / ParseConfig / convertSeverity / NewScanner
    .................................. pkg/fanal/secret/scanner.go:28-48,272-359
  * SecretAnalyzer.Analyze / Required . pkg/fanal/analyzer/secret/secret.go:79-153
  * utils.IsBinary ................... pkg/fanal/utils/utils.go:77-95
  * Go regexp (RE2 syntax, leftmost-first, rune-based; go1.22 stdlib, not in
    the reference tree): restated by translating each Go pattern into the
    third-party ``regex`` module's dialect (explicit ASCII \\s \\d \\w \\b,
    ``$``=\\z unless (?m), scoped (?i) groups, numbered groups so duplicate
    names keep Go's one-group-per-occurrence meaning) and replaying Go's
    ``allMatches`` iteration loop (regexp.go) on the text decoded with
    ``surrogateescape`` so that each invalid UTF-8 byte is one rune, as
    ``utf8.DecodeRune`` yields.

Pinning: the restatement is checked against every known-answer case of the
reference's own tests (tests/golden/, transcribed by tools/extract_golden.py):
34 scanner_test.go cases, 5+5 analyzer cases and the integration golden.
Behaviour NOT pinned by any reference test (invalid UTF-8, non-ASCII case
folding, empty-match iteration, \\r handling, huge inputs) is
"restatement-derived, not Go-verified".  Known deviation: Python's (?i)
folds U+0130 with 'i', Go's simple folding does not.
"""
from __future__ import annotations

import dataclasses
import os
import re
from typing import List, Optional

import numpy as np
import regex as _re
import yaml

from oracle import go_unicode as _go_unicode

# --------------------------------------------------------------------------- #
# Go RE2 syntax -> python `regex` translation
# --------------------------------------------------------------------------- #

_WORD = "0-9A-Za-z_"
_SPACE = "\\t\\n\\f\\r "
_POSIX = {
    "alnum": "0-9A-Za-z", "alpha": "A-Za-z", "ascii": "\\x00-\\x7f", "blank": "\\t ",
    "cntrl": "\\x00-\\x1f\\x7f", "digit": "0-9", "graph": "!-~", "lower": "a-z",
    "print": " -~", "punct": "!-/:-@\\[-`{-~", "space": "\\t\\n\\v\\f\\r ",
    "upper": "A-Z", "word": _WORD, "xdigit": "0-9A-Fa-f",
}


class GoSyntaxError(ValueError):
    pass


def _esc_char(c: str) -> str:
    cp = ord(c)
    if c.isalnum() and cp < 128:
        return c
    return "\\U%08x" % cp


class _Translator:
    """Recursive-descent reader of Go regexp/syntax (Perl flags) that emits an
    equivalent `regex`-module pattern."""

    def __init__(self, pat: str):
        self.p = pat
        self.i = 0
        self.names: List[str] = [""]  # group 0
        self.pending = ""

    def peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else ""

    def translate(self):
        out = self.alt({"i": False, "m": False, "s": False, "U": False})
        if self.i != len(self.p):
            raise GoSyntaxError("unexpected )")
        return out

    def alt(self, flags):
        # Go's parser keeps flags as parser state restored only at the group's
        # closing paren: a (?i) in one branch also covers later branches.
        flags = dict(flags)
        parts = [self.concat(flags)]
        while self.peek() == "|":
            self.i += 1
            parts.append(self.concat(flags))
        return "|".join(parts)

    def concat(self, flags):
        out = []
        while self.i < len(self.p) and self.peek() not in "|)":
            if self.p.startswith("(?", self.i) and self._try_flags(flags):
                continue
            self.pending = ""
            atom = self.atom(flags)
            if atom is None:
                continue
            if self.pending:
                out.append(self.pending)
            out.append(self.repeat(atom, flags))
        return "".join(out)

    def _try_flags(self, flags):
        # (?flags) or (?flags:re) — the latter handled in atom()
        j = self.i + 2
        k = j
        while k < len(self.p) and self.p[k] in "imsU-":
            k += 1
        if k < len(self.p) and self.p[k] == ")" and k > j:
            self._apply_flags(self.p[j:k], flags)
            self.i = k + 1
            return True
        return False

    @staticmethod
    def _apply_flags(spec, flags):
        neg = False
        seen_neg = False
        for c in spec:
            if c == "-":
                if seen_neg:
                    raise GoSyntaxError("bad flags")
                neg = seen_neg = True
                continue
            flags[c] = not neg

    def repeat(self, atom, flags):
        while True:
            c = self.peek()
            if c in ("*", "+", "?"):
                self.i += 1
                op = c
            elif c == "{":
                m = _re.match(r"\{(\d+)(,(\d*))?\}", self.p[self.i:])
                if not m:
                    return atom
                lo = int(m.group(1))
                hi = lo if m.group(2) is None else (None if m.group(3) == "" else int(m.group(3)))
                if lo > 1000 or (hi is not None and (hi > 1000 or hi < lo)):
                    raise GoSyntaxError("invalid repeat count")
                self.i += m.end()
                op = m.group(0)
            else:
                return atom
            lazy = False
            if self.peek() == "?":
                self.i += 1
                lazy = True
            if flags["U"]:
                lazy = not lazy
            if not atom:
                raise GoSyntaxError("missing argument to repetition operator")
            atom = "(?:%s)%s%s" % (atom, op, "?" if lazy else "")
            nxt = self.peek()
            if nxt in ("*", "+", "?") or (nxt == "{" and _re.match(r"\{(\d+)(,(\d*))?\}", self.p[self.i:])):
                raise GoSyntaxError("invalid nested repetition operator")

    def wrap(self, s, flags, cls=False):
        if not flags["i"]:
            return s
        # Go's simple folding keeps U+0130/U+0131 out of the i/I orbit (each
        # is its own orbit); the `regex` module relates them to i / I, so they
        # never reach its (?i): a class decides them case-sensitively, a
        # folded literal (never one of them, see fold_lit) not at all.
        if cls:
            return "(?:(?=[\\u0130\\u0131])%s|(?![\\u0130\\u0131])(?i:%s))" % (s, s)
        return "(?:(?![\\u0130\\u0131])(?i:%s))" % s

    def fold_lit(self, ch, flags):
        """A literal rune under the current flags (U+0130/U+0131 fold to themselves only)."""
        if ch in "\u0130\u0131":
            return _esc_char(ch)
        return self.wrap(_esc_char(ch), flags)

    def atom(self, flags):
        c = self.peek()
        if c == "(":
            return self.group(flags)
        if c == "[":
            return self.char_class(flags)
        if c == ".":
            self.i += 1
            return "(?s:.)" if flags["s"] else "[^\\n]"
        if c == "^":
            self.i += 1
            return "(?:(?<=\\n)|\\A)" if flags["m"] else "\\A"
        if c == "$":
            self.i += 1
            return "(?=\\n|\\Z)" if flags["m"] else "\\Z"
        if c in "*+?":
            raise GoSyntaxError("missing argument to repetition operator")
        if c == "\\":
            return self.escape(flags)
        self.i += 1
        return self.fold_lit(c, flags)

    def group(self, flags):
        self.i += 1  # (
        inner_flags = dict(flags)
        if self.p.startswith("?P<", self.i) or self.p.startswith("?<", self.i):
            self.i += 3 if self.p[self.i + 1] == "P" else 2
            end = self.p.index(">", self.i)
            name = self.p[self.i:end]
            if not name or not _re.fullmatch(r"[A-Za-z0-9_]+", name):
                raise GoSyntaxError("invalid named capture")
            self.i = end + 1
            self.names.append(name)
            body = self.alt(inner_flags)
            prefix = "("
        elif self.p.startswith("?", self.i):
            j = self.i + 1
            k = j
            while k < len(self.p) and self.p[k] in "imsU-":
                k += 1
            if k >= len(self.p) or self.p[k] != ":":
                raise GoSyntaxError("invalid or unsupported Perl syntax")
            self._apply_flags(self.p[j:k], inner_flags)
            self.i = k + 1
            body = self.alt(inner_flags)
            prefix = "(?:"
        else:
            self.names.append("")
            body = self.alt(inner_flags)
            prefix = "("
        if self.peek() != ")":
            raise GoSyntaxError("missing closing )")
        self.i += 1
        return prefix + body + ")"

    def escape(self, flags, in_class=False):
        self.i += 1
        c = self.peek()
        if c == "":
            raise GoSyntaxError("trailing backslash")
        self.i += 1
        perl = {"d": "0-9", "w": _WORD, "s": _SPACE}
        if c in perl:  # Go folds the group under (?i): (?i)\\w holds U+017F and U+212A
            return perl[c] if in_class else self.wrap("[%s]" % perl[c], flags, cls=True)
        if c in "DWS":
            if in_class:
                raise GoSyntaxError("negated perl class inside class unsupported by oracle")
            return self.wrap("[^%s]" % perl[c.lower()], flags, cls=True)
        if not in_class:
            if c == "b":
                return "(?:(?<=[%s])(?![%s])|(?<![%s])(?=[%s]))" % ((_WORD,) * 4)
            if c == "B":
                return "(?:(?<=[%s])(?=[%s])|(?<![%s])(?![%s]))" % ((_WORD,) * 4)
            if c == "A":
                return "\\A"
            if c == "z":
                return "\\Z"
            if c == "Q":
                end = self.p.find("\\E", self.i)
                lit = self.p[self.i:] if end < 0 else self.p[self.i:end]
                self.i = len(self.p) if end < 0 else end + 2
                # Go pushes \Q..\E as single-rune literals: a following
                # repetition binds to the last rune only.
                if not lit:
                    return None
                self.pending = "".join(self.fold_lit(ch, flags) for ch in lit[:-1])
                return self.fold_lit(lit[-1], flags)
        if c in "pP":
            # parse.go parseUnicodeClass: the set is explicit (Go's tables and
            # fold closure, oracle/go_unicode.py), so it needs no (?i) wrap
            start = self.i - 2
            if self.peek() == "{":
                end = self.p.find("}", self.i)
                if end < 0:
                    raise GoSyntaxError("invalid character class range: `%s`" % self.p[start:])
                name = self.p[self.i + 1:end]
                self.i = end + 1
            else:
                name = self.peek()
                self.i += len(name)
            neg = c == "P"
            if name.startswith("^"):
                name, neg = name[1:], not neg
            rs = _go_unicode.go_class(name, neg, flags["i"])
            if rs is None:
                raise GoSyntaxError("invalid character class range: `%s`" % self.p[start:self.i])
            # the text's invalid bytes are U+DC80..U+DCFF here (see _decode) and
            # U+FFFD in Go; no valid UTF-8 decodes to a surrogate
            cut = []
            for lo, hi in rs:
                if lo < 0xD800:
                    cut.append((lo, min(hi, 0xD7FF)))
                if hi > 0xDFFF:
                    cut.append((max(lo, 0xE000), hi))
            if any(lo <= 0xFFFD <= hi for lo, hi in rs):
                cut.append((0xDC80, 0xDCFF))
            body = "".join("\\U%08x-\\U%08x" % (lo, hi) for lo, hi in cut)
            return ("p", body) if in_class else ("[%s]" % body if body else "(?!)")
        simple = {"a": 7, "f": 12, "t": 9, "n": 10, "r": 13, "v": 11}
        if c in simple:
            ch = chr(simple[c])
        elif c == "x":
            if self.peek() == "{":
                end = self.p.index("}", self.i)
                ch = chr(int(self.p[self.i + 1:end], 16))
                self.i = end + 1
            else:
                ch = chr(int(self.p[self.i:self.i + 2], 16))
                self.i += 2
        elif c in "01234567":
            if c != "0" and not (self.peek() and self.peek() in "01234567"):
                raise GoSyntaxError("backreferences unsupported")
            digs = c
            while len(digs) < 3 and self.peek() and self.peek() in "01234567":
                digs += self.peek()
                self.i += 1
            ch = chr(int(digs, 8))
        elif ord(c) < 128 and not c.isalnum():
            ch = c
        else:
            raise GoSyntaxError("invalid escape \\" + c)
        return _esc_char(ch) if in_class else self.fold_lit(ch, flags)

    def char_class(self, flags):
        """A bracket class, (?i)-wrapped here: the \\p members (already Go's
        folded sets) stay outside the wrap, whose U+0130/U+0131 exclusion is
        for folded literals only."""
        self.i += 1
        neg = False
        if self.peek() == "^":
            neg = True
            self.i += 1
        items = []
        pitems = []
        first = True
        while True:
            c = self.peek()
            if c == "":
                raise GoSyntaxError("missing closing ]")
            if c == "]" and not first:
                self.i += 1
                break
            first = False
            if c == "[" and self.peek(1) == ":":
                end = self.p.find(":]", self.i + 2)
                name = self.p[self.i + 2:end]
                pneg = name.startswith("^")
                if pneg:
                    raise GoSyntaxError("negated posix class unsupported by oracle")
                items.append(_POSIX[name])
                self.i = end + 2
                continue
            lo = self._class_char(flags)
            if lo is None:
                continue
            if isinstance(lo, tuple):  # a perl class expansion
                if isinstance(lo[0], tuple):  # \\p{..}: an explicit set
                    pitems.append(lo[0][1])
                else:
                    items.append(lo[0])
                continue
            if self.peek() == "-" and self.peek(1) not in ("]", ""):
                self.i += 1
                hi = self._class_char(flags)
                if isinstance(hi, tuple) or hi is None:
                    raise GoSyntaxError("bad class range")
                if ord(hi) < ord(lo):
                    raise GoSyntaxError("invalid character class range")
                items.append("%s-%s" % (_esc_char(lo), _esc_char(hi)))
            else:
                items.append(_esc_char(lo))
        if not pitems:
            return self.wrap("[%s%s]" % ("^" if neg else "", "".join(items)), flags, cls=True)
        pset = "".join(pitems)
        if not items:
            return "[%s%s]" % ("^" if neg else "", pset) if pset else ("(?s:.)" if neg else "(?!)")
        if neg:  # neither a \\p member nor a (folded) literal member
            return "(?:%s%s)" % ("(?![%s])" % pset if pset else "",
                                 self.wrap("[^%s]" % "".join(items), flags, cls=True))
        return "(?:%s%s)" % ("[%s]|" % pset if pset else "", self.wrap("[%s]" % "".join(items), flags, cls=True))

    def _class_char(self, flags):
        c = self.peek()
        if c == "\\":
            nxt = self.peek(1)
            if nxt in "dwspP":
                return (self.escape(flags, in_class=True),)
            if nxt in "DWS":
                self.escape(flags, in_class=True)
            save = self.i
            s = self.escape(flags, in_class=True)
            # decode our own escaping back to a char
            m = _re.fullmatch(r"\\U([0-9a-f]{8})", s)
            if m:
                return chr(int(m.group(1), 16))
            if len(s) == 1:
                return s
            self.i = save
            raise GoSyntaxError("bad escape in class")
        self.i += 1
        return c


def translate_go_regex(pat: str):
    """Return (compiled `regex` pattern, subexp names) for a Go RE2 pattern."""
    t = _Translator(pat)
    py = t.translate()
    return _re.compile(py), t.names


class GoRegexp:
    """The subset of Go's *regexp.Regexp API the secret scanner calls."""

    def __init__(self, pat: str):
        self.source = pat
        self.rx, self.names = translate_go_regex(pat)

    # Go: Regexp.SubexpNames
    def subexp_names(self):
        return list(self.names)

    def _iter(self, data: bytes):
        """Go's allMatches loop (regexp.go) over rune-decoded text, yielding
        the span tuples (in rune indices) of each delivered match."""
        s, _ = _decode(data)
        pos, prev_end = 0, -1
        end = len(s)
        while pos <= end:
            m = self.rx.search(s, pos)
            if m is None:
                break
            accept = True
            if m.end() == pos:
                if m.start() == prev_end:
                    accept = False
                pos += 1  # one rune forward (str index == rune index)
            else:
                pos = m.end()
            prev_end = m.end()
            if accept:
                yield m

    def find_all_index(self, data: bytes):
        _, off = _decode(data)
        return [[int(off[m.start()]), int(off[m.end()])] for m in self._iter(data)]

    def find_all_submatch_index(self, data: bytes):
        _, off = _decode(data)
        res = []
        for m in self._iter(data):
            idx = []
            for g in range(len(self.names)):
                a, b = m.span(g)
                idx += [int(off[a]), int(off[b])] if a >= 0 else [-1, -1]
            res.append(idx)
        return res

    def match_string(self, s: bytes) -> bool:
        t, _ = _decode(s)
        return self.rx.search(t) is not None


_DECODE_CACHE = [None, None]  # (bytes object, result): Scan decodes one content once per rule


def _decode(data: bytes):
    """Rune-decode like Go's utf8.DecodeRune (invalid byte -> one rune) and
    return (text, byte offset of each rune index incl. the end)."""
    if data.isascii():
        return data.decode("ascii"), range(len(data) + 1)
    if _DECODE_CACHE[0] is data:
        return _DECODE_CACHE[1]
    s = data.decode("utf-8", "surrogateescape")
    # rune widths: escaped invalid bytes (U+DC80..U+DCFF) are 1 byte, else the UTF-8 length
    cp = np.frombuffer(s.encode("utf-32-le", "surrogatepass"), dtype=np.uint32)
    w = np.where(cp < 0x80, 1, np.where(cp < 0x800, 2, np.where(cp < 0x10000, 3, 4)))
    w[(cp >= 0xDC80) & (cp <= 0xDCFF)] = 1
    off = np.zeros(len(s) + 1, dtype=np.int64)
    np.cumsum(w, out=off[1:])
    res = (s, off)
    _DECODE_CACHE[0], _DECODE_CACHE[1] = data, res
    return res


# --------------------------------------------------------------------------- #
# bytes.ToLower (Go) for the keyword gate — scanner.go:175
# --------------------------------------------------------------------------- #

_INVALID = re.compile("[\udc80-\udcff]")


def go_bytes_to_lower(b: bytes) -> bytes:
    if b.isascii():
        return b.lower()
    s = b.decode("utf-8", "surrogateescape")
    if "\u03a3" in s:  # str.lower() applies Final_Sigma in context; Go maps each rune alone
        return _go_bytes_to_lower_slow(s)
    # invalid byte -> RuneError (re-encoded as EF BF BD); U+0130 -> 'i' (unicode.ToLower's
    # simple mapping: the only rune whose str.lower() is not one rune); every other rune
    # maps alone, as str.lower() does
    s = _INVALID.sub("\ufffd", s).replace("\u0130", "i")
    return s.lower().encode("utf-8")


def _go_bytes_to_lower_slow(s: str) -> bytes:
    out = []
    for ch in s:
        cp = ord(ch)
        if 0xDC80 <= cp <= 0xDCFF:
            out.append("\ufffd")  # invalid byte -> RuneError, re-encoded
        elif ch == "\u0130":
            out.append("i")  # unicode.ToLower(U+0130) = 'i' (simple mapping)
        else:
            lo = ch.lower()
            out.append(lo if len(lo) == 1 else ch)
    return "".join(out).encode("utf-8")


# --------------------------------------------------------------------------- #
# Data model — pkg/fanal/secret/scanner.go:28-95, pkg/fanal/types/secret.go
# --------------------------------------------------------------------------- #

@dataclasses.dataclass
class AllowRule:
    id: str = ""
    description: str = ""
    regex: Optional[GoRegexp] = None
    path: Optional[GoRegexp] = None


@dataclasses.dataclass
class Rule:
    id: str = ""
    category: str = ""
    title: str = ""
    severity: str = ""
    regex: Optional[GoRegexp] = None
    keywords: List[str] = dataclasses.field(default_factory=list)
    path: Optional[GoRegexp] = None
    allow_rules: List[AllowRule] = dataclasses.field(default_factory=list)
    exclude_block: List[GoRegexp] = dataclasses.field(default_factory=list)
    secret_group_name: str = ""


def _allow_path(rules, path: str) -> bool:  # scanner.go:200-207
    return any(r.path is not None and r.path.match_string(path.encode()) for r in rules)


def _allow(rules, match: bytes) -> bool:  # scanner.go:209-216
    return any(r.regex is not None and r.regex.match_string(match) for r in rules)


def _rx(v):
    return GoRegexp(v) if v is not None else None


def _load_builtin():
    here = os.path.dirname(os.path.abspath(__file__))
    import json
    with open(os.path.join(here, "..", "trivy_amd", "data", "builtin_rules.json")) as fh:
        d = json.load(fh)
    rules = [Rule(id=r["id"], category=r["category"], title=r["title"], severity=r["severity"],
                  regex=GoRegexp(r["regex"]), keywords=list(r["keywords"]),
                  secret_group_name=r["secret_group_name"]) for r in d["rules"]]
    allows = [AllowRule(id=a["id"], description=a["description"], regex=_rx(a["regex"]),
                        path=_rx(a["path"])) for a in d["allow_rules"]]
    return rules, allows


_BUILTIN = None


def builtin():
    global _BUILTIN
    if _BUILTIN is None:
        _BUILTIN = _load_builtin()
    return _BUILTIN


def _convert_severity(sev) -> str:  # scanner.go:305-313
    sev = "" if sev is None else str(sev)
    if sev.lower() in ("low", "medium", "high", "critical", "unknown"):
        return sev.upper()
    return "UNKNOWN"


def _allow_rules_from(lst):
    return [AllowRule(id=a.get("id", "") or "", description=a.get("description", "") or "",
                      regex=_rx(a.get("regex")), path=_rx(a.get("path"))) for a in (lst or [])]


def parse_config(path: str):
    """ParseConfig (scanner.go:272-302): None when path is empty/missing."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        raw = yaml.safe_load(fh) or {}
    cfg = {
        "enable": list(raw.get("enable-builtin-rules") or []),
        "disable": list(raw.get("disable-rules") or []),
        "disable_allow": list(raw.get("disable-allow-rules") or []),
        "rules": [],
        "allow_rules": _allow_rules_from(raw.get("allow-rules")),
        "exclude_block": [GoRegexp(x) for x in ((raw.get("exclude-block") or {}).get("regexes") or [])],
    }
    for r in raw.get("rules") or []:
        cfg["rules"].append(Rule(
            id=r.get("id", "") or "", category=r.get("category", "") or "",
            title=r.get("title", "") or "", severity=_convert_severity(r.get("severity")),
            regex=_rx(r.get("regex")), keywords=list(r.get("keywords") or []),
            path=_rx(r.get("path")), allow_rules=_allow_rules_from(r.get("allow-rules")),
            exclude_block=[GoRegexp(x) for x in ((r.get("exclude-block") or {}).get("regexes") or [])],
            secret_group_name=r.get("secret-group-name", "") or ""))
    return cfg


@dataclasses.dataclass
class Line:
    Number: int = 0
    Content: str = ""
    IsCause: bool = False
    Annotation: str = ""
    Truncated: bool = False
    Highlighted: str = ""
    FirstCause: bool = False
    LastCause: bool = False


@dataclasses.dataclass
class SecretFinding:
    RuleID: str = ""
    Category: str = ""
    Severity: str = ""
    Title: str = ""
    StartLine: int = 0
    EndLine: int = 0
    Code: dict = dataclasses.field(default_factory=lambda: {"Lines": []})
    Match: str = ""
    # internal byte offsets (scanner.go:223-226), not part of types.SecretFinding
    Start: int = -1
    End: int = -1


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


class Scanner:
    """NewScanner + Scan (scanner.go:315-452)."""

    def __init__(self, config=None):
        brules, ballows = builtin()
        if config is None:
            self.rules = list(brules)
            self.allow_rules = list(ballows)
            self.exclude_block = []
            return
        enabled = brules
        if config["enable"]:
            enabled = [r for r in brules if r.id in config["enable"]]
        enabled = list(enabled) + list(config["rules"])
        self.rules = [r for r in enabled if r.id not in config["disable"]]
        allows = list(ballows) + list(config["allow_rules"])
        self.allow_rules = [a for a in allows if a.id not in config["disable_allow"]]
        self.exclude_block = list(config["exclude_block"])

    def allow_path(self, path: str) -> bool:
        return _allow_path(self.allow_rules, path)

    # scanner.go:169-181
    @staticmethod
    def match_keywords(rule: Rule, content: bytes, lowered=None) -> bool:
        if not rule.keywords:
            return True
        low = go_bytes_to_lower(content) if lowered is None else lowered
        return any(go_bytes_to_lower(kw.encode()) in low for kw in rule.keywords)

    def _allow_location(self, rule, content, s, e) -> bool:  # scanner.go:145-148
        m = content[s:e]
        return _allow(self.allow_rules, m) or _allow(rule.allow_rules, m)

    def find_locations(self, rule, content):  # scanner.go:97-163
        if rule.regex is None:
            return []
        locs = []
        if not rule.secret_group_name:
            for s, e in rule.regex.find_all_index(content):
                if not self._allow_location(rule, content, s, e):
                    locs.append((s, e))
            return locs
        names = rule.regex.subexp_names()
        for idx in rule.regex.find_all_submatch_index(content):
            if self._allow_location(rule, content, idx[0], idx[1]):
                continue
            for g, name in enumerate(names):
                if name == rule.secret_group_name:
                    locs.append((idx[2 * g], idx[2 * g + 1]))
        return locs

    def scan(self, file_path: str, content: bytes, with_offsets=False):
        """Returns {"FilePath":..., "Findings":[...]} like types.Secret."""
        if self.allow_path(file_path):
            return {"FilePath": file_path, "Findings": []}
        censored = None
        matched = []
        gblocks = None
        lowered = None
        for rule in self.rules:
            if rule.path is not None and not rule.path.match_string(file_path.encode()):
                continue
            if _allow_path(rule.allow_rules, file_path):
                continue
            if rule.keywords and lowered is None:
                lowered = go_bytes_to_lower(content)
            if not self.match_keywords(rule, content, lowered):
                continue
            locs = self.find_locations(rule, content)
            if not locs:
                continue
            lblocks = None
            for (s, e) in locs:
                if gblocks is None:
                    gblocks = _blocks(content, self.exclude_block)
                if lblocks is None:
                    lblocks = _blocks(content, rule.exclude_block)
                if any(bs <= s and e <= be for bs, be in gblocks) or \
                        any(bs <= s and e <= be for bs, be in lblocks):
                    continue
                if s < 0:
                    raise IndexError("secret group did not participate (reference panics)")
                matched.append((rule, s, e))
                if censored is None:
                    censored = bytearray(content)
                censored[s:e] = b"*" * (e - s)
        findings = [_to_finding(r, s, e, bytes(censored)) for r, s, e in matched]
        if not findings:
            return {"FilePath": "", "Findings": []}
        findings.sort(key=lambda f: (f.RuleID.encode(), f.Match.encode("utf-8", "surrogateescape")))
        if not with_offsets:
            for f in findings:
                f.Start = f.End = -1
        return {"FilePath": file_path, "Findings": findings}


def _blocks(content, regexes):  # scanner.go:257-270
    locs = []
    for rx in regexes:
        for s, e in rx.find_all_index(content):
            locs.append((s, e))
    return locs


def _to_finding(rule, s, e, content) -> SecretFinding:  # scanner.go:464-477
    sl, el, code, match = find_location(s, e, content)
    return SecretFinding(RuleID=rule.id, Category=rule.category,
                         Severity=rule.severity or "UNKNOWN", Title=rule.title,
                         StartLine=sl, EndLine=el, Code=code, Match=match, Start=s, End=e)


def find_location(start, end, content: bytes):  # scanner.go:481-537
    start_line = content.count(b"\n", 0, start)
    ls = content.rfind(b"\n", 0, start)
    line_start = 0 if ls == -1 else ls + 1
    le = content.find(b"\n", start)
    line_end = len(content) if le == -1 else le
    if line_end - line_start > 100:
        line_start = max(start - 30, 0)
        line_end = min(end + 20, len(content))
    match_line = _s(content[line_start:line_end])
    end_line = start_line + content.count(b"\n", start, end)
    lines = content.split(b"\n")
    cs = max(start_line - 2, 0)
    ce = min(end_line + 2, len(lines))
    out = []
    found_first = False
    for i, raw in enumerate(lines[cs:ce]):
        real = cs + i
        cause = start_line <= real <= end_line
        txt = _s(raw)
        out.append(dataclasses.asdict(Line(Number=real + 1, Content=txt, IsCause=cause,
                                           Highlighted=txt, FirstCause=(not found_first) and cause)))
        found_first = found_first or cause
    for ln in reversed(out):
        if ln["IsCause"]:
            ln["LastCause"] = True
            break
    return start_line + 1, end_line + 1, {"Lines": out}, match_line


# --------------------------------------------------------------------------- #
# Analyzer front end — pkg/fanal/analyzer/secret/secret.go:28-153
# --------------------------------------------------------------------------- #

SKIP_FILES = ["go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
              "Pipfile.lock", "Gemfile.lock"]
SKIP_DIRS = [".git", "node_modules"]
SKIP_EXTS = [".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm",
             ".zip", ".gz", ".gzip", ".tar", ".pyc"]


def is_binary(head: bytes, size: int) -> bool:  # utils.go:77-95
    n = min(size, 300)
    for b in head[:n]:
        if b < 7 or b == 11 or (13 < b < 27) or (27 < b < 0x20) or b == 0x7F:
            return True
    return False


class SecretAnalyzer:
    def __init__(self, config_path: str = ""):
        self.config_path = config_path
        self.scanner = Scanner(parse_config(config_path))

    def required(self, file_path: str, size: int) -> bool:
        if size < 10:
            return False
        d, name = os.path.split(file_path)
        dirs = (d + "/" if d else "").split("/")
        if any(sd in dirs for sd in SKIP_DIRS):
            return False
        if name in SKIP_FILES:
            return False
        if os.path.basename(self.config_path) == file_path:
            return False
        ext = _go_ext(name)
        if ext in SKIP_EXTS:
            return False
        if self.scanner.allow_path(file_path):
            return False
        return True

    def analyze(self, file_path: str, content: bytes, dir_: str = ""):
        if is_binary(content, len(content)):
            return None
        content = content.replace(b"\r", b"")
        fp = file_path if dir_ != "" else "/" + file_path
        res = self.scanner.scan(fp, content)
        if not res["Findings"]:
            return None
        return [res]


def _go_ext(path: str) -> str:
    """filepath.Ext: suffix from the final dot in the final element."""
    for i in range(len(path) - 1, -1, -1):
        if path[i] == "/":
            break
        if path[i] == ".":
            return path[i:]
    return ""
