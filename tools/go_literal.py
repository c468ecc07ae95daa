"""Minimal reader for the Go composite-literal subset used by Trivy's secret
rule tables and test tables.

Used only by the offline extraction tools in ``tools/`` (they run in the build
container where ``/root/reference`` exists) to turn the reference's Go data
tables into JSON fixtures.  Nothing under ``trivy_amd/`` imports this.

Supported grammar (enough for pkg/fanal/secret/builtin-rules.go,
builtin-allow-rules.go, scanner_test.go and analyzer/secret/secret_test.go):

    value   := string | int | bool | ident | call | composite
    string  := "..." (Go escapes) | `...`
    call    := ident '(' value {',' value} ')'      e.g. MustCompile(...), fmt.Sprintf(...)
    composite := [type] '{' [elem {',' elem} [',']] '}'
    elem    := [key ':'] value
"""
from __future__ import annotations

import re

_TOKEN = re.compile(
    r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:\\.|[^"\\\n])*")
  | (?P<num>-?\d+)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_.]*)
  | (?P<punct>\[\]|:=|[^\sA-Za-z0-9_`\x22])
    """,
    re.S | re.X,
)


def go_unquote(tok: str) -> str:
    """Decode a Go interpreted ("...") or raw (`...`) string literal."""
    if tok[0] == "`":
        return tok[1:-1]
    body = tok[1:-1]
    out = bytearray()
    i = 0
    while i < len(body):
        c = body[i]
        if c != "\\":
            out += c.encode("utf-8")
            i += 1
            continue
        n = body[i + 1]
        simple = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11,
                  "\\": 92, '"': 34, "'": 39}
        if n in simple:
            out.append(simple[n])
            i += 2
        elif n == "x":
            out.append(int(body[i + 2:i + 4], 16))
            i += 4
        elif n in "01234567":
            out.append(int(body[i + 1:i + 4], 8))
            i += 4
        elif n == "u":
            out += chr(int(body[i + 2:i + 6], 16)).encode("utf-8")
            i += 6
        elif n == "U":
            out += chr(int(body[i + 2:i + 10], 16)).encode("utf-8")
            i += 10
        else:
            raise ValueError(f"bad escape \\{n}")
    return out.decode("utf-8", "surrogateescape")


class Call:
    def __init__(self, name, args):
        self.name, self.args = name, args

    def __repr__(self):
        return f"Call({self.name},{self.args!r})"


class Ident:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"Ident({self.name})"


class Composite:
    """A Go composite literal: ``type`` may be None; ``elems`` is a list of
    (key or None, value)."""

    def __init__(self, type_, elems):
        self.type, self.elems = type_, elems

    def fields(self):
        return {k: v for k, v in self.elems if k is not None}

    def items(self):
        return [v for _, v in self.elems]

    def __repr__(self):
        return f"Composite({self.type},{self.elems!r})"


class Parser:
    def __init__(self, text: str):
        self.toks = []
        pos = 0
        while pos < len(text):
            m = _TOKEN.match(text, pos)
            if not m:
                raise ValueError(f"lex error at {text[pos:pos+40]!r}")
            pos = m.end()
            kind = m.lastgroup
            if kind == "ws":
                continue
            self.toks.append((kind, m.group(kind)))
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.toks[j] if j < len(self.toks) else (None, None)

    def take(self, val=None):
        t = self.toks[self.i]
        if val is not None and t[1] != val:
            raise ValueError(f"expected {val!r} got {t!r} near {self.toks[self.i-3:self.i+3]}")
        self.i += 1
        return t

    def value(self):
        kind, v = self.peek()
        if kind in ("raw", "str"):
            self.take()
            s = go_unquote(v)
            # Go string concatenation with '+'
            while self.peek()[1] == "+":
                self.take("+")
                s += self.value()
            return s
        if kind == "num":
            self.take()
            return int(v)
        if v == "&":
            self.take()
            return self.value()
        if v == "{":
            return self.composite(None)
        if v == "[]":
            self.take()
            tname = self.take()[1]
            return self.composite("[]" + tname)
        if kind == "ident":
            self.take()
            if v in ("true", "false"):
                return v == "true"
            if v == "nil":
                return None
            nk, nv = self.peek()
            if nv == "(":
                self.take("(")
                args = []
                while self.peek()[1] != ")":
                    args.append(self.value())
                    if self.peek()[1] == ",":
                        self.take(",")
                self.take(")")
                return Call(v, args)
            if nv == "{":
                return self.composite(v)
            if nv == "[":  # indexing, e.g. `want[0]` — not used by the tables we read
                raise ValueError("indexing unsupported")
            return Ident(v)
        raise ValueError(f"unexpected token {kind} {v!r}")

    def composite(self, type_):
        self.take("{")
        elems = []
        while self.peek()[1] != "}":
            kind, v = self.peek()
            key = None
            if kind == "ident" and self.peek(1)[1] == ":":
                key = v
                self.take()
                self.take(":")
            elems.append((key, self.value()))
            if self.peek()[1] == ",":
                self.take(",")
        self.take("}")
        return Composite(type_, elems)


def parse_value(text: str):
    p = Parser(text)
    return p.value()


def find_block(src: str, marker: str) -> str:
    """Return the text of the balanced-brace literal that starts at the first
    '{' after ``marker``."""
    start = src.index(marker)
    j = src.index("{", start + len(marker))
    depth = 0
    k = j
    in_raw = in_str = False
    while k < len(src):
        c = src[k]
        if in_raw:
            in_raw = c != "`"
        elif in_str:
            if c == "\\":
                k += 1
            elif c == '"':
                in_str = False
        elif c == "`":
            in_raw = True
        elif c == '"':
            in_str = True
        elif c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return src[j:k + 1]
        k += 1
    raise ValueError("unbalanced")
