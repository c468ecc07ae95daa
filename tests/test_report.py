"""Trivy's JSON report of secret findings (trivy_amd/report.py) against the
reference's own golden report (integration/testdata/secrets.json.golden,
copied to tests/golden/integration): the same findings render to the same
bytes (pkg/report/json.go MarshalIndent, omitempty, Go string escaping).
The GPU variant renders what the engine itself found in the golden repo."""
import json
import os

import pytest

from .conftest import GOLDEN

R = pytest.importorskip("trivy_amd.report")
T = pytest.importorskip("trivy_amd.types")

GOLDEN_JSON = os.path.join(GOLDEN, "integration", "secrets.json.golden")


def _secrets_from_golden(g):
    out = []
    for res in g["Results"]:
        fs = []
        for f in res["Secrets"]:
            lines = [T.Line(**{k: v for k, v in ln.items()}) for ln in (f["Code"]["Lines"] or [])]
            fs.append(T.SecretFinding(RuleID=f["RuleID"], Category=f["Category"], Severity=f["Severity"],
                                      Title=f["Title"], StartLine=f["StartLine"], EndLine=f["EndLine"],
                                      Code=T.Code(Lines=lines), Match=f["Match"]))
        out.append(T.Secret(FilePath=res["Target"], Findings=fs))
    return out


def _render(g, secrets):
    return R.report_json(secrets, artifact_name=g["ArtifactName"], artifact_type=g["ArtifactType"],
                         created_at=g["CreatedAt"], metadata=g["Metadata"], schema_version=g["SchemaVersion"])


def test_golden_report_round_trip():
    text = open(GOLDEN_JSON, encoding="utf-8").read()
    g = json.loads(text)
    assert _render(g, _secrets_from_golden(g)) == text


def test_go_escaping_and_omitempty():
    f = T.SecretFinding(RuleID="r", Title="<a & b>", Match="x y", Code=T.Code(Lines=[]))
    out = R.dumps(R.secret_results([T.Secret(FilePath="p", Findings=[f]), T.Secret(FilePath="q")]))
    assert "\\u003ca \\u0026 b\\u003e" in out and "x\\u2028y" in out
    assert '"Lines": null' in out and '"Target": "q"' not in out
    ln = R.line_json(T.Line(Number=1, Content="", Highlighted=""))
    assert "Highlighted" not in ln and list(ln) == ["Number", "Content", "IsCause", "Annotation", "Truncated",
                                                    "FirstCause", "LastCause"]


def test_invalid_utf8_renders_as_go_does():
    """encoding/json (go1.22 encode.go appendString): utf8.DecodeRuneInString
    returns RuneError of width 1 for every byte that starts no valid sequence,
    and each such byte is written as the escape text \\ufffd; a valid U+FFFD
    (EF BF BD) is written raw.  Cases: a truncated 3-byte sequence, a lone
    continuation byte, an encoded surrogate (ED A0 80: three invalid bytes),
    an overlong NUL (C0 80), a byte that never starts a rune (FF).  Parity
    unpinned (no reference fixture holds invalid UTF-8): the expected text is
    Go's documented escaping rule restated here."""
    raw = b"a\xe2\x82b \x80 \xed\xa0\x80 \xc0\x80 \xff \xef\xbf\xbd z"
    s = raw.decode("utf-8", "surrogateescape")
    f = T.SecretFinding(RuleID="r", Match=s, Code=T.Code(Lines=[T.Line(Number=1, Content=s, Highlighted=s)]))
    out = R.dumps(R.secret_results([T.Secret(FilePath="p", Findings=[f])]))
    want = 'a\\ufffd\\ufffdb \\ufffd \\ufffd\\ufffd\\ufffd \\ufffd\\ufffd \\ufffd � z'
    assert out.count(want) == 3  # Match, Content, Highlighted
    out.encode("utf-8")  # no lone surrogate left


def test_invalid_utf8_dicts_keep_the_bytes():
    """secret_results' dicts keep invalid bytes as lone surrogates (report.py
    contract): dumps() renders Go's escapes from them, a surrogateescape
    encode gives back the scanned bytes, a strict encode refuses them."""
    raw = b"k=\xff\xfe \xe2\x84\xaa"
    s = raw.decode("utf-8", "surrogateescape")
    f = T.SecretFinding(RuleID="r", Match=s, Code=T.Code(Lines=[T.Line(Number=1, Content=s, Highlighted=s)]))
    d = R.secret_results([T.Secret(FilePath="p", Findings=[f])])
    m = d[0]["Secrets"][0]["Match"]
    assert m.encode("utf-8", "surrogateescape") == raw
    with pytest.raises(UnicodeEncodeError):
        m.encode("utf-8")
    out = R.dumps(d)
    assert out.count('k=\\ufffd\\ufffd \u212a') == 3
    out.encode("utf-8")


@pytest.mark.gpu
def test_gpu_findings_render_the_golden_report():
    from trivy_amd.analyzer import SecretAnalyzer

    text = open(GOLDEN_JSON, encoding="utf-8").read()
    g = json.loads(text)
    repo = os.path.join(GOLDEN, "integration", "repo")
    a = SecretAnalyzer()
    a.init(os.path.join(repo, "trivy-secret.yaml"))
    got = []
    for name in sorted(os.listdir(repo)):
        data = open(os.path.join(repo, name), "rb").read()
        if not a.required(name, len(data)):
            continue
        res = a.analyze(name, data, ".")
        for s in res or []:
            # AnalysisResult.Sort (analyzer.go:218-229): findings by (RuleID, StartLine)
            s.Findings.sort(key=lambda f: (f.RuleID, f.StartLine))
            got.append(s)
    assert _render(g, got) == text
