#!/usr/bin/env python3
"""Extract Trivy's builtin secret rules and builtin allow rules into JSON data.

Run in the build container (the only place /root/reference exists):

    python tools/extract_builtin_rules.py /root/reference

Reads  pkg/fanal/secret/builtin-rules.go:12-83 (categories + regex consts),
       pkg/fanal/secret/builtin-rules.go:95-823 (builtinRules),
       pkg/fanal/secret/builtin-allow-rules.go:3-65 (builtinAllowRules)
and writes trivy_amd/data/builtin_rules.json.  The JSON is rule *data*
(IDs, titles, regex sources with fmt.Sprintf expanded, keywords); the
regexes are compiled by our own Go-RE2 compiler (trivy_amd/csrc/gre_*).
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(__file__))
from go_literal import Call, Composite, Ident, find_block, go_unquote, parse_value  # noqa: E402


def expand(v, consts):
    if isinstance(v, str):
        return v
    if isinstance(v, Ident):
        return consts[v.name]
    if isinstance(v, Call):
        if v.name == "MustCompile":
            return expand(v.args[0], consts)
        if v.name == "fmt.Sprintf":
            fmt = expand(v.args[0], consts)
            args = [expand(a, consts) for a in v.args[1:]]
            assert fmt.count("%s") == len(args), (fmt, args)
            out = fmt
            for a in args:
                out = out.replace("%s", a.replace("%", "\x00"), 1)
            return out.replace("\x00", "%")
        if v.name == "types.SecretRuleCategory":
            return expand(v.args[0], consts)
    raise ValueError(f"cannot expand {v!r}")


def main(ref):
    src = open(os.path.join(ref, "pkg/fanal/secret/builtin-rules.go")).read()
    consts = {}
    # var ( CategoryX = types.SecretRuleCategory("X") ... )
    for m in re.finditer(r'(Category\w+)\s*=\s*types\.SecretRuleCategory\("([^"]*)"\)', src):
        consts[m.group(1)] = m.group(2)
    cblock = src[src.index("const ("):]
    cblock = cblock[:cblock.index("\n)")]
    for m in re.finditer(r'(\w+)\s*=\s*(`[^`]*`|"(?:\\.|[^"\\])*")', cblock):
        consts[m.group(1)] = go_unquote(m.group(2))

    lit = parse_value(find_block(src, "var builtinRules = []Rule"))
    rules = []
    for item in lit.items():
        f = item.fields()
        rules.append({
            "id": f["ID"],
            "category": expand(f.get("Category", ""), consts),
            "title": f.get("Title", ""),
            "severity": f.get("Severity", ""),
            "regex": expand(f["Regex"], consts),
            "keywords": list(f["Keywords"].items()) if "Keywords" in f else [],
            "secret_group_name": f.get("SecretGroupName", ""),
        })

    asrc = open(os.path.join(ref, "pkg/fanal/secret/builtin-allow-rules.go")).read()
    alit = parse_value(find_block(asrc, "var builtinAllowRules = []AllowRule"))
    allows = []
    for item in alit.items():
        f = item.fields()
        allows.append({
            "id": f["ID"],
            "description": f.get("Description", ""),
            "regex": expand(f["Regex"], consts) if "Regex" in f else None,
            "path": expand(f["Path"], consts) if "Path" in f else None,
        })

    out = {
        "source": "pkg/fanal/secret/builtin-rules.go:95-823, builtin-allow-rules.go:3-65 (trivy v2 snapshot)",
        "rules": rules,
        "allow_rules": allows,
    }
    dst = os.path.join(os.path.dirname(__file__), "..", "trivy_amd", "data", "builtin_rules.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)
        fh.write("\n")
    print(f"{len(rules)} rules, {len(allows)} allow rules -> {os.path.normpath(dst)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
