"""Output records — pkg/fanal/types/secret.go:5-20 and misconf.go:49-62."""
from __future__ import annotations

import dataclasses
from typing import List


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
class Code:
    Lines: List[Line] = dataclasses.field(default_factory=list)


@dataclasses.dataclass
class SecretFinding:
    RuleID: str = ""
    Category: str = ""
    Severity: str = ""
    Title: str = ""
    StartLine: int = 0
    EndLine: int = 0
    Code: Code = dataclasses.field(default_factory=Code)
    Match: str = ""


@dataclasses.dataclass
class Secret:
    FilePath: str = ""
    Findings: List[SecretFinding] = dataclasses.field(default_factory=list)

    def to_dict(self):
        return dataclasses.asdict(self)
