"""trivy_amd — MI355X-native backend for Trivy's secret-scanning hot path.

Public API mirrors pkg/fanal/secret (parse_config, new_scanner, Scanner.scan)
and pkg/fanal/analyzer/secret (SecretAnalyzer); see DESIGN.md.
"""
from .types import Code, Line, Secret, SecretFinding  # noqa: F401

__all__ = ["Code", "Line", "Secret", "SecretFinding"]
