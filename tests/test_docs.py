"""The evidence files and scripts the documents cite exist (profiles/r0N_*, tools/...)."""
import os
import re

from conftest import REPO

DOCS = ("DESIGN.md", "README.md", "INTEGRATION.md")


def _text():
    return "\n".join(open(os.path.join(REPO, d)).read() for d in DOCS)


def test_cited_profiles_exist():
    refs = set(re.findall(r"\b(r0[1-9]_[A-Za-z0-9_.\-]+\.(?:json|txt|log|csv))", _text()))
    missing = sorted(r for r in refs if not os.path.exists(os.path.join(REPO, "profiles", r)))
    assert refs and not missing, missing


def test_cited_tools_exist():
    refs = set(re.findall(r"\btools/[A-Za-z0-9_/.\-]+\.(?:py|sh|hip)", _text()))
    missing = sorted(r for r in refs if not os.path.exists(os.path.join(REPO, r)))
    assert refs and not missing, missing
