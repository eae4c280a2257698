"""Every measurement record the documents cite is in the tree: each `profiles/<name>` mentioned in
DESIGN.md, README.md or INTEGRATION.md exists (a `*` in the name is a glob that must match)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "README.md", "INTEGRATION.md")


def _refs(doc):
    text = open(os.path.join(ROOT, doc)).read()
    return sorted(set(re.findall(r"profiles/([A-Za-z0-9_.*\-]+[A-Za-z0-9*])", text)))


@pytest.mark.parametrize("doc", DOCS)
def test_cited_profiles_exist(doc):
    missing = [r for r in _refs(doc) if not glob.glob(os.path.join(ROOT, "profiles", r))]
    assert not missing, f"{doc} cites profiles/ records that are not in the tree: {missing}"


def test_session_index_lists_every_script():
    sessions = os.path.join(ROOT, "tools", "sessions")
    index = open(os.path.join(sessions, "INDEX.md")).read()
    scripts = sorted(f for f in os.listdir(sessions) if f.endswith(".sh"))
    assert scripts
    unlisted = [f for f in scripts if f"`{f}`" not in index]
    assert not unlisted, f"tools/sessions/INDEX.md does not list {unlisted}"
