"""CPU: the documents cite evidence that exists.  Every `profiles/...`, `tools/...` and `tests/...` path
named in DESIGN.md, README.md, HISTORY.md and INTEGRATION.md is in the tree (globs and placeholders such
as KEY excepted), and DESIGN.md stays a design document of at most 500 lines (the round history lives in
HISTORY.md)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "HISTORY.md", "INTEGRATION.md"]
DELETED = {"tools/gpu_r4_[a-z].sh"}  # named by HISTORY.md as deleted in round 5


def cited(doc):
    text = open(os.path.join(ROOT, doc)).read()
    for m in re.findall(r"`((?:profiles|tools|tests)/[^`\s]+?)`", text):
        p = m.rstrip("/").split("::")[0]
        if "KEY" in p or "DIR" in p or "<" in p or p in DELETED:
            continue
        yield p


@pytest.mark.parametrize("doc", DOCS)
def test_cited_paths_exist(doc):
    missing = []
    for p in cited(doc):
        full = os.path.join(ROOT, p)
        if any(c in p for c in "*?["):
            if not glob.glob(full, recursive=True):
                missing.append(p)
        elif not os.path.exists(full):
            missing.append(p)
    assert not missing, (doc, missing)


def test_design_is_short():
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        assert sum(1 for _ in f) <= 500
