"""The documents' evidence exists: every profiles/..., tools/... and tests/...
path that DESIGN.md, README.md or INTEGRATION.md cites is in the tree (a
trailing `_*` family cites at least one matching file)."""
import re

import pytest

from conftest import ROOT

DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md"]
# repository paths only: the documents cite /root/reference files by their own
# relative paths too (include/packet_defs.h, tests/tas_unit/fastpath.c, ...)
PATH = re.compile(r"(?<![\w/.])((?:profiles/|tools/|tests/test_|tests/golden/|tests/c/|oracle/|tas_amd/|include/tasx_)"
                  r"[A-Za-z0-9_./*\-]*[A-Za-z0-9_*\-])")


# paths the documents name as absent ("there is no oracle/_ref")
ABSENT = {"oracle/_ref"}


def cited(doc):
    text = (ROOT / doc).read_text()
    return sorted({m.group(1).rstrip(".") for m in PATH.finditer(text)})


@pytest.mark.parametrize("doc", DOCS)
def test_cited_paths_exist(doc):
    missing = []
    for c in cited(doc):
        if c in ABSENT:
            continue
        if "*" in c or c.endswith("_"):
            pat = c if "*" in c else c + "*"
            if not list(ROOT.glob(pat)):
                missing.append(c)
        elif not (ROOT / c).exists():
            missing.append(c)
    assert not missing, missing


def test_docs_cite_evidence():
    assert len(cited("DESIGN.md")) >= 20
