"""Every repository path the design and integration documents cite resolves (evidence paths
must survive pruning of profiles/)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOPS = "profiles|tools|tests|oracle|include|4d_ray_tracing_amd|scenes"
NOT_FILES = {"oracle/_ref"}  # named as what could not be built


def cited(doc):
    s = open(os.path.join(ROOT, doc)).read()
    paths = set(re.findall(rf"`((?:{TOPS})/[^`\s:]+)`", s)) | set(re.findall(r"\((profiles/[^)\s:,]+)", s))
    return sorted(p.rstrip(".,;") for p in paths)


@pytest.mark.parametrize("doc", ["DESIGN.md", "INTEGRATION.md", "README.md"])
def test_cited_paths_resolve(doc):
    if not os.path.exists(os.path.join(ROOT, doc)):
        pytest.skip(f"{doc} absent")
    missing = []
    for p in cited(doc):
        if p in NOT_FILES:
            continue
        pat = re.sub(r"\{[^}]*\}|<[^>]*>|\*", "*", p)
        if not glob.glob(os.path.join(ROOT, pat)):
            missing.append(p)
    assert not missing, f"{doc} cites paths that do not exist: {missing}"
