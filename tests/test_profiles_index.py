"""profiles/ stays an index of evidence, not an archive: every file under
profiles/ is listed in profiles/INDEX.md under the claim it backs, INDEX.md is current, and every
profiles file the docs, headers and product sources cite exists (brace and <config> patterns expanded)."""
import fnmatch
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import profiles_index  # noqa: E402


def test_index_lists_every_file_and_is_current():
    assert profiles_index.check() == []


def _expand(t):
    m = re.search(r"\{([^{}]*)\}", t)
    if not m:
        return [t]
    return [x for alt in m.group(1).split(",") for x in _expand(t[:m.start()] + alt + t[m.end():])]


CITING = ["DESIGN.md", "README.md", "INTEGRATION.md", "include/nexr.h", "include/nexr_ring.h", "include/nexr_extras.h"]
CITING_DIRS = ["nex-nccl_amd/csrc"]


def _citing_files():
    out = [os.path.join(ROOT, f) for f in CITING]
    for d in CITING_DIRS:
        out += [os.path.join(ROOT, d, f) for f in sorted(os.listdir(os.path.join(ROOT, d)))
                if f.endswith((".cpp", ".h", ".hpp", ".hip"))]
    return out


@pytest.mark.parametrize("path", _citing_files(), ids=lambda p: os.path.relpath(p, ROOT))
def test_citations_resolve(path):
    """Every profiles/ file DESIGN.md, README.md, INTEGRATION.md, the headers and the product
    sources' comments cite exists (a comment cited a file that was never committed)."""
    text = open(path).read()
    files = os.listdir(os.path.join(ROOT, "profiles"))
    toks = set(re.findall(r"`(?:profiles/)?((?:r0\d|pmc_)[^`\s]*)`", text)) if path.endswith(".md") else set()
    toks |= {t for t in re.findall(r"profiles/([^\s`]+)", text)}
    missing = []
    for t in toks:
        t = t.rstrip(".,;:)")
        if "{" in t and "}" not in t:
            continue  # a brace list cut by the prose regex; the backticked form is checked
        pats = [re.sub(r"<[^>]*>", "*", e) for e in _expand(t)]
        if not any(fnmatch.fnmatch(f, p) or fnmatch.fnmatch(f, p + "*") for p in pats for f in files):
            missing.append(t)
    assert not missing, missing
