"""CPU-side checks of the C-ABI library: it loads, exports every entry point
include/*.h declares, and the Python binding covers exactly those."""

import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))


INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")


def _header_text() -> str:
    return "\n".join(open(h).read() for h in HEADERS)


def header_functions():
    text = _header_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(agx_[a-z0-9_]+)\s*\(", text)))


def _top_level_args(s: str, start: int) -> tuple[int, str]:
    """Argument text of the call whose '(' is at s[start]: (end index, text)."""
    depth = 0
    for i in range(start, len(s)):
        if s[i] in "([{":
            depth += 1
        elif s[i] in ")]}":
            depth -= 1
            if depth == 0:
                return i, s[start + 1:i]
    raise ValueError("unbalanced call")


def _count_args(text: str) -> int:
    text = text.strip()
    if text in ("", "void"):
        return 0
    depth, n = 0, 1
    for ch in text:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            n += 1
    return n


def header_arity() -> dict[str, int]:
    text = re.sub(r"/\*.*?\*/", "", _header_text(), flags=re.S)
    return {m.group(1): _count_args(m.group(2))
            for m in re.finditer(r"\b(agx_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S)}


@pytest.fixture(scope="module")
def lib():
    from agilerl_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    return _lib.load(require_gpu=False)


def test_header_parses():
    fns = header_functions()
    assert "agx_gae" in fns and "agx_per_sample" in fns and len(fns) >= 18


def test_library_exports_every_header_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_binding_matches_header():
    from agilerl_amd import _lib

    assert sorted(_lib.SIGNATURES) == header_functions()


def test_error_path_without_gpu_work(lib):
    assert lib.agx_version() >= 100
    # argument validation happens before any HIP call
    rc = lib.agx_gae(None, None, None, None, None, 0, 0, 0, 0.99, 0.95, 1, None, None, None, None, None)
    assert rc == -1
    assert b"empty shape" in lib.agx_last_error()
    rc = lib.agx_per_init(None, None, 3, None)
    assert rc == -1 and b"power of 2" in lib.agx_last_error()
    rc = lib.agx_c51_project_loss(*([None] * 7), 1, 1, 1, 0.0, 1.0, 0.9, None, None, None)
    assert rc == -1


def test_library_is_gfx950_code_object():
    from agilerl_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_integration_doc_calls_match_header():
    """Every agx_* call INTEGRATION.md quotes (code blocks and inline) names a
    header function and passes its number of arguments ('...' elisions are
    checked by name only)."""
    arity = header_arity()
    doc = open(INTEGRATION).read()
    seen = 0
    for m in re.finditer(r"\b(agx_[a-z0-9_]+)\(", doc):
        name = m.group(1)
        assert name in arity, f"INTEGRATION.md calls {name}, which include/*.h does not declare"
        _, args = _top_level_args(doc, m.end() - 1)
        if "..." in args:
            continue
        assert _count_args(args) == arity[name], \
            f"INTEGRATION.md: {name}({args.strip()[:60]}...) has {_count_args(args)} arguments, the header {arity[name]}"
        seen += 1
    assert seen >= 12
