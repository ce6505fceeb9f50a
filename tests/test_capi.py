"""The C-ABI library builds, loads and exports every entry point include/pinot_amd.h declares (no GPU calls)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "pinot_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pa_[a-z_0-9]+)\s*\(", src)))


def test_header_matches_binding():
    from pinot_amd import _lib
    assert _declared() == sorted(_lib.EXPORTED)


def test_library_exports_every_symbol():
    from pinot_amd import build, _lib
    path = build.build()
    lib = ctypes.CDLL(path)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing
    assert _lib.lib().pa_abi_version() == _lib.ABI_VERSION


def test_struct_layout_matches_header():
    """ctypes mirrors of the C structs have the sizes the compiled library expects."""
    from pinot_amd import _lib as L
    # pa_query_spec: 4 + 16*8 + 4 + 48*4 + 4 + 8*4 (+4 pad) + 8*8 + 4 (+4 pad) + 16*24 + 4 + 4
    assert ctypes.sizeof(L.LeafSpec) == 8
    assert ctypes.sizeof(L.AggSpec) == 24
    assert ctypes.sizeof(L.LeafParams) == 72  # (+ RAW_SET values, num_values: ABI 4)
    assert ctypes.sizeof(L.QuerySpec) == 848  # (+ flags2, reserved2)


def test_product_path_does_not_import_oracle():
    """The oracle is a checker only: nothing under pinot_amd/ may import, link or execute it."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "pinot_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text and "liboracle" not in text, f


def test_jit_descriptors_have_one_definition():
    """The hiprtc kernels' descriptors (JitSeg, JitArgs, PveSeg, PveArgs) have one definition, pa_jit_abi.h, with its
    layout static_asserts: the host includes it and build.py pastes it into the kernels' source strings, so no kernel
    source defines a copy of its own (round 5 kept hand-mirrored host structs)."""
    from pinot_amd import build
    csrc = os.path.join(ROOT, "pinot_amd", "csrc")
    abi = open(os.path.join(csrc, build.JIT_ABI)).read()
    assert "static_assert(sizeof(JitSeg)" in abi and "static_assert(sizeof(PveSeg)" in abi
    for name in build.JIT_SOURCES:
        raw = open(os.path.join(csrc, name)).read()
        assert '#include "%s"' % build.JIT_ABI in raw, name
        for st in ("struct JitSeg", "struct JitArgs", "struct PveSeg", "struct PveArgs"):
            assert st not in raw, (name, st)
        text = build.jit_source_text(name)
        assert abi.replace("#pragma once\n", "") in text and '#include "' not in text, name
    assert '#include "%s"' % build.JIT_ABI in open(os.path.join(csrc, "pa_host.h")).read()
