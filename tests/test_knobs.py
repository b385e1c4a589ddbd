"""The native libraries read only documented environment variables (docs/ARCHITECTURE.md,
"Environment variables"): test and modelling switches go through gs_debug_set instead
(csrc/include/gs/debug.h), so a stray variable cannot change the shipped kernels."""
import glob
import os
import re

from grayscott_amd.ops import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _getenv_names():
    names = set()
    srcs = [f for pat in ("csrc/**/*.h", "csrc/**/*.hpp", "csrc/**/*.hip", "csrc/**/*.cpp")
            for f in glob.glob(os.path.join(ROOT, pat), recursive=True)
            if "/tools/" not in f]  # micro-benchmarks and self-tests are not shipped
    for f in srcs:
        names |= set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', open(f).read()))
    return names


def test_every_native_getenv_is_documented():
    doc = open(os.path.join(ROOT, "docs", "ARCHITECTURE.md")).read()
    table = doc.split("## Environment variables")[1].split("\n## ")[0]
    names = _getenv_names()
    assert names, "no getenv found: the scan is broken"
    missing = sorted(n for n in names if f"`{n}" not in table)
    assert not missing, f"undocumented environment variables read by native code: {missing}"


def test_test_switches_are_not_environment_variables():
    names = _getenv_names()
    for gone in ("GS_IPC_EMULATE_US", "GS_OVERLAP_CHAIN", "GS_PHILOX_GENERIC"):
        assert gone not in names


def test_debug_set_core_library():
    native.debug_set("overlap_chain", 0, "core")
    native.debug_set("overlap_chain", 1, "core")
    import pytest
    with pytest.raises(ValueError):
        native.debug_set("no_such_switch", 1, "core")
