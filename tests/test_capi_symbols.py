"""The C-ABI library loads on a CPU-only host and exports every symbol include/fakepta_amd.h
declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fakepta_amd.h")
LIB = os.path.join(ROOT, "fakepta_amd", "lib", "libfakepta_amd.so")


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "fakepta_amd", "csrc")], check=True)


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|fpta_ctx\*)\s+(fpta_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_api():
    names = declared()
    assert "fpta_gp_accumulate" in names and "fpta_batch_synth" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_binding_covers_header():
    from fakepta_amd import _capi
    assert sorted(_capi.EXPORTED) == declared()


def test_version_and_errors_without_gpu():
    from fakepta_amd import _capi
    assert _capi._lib.fpta_version() == 10200  # FPTA_VERSION: ABI 1, behaviour revision 2
    # no device here: creation fails loudly with a message, never silently
    if _capi.device_count() == 0:
        with pytest.raises(_capi.FptaError):
            _capi.Context(0)
        with pytest.raises(_capi.FptaError):
            _capi.MultiContext([0, 0])


def test_release_build_reads_no_environment():
    """The shipped library is the release build and its code reads no FPTA_* environment variable
    (debug switches live in the separate -DFPTA_DEBUG build, which bench.py refuses)."""
    from fakepta_amd import _capi
    assert _capi.build_flags() == 0
    csrc = os.path.join(ROOT, "fakepta_amd", "csrc")
    for name in os.listdir(csrc):
        if name.endswith((".hip", ".h")):
            assert "getenv" not in open(os.path.join(csrc, name)).read(), name


def test_built_for_gfx950():
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
