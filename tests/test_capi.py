"""The C-ABI boundary: libtwhip.so builds, loads, and exports exactly what include/tw_whisper.h and
include/tw_audio.h declare.
CPU only (no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDRS = [os.path.join(ROOT, "include", h) for h in ("tw_whisper.h", "tw_audio.h")]
LIB = os.path.join(ROOT, "turbo-whisper-workspace_amd", "twamd", "libtwhip.so")


def _declared():
    src = "".join(open(h).read() for h in HDRS)
    return sorted(set(re.findall(r"^(?:int|size_t|const char\*)\s+(tw_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib_path():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "turbo-whisper-workspace_amd", "csrc"), "-j8"], check=True,
                       capture_output=True)
    return LIB


def test_header_declares_entry_points():
    names = _declared()
    assert "tw_gemm_bf16" in names and "tw_logits_select" in names and len(names) >= 14


def test_library_exports_every_declared_symbol(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (tw_\w+)", out))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing


def test_library_loads_and_binding_matches(lib_path):
    import torch  # noqa: F401  (HIP runtime first, as the product loads it)
    from twamd import _lib

    lib = ctypes.CDLL(lib_path)
    assert lib.tw_version() == 1
    assert sorted(_lib.EXPORTED) == _declared()
    assert set(_lib._SIGS) == set(_declared())
    bound = _lib.load(lib_path)
    assert bound.tw_version() == 1


def test_errors_are_reported_not_raised_in_c(lib_path):
    import torch  # noqa: F401
    from twamd import _lib

    _lib.load(lib_path)
    with pytest.raises(_lib.TwError, match="K % 64"):
        _lib.call("tw_gemm_bf16", 1, 1, 16, 16, 48, 48, 48, 0, 1, 16, None, None, 0, None, None)
    with pytest.raises(_lib.TwError, match="null"):
        _lib.call("tw_logmel", None, 1, None, None, None, 80, None, None, None)


def test_debug_library_exports_the_same_abi_and_says_so():
    """libtwhip_dbg.so (make debug: -DTW_DEBUG=1, the C-ABI contract checks) exports the same symbols and reports
    itself as the debug build; the product library does not."""
    dbg = os.path.join(ROOT, "turbo-whisper-workspace_amd", "twamd", "libtwhip_dbg.so")
    # (incremental: rebuilds only what changed since the last debug build)
    subprocess.run(["make", "-C", os.path.join(ROOT, "turbo-whisper-workspace_amd", "csrc"), "-j8", "debug"],
                   check=True, capture_output=True)
    out = subprocess.run(["nm", "-D", "--defined-only", dbg], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (tw_\w+)", out))
    assert not [n for n in _declared() if n not in exported]
    import torch  # noqa: F401
    assert ctypes.CDLL(dbg).tw_debug_build() == 1
    assert ctypes.CDLL(LIB).tw_debug_build() == 0


def test_tw_lib_override_is_refused(monkeypatch):
    """The old A/B scripts' TW_LIB variable is refused, not silently ignored."""
    import torch  # noqa: F401
    from twamd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setenv("TW_LIB", "/tmp/other.so")
    with pytest.raises(_lib.TwError, match="TW_LIB"):
        _lib.load()
