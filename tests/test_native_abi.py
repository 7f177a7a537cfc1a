"""The C-ABI library loads and exports every symbol include/pokegym_amd.h declares (no GPU calls)."""
import ctypes
import os
import re

import pytest

from pokegym_amd import _native, build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(REPO, "include", "pokegym_amd.h")).read()
    return sorted(set(re.findall(r"\b(pk_[a-z_0-9]+)\s*\(", hdr)))


def test_header_and_binding_agree():
    assert sorted(_native.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    path = build.build()
    lib = ctypes.CDLL(path)
    for sym in _declared():
        assert hasattr(lib, sym), sym
    assert lib.pk_abi_version() == _native.ABI_VERSION


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pokegym_amd.emulator import BatchedEmulator
    with pytest.raises(_native.PkError):
        BatchedEmulator(bytes(0x8000), 4)
