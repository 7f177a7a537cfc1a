"""Static properties of K1's gfx950 code that the round-5 analysis relies on (CPU: hipcc cross-compiles).

For every instance of both builds (default and small-LDS; PRIO x ALL), the main loop's common path
(tools/isa_count.py's walk: conditional branches not taken, s_branch followed) must
  * touch no scratch and move no spilled SGPR (the spills and flush_lines' stack frame stay on rare
    paths: profiles/r05/k1_resource_usage.txt);
  * issue its operand read without first draining the memory counter: no `s_waitcnt vmcnt(0)`
    between the loop header and the first image load — a rare path leaving a load outstanding made
    every iteration wait for the previous iteration's store acknowledgements there (PK_VM_DRAIN);
  * in the unstaged-bank instance, wait for the next-fetch global-ROM dwords with vmcnt(N>0), not
    vmcnt(0) (the branch-free stores of pk_write<BF>)."""
import os
import re
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "tools"))

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    import isa_count as IC
    out = {}
    d = tmp_path_factory.mktemp("k1isa")
    for small in (False, True):
        path = str(d / f"k{int(small)}.s")
        IC.compile_s(["-DPK_K1_SMALL"] if small else [], out=path)
        out[small] = open(path).read().splitlines()
    return out


def _common_path(lines, prio, all_, small):
    import k1_resources as KR
    return KR.common_path(lines, prio, all_, small)


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("prio", [0, 1])
@pytest.mark.parametrize("all_", [0, 1])
def test_k1_common_path_waits_and_spills(asm, small, prio, all_):
    p = _common_path(asm[small], prio, all_, small)
    assert len(p) > 300
    assert not [s for s in p if s.startswith("scratch_")]
    assert not [s for s in p if s.startswith("v_writelane") or s.startswith("v_readlane")]
    first_load = next(i for i, s in enumerate(p) if s.startswith("global_load_ubyte"))
    assert not [s for s in p[:first_load] if re.match(r"s_waitcnt .*vmcnt\(0\)", s)], p[:first_load]
    if not all_:
        rom = next(i for i, s in enumerate(p) if s.startswith("global_load_dwordx2"))
        later = [s for s in p[rom:] if "vmcnt(" in s]
        assert later and not re.search(r"vmcnt\(0\)", later[0]), later[:2]
