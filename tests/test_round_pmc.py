"""tools/round_pmc.py: the PMC summaries bench.py cites (CPU)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_sane_drops_a_doubled_dispatch_row():
    """profiles/r06q: rocprofv3 once reported a 1,024-wave K1 dispatch as 2,048 waves with every
    counter of the row doubled; the means must not take it."""
    import round_pmc as RP
    v = {i: {"SQ_WAVES": 1024.0, "SQ_WAIT_ANY": 10.0} for i in (1, 2, 3, 4, 5)}
    v[4] = {"SQ_WAVES": 2048.0, "SQ_WAIT_ANY": 20.0}
    s = RP.sane(v)
    assert sorted(s) == [1, 2, 3, 5]
    assert RP.mean(s, "SQ_WAIT_ANY") == 10.0 and RP.mean(s, "SQ_WAVES") == 1024.0
    # passes without SQ_WAVES (FETCH_SIZE, WRITE_SIZE) are left alone
    f = {1: {"FETCH_SIZE": 1.0}, 2: {"FETCH_SIZE": 3.0}}
    assert RP.sane(f) == f
