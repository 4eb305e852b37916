"""CPU checks of the C ABI: the library loads, exports every symbol that
include/bote_hip.h declares, and its pure host helpers agree with the
reference's formulas.  No compute calls that need a GPU."""
import math
import re

import pytest

from fantoch_amd import _lib


def header_functions():
    src = open(_lib.INCLUDE_H).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bote_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header():
    L = _lib.lib()
    declared = header_functions()
    assert declared, "no functions parsed from include/bote_hip.h"
    for name in declared:
        assert hasattr(L, name), f"{name} declared in bote_hip.h but not exported"
    assert sorted(_lib.EXPORTS) == declared


def test_quorum_sizes_match_reference():
    # protocol.rs:122-137 and config.rs:531-548
    cases = [(_lib.FPAXOS, 3, 1, 2), (_lib.FPAXOS, 5, 2, 3), (_lib.EPAXOS, 3, 0, 2), (_lib.EPAXOS, 7, 0, 5),
             (_lib.EPAXOS, 13, 0, 9), (_lib.EPAXOS, 17, 0, 12), (_lib.ATLAS, 5, 1, 3), (_lib.ATLAS, 5, 2, 4),
             (_lib.TEMPO, 7, 1, 4), (_lib.TEMPO, 7, 2, 5), (_lib.TEMPO_TINY, 7, 1, 2), (_lib.TEMPO_TINY, 7, 2, 4)]
    for proto, n, f, want in cases:
        assert _lib.lib().bote_quorum_size(proto, n, f) == want
    assert _lib.lib().bote_quorum_size(99, 3, 1) == -1


def test_max_f_binomial_unrank():
    L = _lib.lib()
    assert [L.bote_max_f(n) for n in range(1, 8)] == [0, 1, 1, 2, 2, 2, 2]
    assert _lib.binomial(64, 7) == 621216192
    assert _lib.binomial(128, 6) == 5423611200 == math.comb(128, 6)
    assert _lib.binomial(20, 5) == 15504
    for r in (0, 1, 12345, 621216191):
        p = _lib.colex_unrank(r, 7, 64).tolist()
        assert sum(math.comb(x, j + 1) for j, x in enumerate(p)) == r and p == sorted(p)
    with pytest.raises(_lib.BoteError):
        _lib.colex_unrank(621216192, 7, 64)


def test_no_device_is_an_error_not_a_fallback():
    import numpy as np
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    import ctypes as C
    h = C.c_void_p()
    rc = _lib.lib().bote_planet_create(np.zeros(4, np.uint16), 2, 0, C.byref(h))
    assert rc == -6  # BOTE_E_NODEV


def test_out_of_range_latency_and_size_are_errors():
    """The device paths hold latencies in 14 bits (BOTE_MAX_LATENCY = 16383;
    the packed fast/group paths need <= 4095 and fall back to the exact
    generic kernel above it).  A larger latency, where the reference takes
    any u64, is refused with BOTE_E_RANGE when the planet is created, before
    any device call, so no eval/sweep entry point ever sees one."""
    import ctypes as C

    import numpy as np
    h = C.c_void_p()
    lat = np.zeros(9, np.uint16)
    lat[1] = 16384
    assert _lib.lib().bote_planet_create(lat, 3, 0, C.byref(h)) == -4  # BOTE_E_RANGE
    assert "16383" in _lib.lib().bote_last_error().decode()
    assert _lib.lib().bote_planet_create(np.zeros(129 * 129, np.uint16), 129, 0, C.byref(h)) == -4
    assert not h.value
