"""The driver's round-end smoke (__graft_entry__.smoke: CIF I+2P through
evx1_encoder::encode() on cuda:0, bit-exact vs the oracle) as a GPU test, so
every GPU run exercises it before the driver does."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_graft_entry_smoke():
    sys.path.insert(0, ROOT)
    import __graft_entry__

    __graft_entry__.smoke()
