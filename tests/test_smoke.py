"""__graft_entry__.smoke() as a GPU test, so the suite catches what the driver's smoke run would."""
import sys

import pytest

from conftest import ROOT


@pytest.mark.gpu
def test_graft_entry_smoke():
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as g

    g.smoke()
