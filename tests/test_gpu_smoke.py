"""The driver's round-end smoke() (__graft_entry__.py) inside the GPU suite, so
a change that breaks it (e.g. a launch-count assertion the fused small-request
path no longer meets) fails here first.  The build-id check inside smoke()
ties the run to this tree."""
import pytest

pytestmark = pytest.mark.gpu


def test_graft_entry_smoke():
    import __graft_entry__ as g
    g.smoke()
