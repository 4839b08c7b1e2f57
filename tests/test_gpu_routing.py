"""The kernel a fixed-length batch launches is the kernel the route names.

fcs::route_fixed (nstack_amd/csrc/fcs_launch.hpp) is the one function that decides the route:
launch_fixed sizes the grid and leases the work counter from it, fcs::launch_fixed_route launches
the kernel it names and records, in the branch that launches, what it launched
(fcs_debug_last_fixed_launch), and fcs_debug_fixed_route names it without a device call. This test
runs every band edge of tests/test_routing.py's table on the GPU and checks, per batch, that the
launched kernel equals the route and that every CRC equals the oracle's.

The small-batch threshold is lowered to 256 frames so that the "big" routes (short, flat) apply to
batches of a few hundred frames; the slot kernels' own conditions (the arena holds two slots, the
item's frames fit the slot) are met by these batches as by the table's 1 M-frame ones.
"""
import numpy as np
import pytest

import nstack_amd as na
from test_routing import PACKED

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

THRESHOLD = 256


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = na.set_var_threshold(THRESHOLD)
    yield torch.device("cuda", 0)
    na.set_var_threshold(old)


def _run(dev, oracle, L, stride, n, align=0):
    size = (n - 1) * stride + L + align
    host = np.random.default_rng(L * 7 + stride + n).integers(0, 256, max(size, 1), dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    base = d.data_ptr() + align
    route = na.fixed_route(base, stride, L, n)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(base, stride, L, n, out)
    torch.cuda.synchronize()
    launched = na.last_fixed_launch()
    exp = np.zeros(n, dtype=np.uint32)
    oracle.oracle_fcs_fixed(host[align:].ctypes.data, stride, L, n, exp.ctypes.data, 1, 8)
    got = out.cpu().numpy().view(np.uint32)
    return route, launched, np.array_equal(got, exp)


@pytest.mark.parametrize("L", sorted(PACKED))
def test_packed_band_edges_launch_their_route(dev, oracle, L):
    n = THRESHOLD + 45 if L <= 9000 else THRESHOLD + 1
    route, launched, exact = _run(dev, oracle, L, L, n)
    assert route == PACKED[L], (route, PACKED[L])        # the same decision as the 1 M-frame table
    assert launched.split("/")[0] == route, (launched, route)
    assert exact


@pytest.mark.parametrize("L,stride,want", [
    (1518, 2048, "single"), (500, 2000, "flat"), (1000, 2049, "flat"), (1600, 1700, "wide16:26"),
    (1600, 1851, "wide16:32"), (64, 4096, "short:16"), (0, 4, "flat"), (1518, 1518, "lds-dma"),
])
def test_strided_routes(dev, oracle, L, stride, want):
    route, launched, exact = _run(dev, oracle, L, stride, THRESHOLD + 33, align=3)
    assert route == want
    assert launched.split("/")[0] == route
    assert exact


@pytest.mark.parametrize("L,stride,n,want", [
    (64, 64, THRESHOLD, "generic"), (64, 64, THRESHOLD + 1, "short:16"), (1518, 1518, 100, "lds-dma"),
    (1518, 1518, 2, "single"), (100, 100, 1, "tiny"), (9000, 9000, 3, "segment:30"), (3049, 3049, 50, "segment:26"), (1600, 5000, 50, "generic"),
])
def test_small_batch_routes(dev, oracle, L, stride, n, want):
    route, launched, exact = _run(dev, oracle, L, stride, n)
    assert route == want
    assert launched.split("/")[0] == route
    assert exact
