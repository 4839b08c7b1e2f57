"""Runs last in the GPU suite (file order): the product library answered every drop-in ether_fcs
call of this session on the GPU. fcs_engine_host_fallbacks counts the calls its host CRC answered
(only after the GPU attempt and its retry both failed, or for buffers >= 4 GiB); on a
healthy MI355X it must be 0, which shows the HIP path served every drop-in call of the suite.
fcs_engine_host_batches counts the host batch calls (ether_fcs_*_host, and through them the TX/RX
queue batches of test_gpu_txq.py, test_gpu_rxq.py and the pcap/RX paths) its host CRC answered after
a failed GPU step; it must be 0 too: every host batch call of the suite ran on the GPU. The
fault-injection tests use the separate libnstack_fcs_faults.so."""
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu


def test_product_library_never_used_its_host_crc():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert na.ether_fcs(b"123456789") == 0xCBF43926
    st = na.engine_stats()
    assert st["dropin_calls"] > 0
    assert st["host_fallbacks"] == 0, st
    assert st["host_batches"] == 0, st
