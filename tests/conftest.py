import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fabric-token-sdk_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
PP_PATH = os.path.join(GOLDEN, "zkatdlog_pp.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels of libfts_gpu.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def pp_raw():
    with open(PP_PATH, "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def oracle_pp(pp_raw):
    from oracle import pp as ppm
    return ppm.load_pp(pp_raw)


_GPU_CTX = {}


@pytest.fixture(scope="session")
def gpu_pp(pp_raw):
    """factory: device contexts per bit length (device 0), shared by the session"""
    import fts_gpu

    def get(bits):
        if bits not in _GPU_CTX:
            _GPU_CTX[bits] = fts_gpu.PublicParams(pp_raw, bit_length=bits, device=0)
        return _GPU_CTX[bits]
    return get


_HOST_CTX = {}


@pytest.fixture(scope="session")
def host_pp(pp_raw):
    """factory: host-only contexts (prover, parsing; no GPU)"""
    import fts_gpu

    def get(bits):
        if bits not in _HOST_CTX:
            _HOST_CTX[bits] = fts_gpu.PublicParams(pp_raw, bit_length=bits, device=fts_gpu.FTS_DEVICE_NONE)
        return _HOST_CTX[bits]
    return get
