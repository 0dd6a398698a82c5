import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _build_native(hip: bool = True):
    """Build libnutexec.so (hipcc, gfx950) and liboracle.so if missing or stale.
    nutdb_amd/build.py is loaded by path: importing the package needs the library."""
    import importlib.util
    if hip:
        spec = importlib.util.spec_from_file_location("_nut_build", ROOT / "nutdb_amd" / "build.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build()
    from oracle import oracle
    oracle.build()
    spec = importlib.util.spec_from_file_location("_nut_c_hosts", ROOT / "tests" / "c" / "build.py")
    hosts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(hosts)
    hosts.build()


def pytest_configure(config):
    # NUT_PREBUILT=1: use the shipped libnutexec.so as it is (a GPU box runs what was built
    # here, even when a source file was touched after the build)
    _build_native(hip=os.environ.get("NUT_PREBUILT") != "1")
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json
    return json.loads((ROOT / "tests" / "golden" / "executor_golden.json").read_text())


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ex():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    from nutdb_amd import Executor
    e = Executor(0)
    yield e
    e.close()


@pytest.fixture
def opts(ex):
    """Set nut_ctx options on the session executor for one test (the library reads no
    environment variables); every option is restored afterwards."""
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            old = ex.set_option(k, v)
            saved.setdefault(k, old)
    yield set_
    for k, v in saved.items():
        ex.set_option(k, v)
