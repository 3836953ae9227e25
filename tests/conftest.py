import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernel)")


def _build():
    jobs = str(min(16, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", str(ROOT / "my-raytracer_amd")], check=True)
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    libs = [ROOT / "my-raytracer_amd/lib/librt_hip.so", ROOT / "my-raytracer_amd/lib/librt_host.so",
            ROOT / "oracle/_build/liboracle.so"]
    if not all(p.exists() for p in libs):
        _build()
    return True


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("tests marked gpu need an MI355X; run the CPU suite with -m 'not gpu'")
    return True
