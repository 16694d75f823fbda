import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the built penroz_kernels extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture
def workdir(tmp_path, monkeypatch):
    """Run a test inside an isolated cwd with its own models/ and data/ folders and SHM dir."""
    monkeypatch.chdir(tmp_path)
    import penroz.utils.loaders as loaders
    monkeypatch.setattr(loaders, "DATA_FOLDER", str(tmp_path / "data"))
    os.makedirs(tmp_path / "data", exist_ok=True)
    from penroz.models.model import NeuralNetworkModel
    shm = tmp_path / "shm"
    shm.mkdir()
    monkeypatch.setattr(NeuralNetworkModel, "SHM_PATH", str(shm))
    return tmp_path


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    """A plain ``pytest tests`` on a machine without a GPU skips the ``gpu``-marked tests instead
    of failing them (``-m gpu`` on the MI355X runs them all)."""
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="needs an MI355X (no HIP device visible)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
