import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _ensure_pkg():
    """Import mlx_mcmc_amd from mlx-mcmc_amd/ even where the symlink is absent."""
    try:
        import mlx_mcmc_amd  # noqa: F401
    except ImportError:
        spec = importlib.util.spec_from_file_location(
            "mlx_mcmc_amd", os.path.join(ROOT, "mlx-mcmc_amd", "__init__.py"),
            submodule_search_locations=[os.path.join(ROOT, "mlx-mcmc_amd")])
        mod = importlib.util.module_from_spec(spec)
        sys.modules["mlx_mcmc_amd"] = mod
        spec.loader.exec_module(mod)


_ensure_pkg()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device")
    config.addinivalue_line("markers", "slow: long statistical run")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mlx_mcmc_amd import _lib

    _lib.load()
    return torch.device("cuda", 0)
