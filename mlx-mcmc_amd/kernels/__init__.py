"""Sampler kernels (mlx_mcmc/kernels/__init__.py): HMC and NUTS on MI355X."""
from .hmc import hmc
from .nuts import nuts

__all__ = ["hmc", "nuts"]
