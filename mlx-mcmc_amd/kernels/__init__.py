"""Sampler kernels (mlx_mcmc/kernels/__init__.py): HMC, NUTS and
Metropolis-Hastings on MI355X."""
from .hmc import hmc
from .metropolis import metropolis_hastings
from .nuts import nuts

__all__ = ["hmc", "nuts", "metropolis_hastings"]
