"""Inference facade (mlx_mcmc/inference/__init__.py)."""
from .mcmc import MCMC

__all__ = ["MCMC"]
