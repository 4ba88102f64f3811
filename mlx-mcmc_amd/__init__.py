"""mlx_mcmc_amd — MI355X-native HMC/NUTS engine with the mlx-mcmc API.

Drop-in for the sampling hot path of korentomas/mlx-mcmc
(mlx_mcmc/__init__.py:24-46): ``Normal``, ``HalfNormal``, ``Exponential``,
``Gamma``, ``Beta``, ``Distribution``,
``hmc``, ``nuts``, ``metropolis_hastings``, ``MCMC``; ``mlx_mcmc_amd.core`` replaces ``mlx.core`` in
user models (``import mlx_mcmc_amd.core as mx``).  Sampling runs in the HIP
kernels of libmcmc355.so (csrc/); there is no CPU fallback.
"""
from . import core, random
from .distributions import Beta, Distribution, Exponential, Gamma, HalfNormal, Normal
from .kernels import hmc, metropolis_hastings, nuts
from .inference import MCMC
from .diagnostics import compute_ess

__version__ = "0.1.0"

__all__ = ["Distribution", "Normal", "HalfNormal", "Exponential", "Gamma", "Beta", "hmc",
           "nuts", "metropolis_hastings", "MCMC", "core", "random", "compute_ess"]
