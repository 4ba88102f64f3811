"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's sampling hot path (korentomas/mlx-mcmc
mlx_mcmc/kernels/hmc.py, kernels/nuts.py, distributions/normal.py,
distributions/halfnormal.py), used only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, always as the checker — never by the
product package mlx_mcmc_amd/ and never as the thing measured.

Pinning (see DESIGN.md "Oracle"): the reference cannot run here (its only
dependency, MLX >= 0.30, is not installed: ModuleNotFoundError), so the
restatement is pinned by every known-answer and statistical assertion the
reference's own tests hold for this path (tests/test_oracle_pins.py) and by
the Random123 known-answer vectors for the shared Philox stream.
"""
