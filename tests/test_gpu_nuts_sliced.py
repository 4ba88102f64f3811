"""The sliced NUTS kernel k_nuts_sl (csrc/nuts_sliced.h; reference
nuts.py:16-358): a chain's log density split over S data slices, one wave
per (chain, slice), one record exchange per leaf.

Parity bars (the oracle, oracle/samplers.py nuts, restating nuts.py):
  * strict replay: the oracle re-runs a chain with the GPU's own step-size
    sequence; tree depths and leaf counts agree at every compared iteration
    until a decision flips, and a flip is allowed only where the oracle
    proves a near-tie (tests/test_gpu_nuts_trace.py `_replay`); the GPU's
    dual averaging recomputed from its own acceptance statistics reproduces
    its step sizes;
  * the same trees as the tape kernel k_nuts until a near-tie (both are
    restatements with different fp32 summation orders);
  * bit-identical across chain splits (chain_offset), launch splits, dead
    waves of a partial chain block, and the 8 / 16-slice layouts' own reruns;
  * the exchange timeout path reported (MC_ERR_TIMEOUT) like the sliced HMC
    kernels'.
The Large-shape fixtures (fixed step size, and dual averaging acting) are in
tests/test_gpu_nuts_trace.py.
"""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _run(lp, init, C, slices, *, W_=10, S_=10, eps=5e-3, adapt=True, offset=0, seed=3,
         tape=False, maxj=10):
    import mlx_mcmc_amd as m

    s, rate, info = m.nuts(lp, init, num_samples=S_, num_warmup=W_, step_size=eps,
                           max_tree_depth=maxj, adapt_step_size=adapt, target_accept=0.65,
                           key=m.random.key(seed), num_chains=C, chain_offset=offset,
                           progress=False, return_info=True, return_trace=True,
                           keep_on_device=True, num_slices=slices,
                           nuts_kernel="tape" if tape else "auto")
    return info


@pytest.mark.parametrize("slices", [4, 8, 16])
def test_sliced_kernel_selected(gpu, slices):
    from mlx_mcmc_amd import _trace

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    prog = _trace.compile_model(lp, init, slices=slices)
    assert prog.num_slices == slices
    assert prog.nuts_kernel(10) == "sliced"
    # beyond the record layout's depth the tape kernel runs
    assert prog.nuts_kernel(13) == "tape"


@pytest.mark.parametrize("slices", [4, 8, 16])
def test_sliced_medium_against_oracle(gpu, slices):
    """Medium hierarchical model (D = 100, N = 10 K) with dual averaging: the
    strict oracle replay of chains 0 and 5 (test_gpu_nuts_trace._replay)."""
    from test_gpu_nuts_trace import _replay

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    info = _run(lp, init, 8, slices, W_=10, S_=10, eps=5e-3)
    assert info.extra["kernel"] == "sliced"
    cfg = dict(num_warmup=10, num_samples=10, step_size=5e-3, max_tree_depth=10,
               target_accept=0.65, seed=3)
    depths = []
    for chain in (0, 5):
        same, d, _ = _replay("medium", {"config": cfg}, info, 0, chain)
        depths.extend(d.tolist())
    assert max(depths) >= 3, "real trees"


def test_sliced_matches_tape_kernel(gpu):
    """k_nuts_sl and k_nuts (the tape) on the same chains: identical trees
    until the first iteration where either's decision sits at a near-tie of
    the oracle's own margins — checked here as: identical for at least the
    first 6 iterations of every chain at a fixed step size, where neither
    side adapts."""
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    a = _run(lp, init, 8, 8, W_=4, S_=6, eps=4e-3, adapt=False)
    b = _run(lp, init, 8, 0, W_=4, S_=6, eps=4e-3, adapt=False, tape=True)
    assert a.extra["kernel"] == "sliced" and b.extra["kernel"] == "tape"
    ta, tb = a.trace, b.trace
    for c in range(8):
        n = 0
        while n < 10 and (ta["tree_depth"][c][n] == tb["tree_depth"][c][n]
                          and ta["n_leapfrog"][c][n] == tb["n_leapfrog"][c][n]):
            n += 1
        assert n >= 6, (c, ta["tree_depth"][c], tb["tree_depth"][c])
        np.testing.assert_allclose(ta["energy"][c][:n], tb["energy"][c][:n], rtol=1e-5)
    assert ta["tree_depth"].max() >= 4


def test_sliced_chain_split_and_dead_waves(gpu):
    """20 chains (the third chain block of 8 has 4 dead waves) against chains
    8..19 alone at chain_offset 8, and against two separate launches of the
    same run: bit-identical draws, trees and step sizes."""
    import torch

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    a = _run(lp, init, 20, 8, W_=6, S_=6)
    b = _run(lp, init, 12, 8, W_=6, S_=6, offset=8)
    sa = a.device_samples.cpu().numpy()
    sb = b.device_samples.cpu().numpy()
    np.testing.assert_array_equal(sa[8:], sb)
    for k in ("tree_depth", "n_leapfrog", "step_size", "accept_stat"):
        np.testing.assert_array_equal(a.trace[k][8:], b.trace[k])
    torch.cuda.synchronize()


def test_sliced_launch_split(gpu):
    """A run split over launches of 1 / 3 iterations equals one launch."""
    import torch

    from mlx_mcmc_amd import _engine, _trace

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    prog = _trace.compile_model(lp, init, slices=8)
    assert prog.nuts_kernel(10) == "sliced"
    q0 = prog.layout.flatten(init)
    cfg = dict(chain_offset=0, num_warmup=4, num_samples=4, sample_begin=0, sample_capacity=4,
               seed=11, step_size=5e-3, target_accept=0.65, max_tree_depth=10,
               adapt_step_size=True, slice_mode=0)

    def run(chunks):
        cs = _engine.ChainSet(prog, 16, q0, 5e-3)
        smp = torch.zeros((16, 4, prog.D), dtype=torch.float32, device=cs.device)
        it = 0
        for n in chunks:
            cs.run_nuts(samples=smp, iter_begin=it, iter_count=n, **cfg)
            it += n
        torch.cuda.synchronize()
        cs.check_status()
        return smp.cpu().numpy(), cs.scalars()

    s1, c1 = run([8])
    s2, c2 = run([1, 3, 1, 3])
    np.testing.assert_array_equal(s1, s2)
    for k in ("step_size", "n_grad", "depth_sum", "alpha_sum", "logp"):
        np.testing.assert_array_equal(c1[k], c2[k])


def test_sliced_exchange_timeout_reported(gpu):
    """mc_debug_exchange_fault: the grid's last workgroup never publishes, so
    its chain block's slices time out; mc_workspace_status reports
    MC_ERR_TIMEOUT, the stranded chains keep their state (the fault comes
    before the first leaf; a timeout after an accept at a completed level
    leaves the chain's state undefined, include/mcmc355.h), the next launch on
    the same workspace runs clean."""
    import torch

    from mlx_mcmc_amd import _engine, _lib, _trace

    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["medium"])
    prog = _trace.compile_model(lp, init, slices=8)
    q0 = prog.layout.flatten(init)
    cfg = dict(chain_offset=0, num_warmup=4, num_samples=0, sample_begin=0, sample_capacity=0,
               seed=5, step_size=5e-3, target_accept=0.65, max_tree_depth=6,
               adapt_step_size=True, slice_mode=0)
    lib = _lib.load()
    cs = _engine.ChainSet(prog, 24, q0, 5e-3)
    cs.run_nuts(iter_begin=0, iter_count=1, **cfg)
    torch.cuda.synchronize()
    cs.check_status()
    before_q = cs.positions().cpu().numpy().copy()
    before_n = cs.scalars()["n_total"].copy()
    lib.mc_debug_exchange_fault(1)
    try:
        cs.run_nuts(iter_begin=1, iter_count=1, **cfg)
        torch.cuda.synchronize()
        with pytest.raises(_lib.EngineError, match="timed out"):
            cs.check_status()
    finally:
        lib.mc_debug_exchange_fault(0)
    after_q = cs.positions().cpu().numpy()
    after_n = cs.scalars()["n_total"]
    kept = np.all(after_q == before_q, axis=1) & (after_n == before_n)
    moved = after_n == before_n + 1
    assert np.all(kept | moved) and kept.any() and moved.any()
    cs.run_nuts(iter_begin=1, iter_count=1, **cfg)
    torch.cuda.synchronize()
    cs.check_status()
