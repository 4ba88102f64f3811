"""Trace comparison with proven near-ties (test helper).

Two HMC runs from the same draws take the same accept decisions until the
fp32 rounding of their log ratios -(H_prop - H_init) puts them on opposite
sides of log U.  A divergence is accepted only at such a near-tie: |log U -
ratio| within TIE of the reference run's ratio, TIE = TIE_ULPS ulp of
|H_init| (H is a float32 sum of the whole log density, summed in a different
order by each kernel / by the oracle).  When H is a small difference of
large terms (a log density near zero), the rounding is that of the terms:
`h_scale` (a bound on the magnitude of the summands) replaces |H_init| when
it is larger.  Reference: hmc.py:139-153."""
import numpy as np

TIE_ULPS = 8
BLOWUP = 1e3     # |log ratio| beyond which the proposal is a diverged trajectory


def tie_bound(energy, h_scale=0.0):
    return TIE_ULPS * np.spacing(np.float32(max(abs(float(energy)), h_scale))).astype(np.float64)


def compare_trace(gpu, ref, label, verbose=False, h_scale=0.0):
    """Decisions / ratios / H_init / step sizes of one chain (dicts of 1-D
    arrays: accepted, ratio, energy, step_size; ref also log_u).  Returns the
    number of leading iterations that agree (all, or up to a proven
    near-tie)."""
    n = len(ref["accepted"])
    worst = 0.0
    for i in range(n):
        tie = tie_bound(ref["energy"][i], h_scale)
        rg, rr = float(gpu["ratio"][i]), float(ref["ratio"][i])
        if not np.isfinite(rr) or rr < -BLOWUP:
            # a diverged trajectory: chaotic in its last digits, but both
            # sides must see it
            assert not np.isfinite(rg) or rg < -BLOWUP, \
                f"{label} it {i}: reference trajectory diverged ({rr}), ratio {rg}"
        else:
            assert abs(rg - rr) <= tie, f"{label} it {i}: ratio {rg} vs reference {rr} (tie {tie})"
            worst = max(worst, abs(rg - rr))
        assert abs(float(gpu["energy"][i]) - float(ref["energy"][i])) <= tie, \
            f"{label} it {i}: H_init {gpu['energy'][i]} vs reference {ref['energy'][i]}"
        assert float(gpu["step_size"][i]) == float(ref["step_size"][i]), \
            f"{label} it {i}: step size {gpu['step_size'][i]} vs {ref['step_size'][i]}"
        if bool(gpu["accepted"][i]) != bool(ref["accepted"][i]):
            gap = abs(float(ref["log_u"][i]) - rr)
            assert gap <= tie, (f"{label} it {i}: decisions differ but |log U - ratio| = "
                                f"{gap} > {tie}: not a near-tie")
            if verbose:
                print(f"{label}: {i} of {n} iterations agree, near-tie at {i} (gap {gap:.4f}), "
                      f"max |ratio diff| {worst:.4f}")
            return i
    if verbose:
        print(f"{label}: all {n} iterations agree, max |ratio diff| {worst:.4f}")
    return n


def log_u(seed, chain, n_iter):
    """f32 log U of the accept draws (the shared Philox stream, oracle/philox.py)."""
    from oracle import philox as R

    return np.array([R.logf_u01(R.uniform(seed, chain, i, R.TAG_ACCEPT)) for i in range(n_iter)],
                    np.float32)
