"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by mlx_mcmc_amd/).

CPU restatement of the reference samplers, float32 throughout as MLX is:

  hmc()   restates mlx_mcmc/kernels/hmc.py:7-206 — two gradient evaluations
          per leapfrog step (hmc.py:81,94), hamiltonian with per-parameter
          kinetic sums (hmc.py:102-111), accept iff f32 log U < -(H_prop -
          H_init) (hmc.py:139-153), cumulative-rate x0.95 / x1.05 warmup rule
          for i > 10 (hmc.py:159-170), counters reset after warmup
          (hmc.py:178-180), ZeroDivisionError at num_warmup = 0 (hmc.py:175).
  metropolis_hastings()  restates mlx_mcmc/kernels/metropolis.py:6-101 —
          q' = q + f32(z * f32(scale)) (:73-74), ratio = f32(lp' - lp)
          (:77-78), accept iff f32 log U < ratio (:81-88, NaN rejects), the
          current point stored every iteration (:90-92), rate over all
          iterations (:99, ZeroDivisionError at num_samples = 0).
  nuts()  restates mlx_mcmc/kernels/nuts.py:16-358 — the recursive
          build_tree (nuts.py:137-218) verbatim, Python min/max semantics
          (NaN alpha counts as 1, nuts.py:173), f32 slice variable
          (nuts.py:234-237), dual averaging with f32 mu/epsilon round trips
          (nuts.py:62-68, 298-319), rate = fraction of alpha > 0.5 (:294).

Gradients come from torch autograd over the user's log_prob evaluated with
oracle.ns (the role of mx.grad, hmc.py:53-67).  Draws come from the shared
Philox stream (oracle/philox.py) addressed exactly as the kernels address
them, so the oracle and the GPU take the same decisions given the same
floating-point values.  float32 log/exp feeding decisions are modelled as
correctly rounded (f64 then one rounding), as the kernels compute them.

This is also the "reference CPU path" the bench times: it
keeps the reference's cost structure (2 gradients per leapfrog step, one
Python iteration loop).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np
import torch

from . import philox as R

F32 = np.float32
DELTA_MAX = 1000.0  # nuts.py:13


class EagerModel:
    """The user's log_prob over a flat float32 parameter vector."""

    def __init__(self, log_prob_fn, initial_params: dict):
        self.fn = log_prob_fn
        self.names, self.shapes, self.offsets = [], [], []
        off = 0
        for k, v in initial_params.items():
            a = np.asarray(v, np.float32)
            self.names.append(k)
            self.shapes.append(a.shape)
            self.offsets.append(off)
            off += a.size
        self.D = off

    def flatten(self, params) -> np.ndarray:
        out = np.empty(self.D, np.float32)
        for k, shp, o in zip(self.names, self.shapes, self.offsets):
            a = np.asarray(params[k], np.float32)
            out[o:o + a.size] = a.ravel()
        return out

    def _params(self, x):
        return {k: x[o:o + (int(np.prod(s)) if s else 1)].reshape(s)
                for k, s, o in zip(self.names, self.shapes, self.offsets)}

    def logp(self, q) -> np.float32:
        with torch.no_grad():
            lp = self.fn(self._params(torch.from_numpy(np.asarray(q, np.float32))))
        return F32(float(lp))

    def logp_grad(self, q):
        x = torch.tensor(np.asarray(q, np.float32), requires_grad=True)
        lp = self.fn(self._params(x))
        (g,) = torch.autograd.grad(lp, x, allow_unused=True)
        if g is None:
            g = torch.zeros_like(x)
        return F32(float(lp.detach())), g.detach().numpy().astype(np.float32)

    def grad(self, q) -> np.ndarray:
        return self.logp_grad(q)[1]

    def kinetic(self, p) -> np.float32:
        # 0.5 * sum(mx.sum(p ** 2) for p in momentum.values())  (hmc.py:110)
        tot = 0
        for s, o in zip(self.shapes, self.offsets):
            n = int(np.prod(s)) if s else 1
            pp = p[o:o + n]
            tot = tot + np.sum(pp * pp, dtype=np.float32)
        return F32(0.5) * F32(tot)

    def hamiltonian(self, q, p) -> np.float32:
        return F32(-self.logp(q)) + self.kinetic(p)

    def leapfrog(self, q, p, eps: float):
        # hmc.py:69-100 / nuts.py:89-111 — two gradient evaluations
        h = F32(0.5 * eps)
        e = F32(eps)
        g = self.grad(q)
        ph = p + h * g
        qn = q + e * ph
        g2 = self.grad(qn)
        pn = ph + h * g2
        return qn.astype(np.float32), pn.astype(np.float32)


@dataclass
class OracleRun:
    samples: np.ndarray                  # [S, D]
    accept_rate: float
    warmup_accept_rate: float
    step_size: float
    trace: Dict[str, List] = field(default_factory=dict)
    n_grad: int = 0


# ---------------------------------------------------------------------------
# HMC
# ---------------------------------------------------------------------------
def hmc(log_prob_fn, initial_params, num_samples=1000, num_warmup=1000, step_size=0.1,
        num_leapfrog_steps=10, adapt_step_size=True, target_accept=0.8, seed=0, chain=0,
        record=True) -> OracleRun:
    M = EagerModel(log_prob_fn, initial_params)
    q = M.flatten(initial_params)
    L = num_leapfrog_steps
    trace = {"accepted": [], "ratio": [], "step_size": [], "energy": []}
    n_grad = 0

    def hmc_step(q, eps, it):
        nonlocal n_grad
        p = R.momentum(seed, chain, it, M.D)
        H_init = M.hamiltonian(q, p)
        qp, pp = q, p
        for _ in range(L):
            qp, pp = M.leapfrog(qp, pp, eps)
            n_grad += 2
        pp = -pp  # hmc.py:136 (no effect on H)
        H_prop = M.hamiltonian(qp, pp)
        ratio = F32(-(H_prop - H_init))
        log_u = R.logf_u01(R.uniform(seed, chain, it, R.TAG_ACCEPT))
        accepted = bool(log_u < ratio)
        if record:
            trace["accepted"].append(accepted)
            trace["ratio"].append(float(ratio))
            trace["step_size"].append(eps)
            trace["energy"].append(float(H_init))
        return (qp if accepted else q), accepted

    n_accept = 0
    n_total = 0
    epsilon = step_size
    for i in range(num_warmup):
        q, acc = hmc_step(q, epsilon, i)
        n_accept += int(acc)
        n_total += 1
        if adapt_step_size and i > 10:
            if n_accept / n_total < target_accept:
                epsilon *= 0.95
            else:
                epsilon *= 1.05
    warmup_accept_rate = n_accept / n_total  # ZeroDivisionError at num_warmup=0
    n_accept = 0
    n_total = 0
    samples = []
    for i in range(num_samples):
        q, acc = hmc_step(q, epsilon, num_warmup + i)
        n_accept += int(acc)
        n_total += 1
        samples.append(q.copy())
    accept_rate = n_accept / n_total
    return OracleRun(np.array(samples, np.float32).reshape(num_samples, M.D), accept_rate,
                     warmup_accept_rate, epsilon, trace, n_grad)


# ---------------------------------------------------------------------------
# Metropolis-Hastings
# ---------------------------------------------------------------------------
def metropolis_hastings(log_prob_fn, initial_params, num_samples=1000, proposal_scale=0.1,
                        random_seed=0, chain=0, record=True) -> OracleRun:
    M = EagerModel(log_prob_fn, initial_params)
    q = M.flatten(initial_params)
    lp = M.logp(q)
    scale = F32(proposal_scale)
    trace = {"accepted": [], "ratio": [], "logp": []}
    samples = []
    n_accepted = 0
    for i in range(num_samples):
        z = R.proposal_noise(random_seed, chain, i, M.D)
        qp = (q + (z * scale).astype(np.float32)).astype(np.float32)
        lpp = M.logp(qp)
        with np.errstate(invalid="ignore", over="ignore"):
            ratio = F32(lpp - lp)
        log_u = R.logf_u01(R.uniform(random_seed, chain, i, R.TAG_ACCEPT))
        accepted = bool(log_u < ratio)
        if accepted:
            q, lp = qp, lpp
            n_accepted += 1
        samples.append(q.copy())
        if record:
            trace["accepted"].append(accepted)
            trace["ratio"].append(float(ratio))
            trace["logp"].append(float(lp))
    rate = n_accepted / num_samples  # ZeroDivisionError at num_samples = 0 (:99)
    return OracleRun(np.array(samples, np.float32).reshape(num_samples, M.D), rate, float("nan"),
                     float(proposal_scale), trace, 0)


# ---------------------------------------------------------------------------
# NUTS
# ---------------------------------------------------------------------------
def _slice_log_u(log_u: float, mode: str) -> float:
    if mode != "reference":
        return log_u
    x = F32(log_u)                       # mx.array(log_u) -> float32
    ed = math.exp(float(x)) if float(x) < 709.0 else math.inf
    if ed < 2.0 ** -126:                 # f32 gradual underflow, round-half-even
        uf = F32(np.rint(ed * 2.0 ** 149) * 2.0 ** -149)
    else:
        with np.errstate(over="ignore"):
            uf = F32(ed)
    if uf == 0:
        return -math.inf
    return float(R.logf_ref(uf))


def nuts(log_prob_fn, initial_params, num_samples=1000, num_warmup=1000, step_size=0.1,
         max_tree_depth=10, adapt_step_size=True, target_accept=0.65, seed=0, chain=0,
         slice_mode="reference", record=True, step_sizes=None) -> OracleRun:
    """Restates nuts.py:16-358.  Test-only extras: ``record`` keeps per
    iteration alpha, depth, eps, H0, leaves and the decision margins (the
    smallest |log u + H'| over the leaves — the slice test nuts.py:170 —,
    the smallest |log u - (1000 - H')| — the divergence test :171 — and the
    smallest relative U-turn dot |d.r| / sum|d_i r_i| of any U-turn check,
    nuts.py:119-135), so a test can prove a flipped decision a near-tie;
    ``step_sizes`` (per iteration) replaces the step size of every iteration
    (the dual-averaging values are still computed and recorded as
    ``da_step_size``): the oracle replays a run's step-size sequence."""
    M = EagerModel(log_prob_fn, initial_params)
    q = M.flatten(initial_params)
    mu = R.logf_ref(F32(10 * step_size))   # nuts.py:63
    epsilon_bar = 1.0
    H_bar = 0.0
    gamma, t0, kappa = 0.05, 10.0, 0.75
    trace = {"alpha": [], "depth": [], "step_size": [], "energy": [], "leaves": [],
             "slice_gap": [], "div_gap": [], "uturn_margin": [], "da_step_size": []}
    n_grad = 0
    margins = {"slice": math.inf, "div": math.inf, "uturn": math.inf}

    def no_u_turn(tm, tp, rm, rp):
        d = tp - tm
        dot_minus = F32(0)
        dot_plus = F32(0)
        for s, o in zip(M.shapes, M.offsets):   # per-parameter sums, nuts.py:128-133
            n = int(np.prod(s)) if s else 1
            dot_minus = F32(dot_minus + np.sum(d[o:o + n] * rm[o:o + n], dtype=np.float32))
            dot_plus = F32(dot_plus + np.sum(d[o:o + n] * rp[o:o + n], dtype=np.float32))
        if record:
            d64 = d.astype(np.float64)
            for dot, r in ((dot_minus, rm), (dot_plus, rp)):
                scale = float(np.sum(np.abs(d64 * r.astype(np.float64))))
                if scale > 0:
                    margins["uturn"] = min(margins["uturn"], abs(float(dot)) / scale)
        return float(dot_minus) >= 0 and float(dot_plus) >= 0

    def build_tree(theta, r, logu, v, j, eps, H0, it, jtop, k0):
        nonlocal n_grad
        if j == 0:
            theta1, r1 = M.leapfrog(theta, r, v * eps)
            n_grad += 2
            H1 = M.hamiltonian(theta1, r1)
            n1 = 1 if logu <= float(-H1) else 0
            s1 = logu < float(F32(DELTA_MAX) - H1)
            if record and math.isfinite(logu) and math.isfinite(float(H1)):
                margins["slice"] = min(margins["slice"], abs(logu + float(H1)))
                margins["div"] = min(margins["div"], abs(logu - float(F32(DELTA_MAX) - H1)))
            alpha = min(1.0, float(R.expf_ref(F32(-H1 + H0))))
            return theta1, theta1, r1, r1, theta1, n1, s1, alpha, 1
        tm, tp, rm, rp, t1, n1, s1, a1, na1 = build_tree(theta, r, logu, v, j - 1, eps, H0,
                                                         it, jtop, k0)
        if s1:
            k1 = k0 + (1 << (j - 1))
            if v == -1:
                tm, _, rm, _, t2, n2, s2, a2, na2 = build_tree(tm, rm, logu, v, j - 1, eps, H0,
                                                               it, jtop, k1)
            else:
                _, tp, _, rp, t2, n2, s2, a2, na2 = build_tree(tp, rp, logu, v, j - 1, eps, H0,
                                                               it, jtop, k1)
            node = ((j - 1) << 20) | (k0 + (1 << j) - 1)
            u = float(R.uniform(seed, chain, it, R.TAG_MERGE, jtop, node))
            if u < n2 / max(n1 + n2, 1.0):
                t1 = t2
            n1 += n2
            a1 += a2
            na1 += na2
            s1 = s2 and no_u_turn(tm, tp, rm, rp)
        return tm, tp, rm, rp, t1, n1, s1, a1, na1

    def nuts_step(theta, eps, it):
        nonlocal n_grad
        r = R.momentum(seed, chain, it, M.D)
        H0 = M.hamiltonian(theta, r)
        U = R.uniform(seed, chain, it, R.TAG_SLICE)
        log_u = float(F32(-H0)) + float(R.logf_u01(U))
        logu = _slice_log_u(log_u, slice_mode)
        theta_minus = theta_plus = theta
        r_minus = r_plus = r
        j, n, s = 0, 1, True
        theta_prime = theta
        alpha_sum, n_alpha = 0.0, 0
        g0 = n_grad
        margins.update(slice=math.inf, div=math.inf, uturn=math.inf)
        while s and j < max_tree_depth:
            w = R.draw(seed, chain, it, R.TAG_DEPTH, j, 0)
            v = 1 if float(R.u01_f32(w[0])) < 0.5 else -1
            if v == -1:
                theta_minus, _, r_minus, _, t2, n1, s1, a1, na1 = build_tree(
                    theta_minus, r_minus, logu, v, j, eps, H0, it, j, 0)
            else:
                _, theta_plus, _, r_plus, t2, n1, s1, a1, na1 = build_tree(
                    theta_plus, r_plus, logu, v, j, eps, H0, it, j, 0)
            if s1:
                accept_prob = min(1.0, n1 / max(n, 1.0))
                if float(R.u01_f32(w[1])) < accept_prob:
                    theta_prime = t2
            n += n1
            s = s1 and no_u_turn(theta_minus, theta_plus, r_minus, r_plus)
            alpha_sum += a1
            n_alpha += na1
            j += 1
        alpha = alpha_sum / max(n_alpha, 1.0)
        if record:
            trace["alpha"].append(alpha)
            trace["depth"].append(j)
            trace["step_size"].append(eps)
            trace["energy"].append(float(H0))
            trace["leaves"].append((n_grad - g0) // 2)
            trace["slice_gap"].append(margins["slice"])
            trace["div_gap"].append(margins["div"])
            trace["uturn_margin"].append(margins["uturn"])
        return theta_prime, alpha, j

    epsilon = step_size
    n_accept = n_total = 0
    total_depth = 0
    for m in range(num_warmup):
        if step_sizes is not None:
            epsilon = float(step_sizes[m])
        q, alpha, depth = nuts_step(q, epsilon, m)
        n_accept += int(alpha > 0.5)
        n_total += 1
        total_depth += depth
        if adapt_step_size:
            eta = 1.0 / (m + t0)
            H_bar = (1 - eta) * H_bar + eta * (target_accept - alpha)
            log_epsilon = F32(mu - F32((math.sqrt(m + 1) / gamma) * H_bar))
            log_epsilon = max(min(log_epsilon, 10.0), -10.0)
            epsilon = float(R.expf_ref(F32(log_epsilon)))
            m_eta = float(m + 1) ** (-kappa)
            log_epsilon_bar = m_eta * math.log(epsilon) + (1 - m_eta) * math.log(epsilon_bar)
            epsilon_bar = float(R.expf_ref(F32(log_epsilon_bar)))
        if record:
            trace["da_step_size"].append(epsilon)
    if adapt_step_size:
        epsilon = epsilon_bar
    warmup_accept_rate = n_accept / n_total       # ZeroDivisionError at num_warmup=0
    _ = total_depth / num_warmup
    n_accept = n_total = 0
    samples = []
    for m in range(num_samples):
        if step_sizes is not None:
            epsilon = float(step_sizes[m + num_warmup])
        q, alpha, depth = nuts_step(q, epsilon, m + num_warmup)
        samples.append(q.copy())
        n_accept += int(alpha > 0.5)
        n_total += 1
    accept_rate = n_accept / n_total
    return OracleRun(np.array(samples, np.float32).reshape(num_samples, M.D), accept_rate,
                     warmup_accept_rate, epsilon, trace, n_grad)


# ---------------------------------------------------------------------------
# ESS (examples/06_nuts_comparison.py:22-41, verbatim semantics)
# ---------------------------------------------------------------------------
def compute_ess(samples) -> float:
    samples = np.asarray(samples, np.float64)
    n = len(samples)
    mean = np.mean(samples)
    var = np.var(samples)
    if var == 0:
        return n
    acf = []
    for lag in range(1, min(n // 2, 100)):
        c = np.mean((samples[:-lag] - mean) * (samples[lag:] - mean)) / var
        acf.append(c)
        if c < 0.05:
            break
    return n / (1 + 2 * np.sum(acf))


def dual_averaging_steps(alpha, eps0, num_warmup, target_accept=0.65):
    """The step size of every warmup iteration and the final eps-bar produced
    by dual averaging (nuts.py:63-68,299-310, with the f32 round trips of
    nuts() above) from a given sequence of mean acceptance statistics."""
    mu = R.logf_ref(F32(10 * eps0))
    eps, eps_bar, h_bar = eps0, 1.0, 0.0
    out = []
    for m in range(num_warmup):
        out.append(eps)
        eta = 1.0 / (m + 10.0)
        h_bar = (1 - eta) * h_bar + eta * (target_accept - float(alpha[m]))
        log_eps = F32(mu - F32((math.sqrt(m + 1) / 0.05) * h_bar))
        log_eps = max(min(log_eps, 10.0), -10.0)
        eps = float(R.expf_ref(F32(log_eps)))
        m_eta = float(m + 1) ** (-0.75)
        eps_bar = float(R.expf_ref(F32(m_eta * math.log(eps) + (1 - m_eta) * math.log(eps_bar))))
    return np.array(out), eps_bar
