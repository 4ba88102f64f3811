"""Debug probe for expression terms on the GPU (prints, no asserts)."""
import sys
import numpy as np
sys.path[:0] = [".", "tests"]
import workloads as W
from oracle import samplers as S
import mlx_mcmc_amd as m
from mlx_mcmc_amd import _engine, _trace

lp, _ = W.two_predictor_regression(W.ns_product())
olp, oinit = W.two_predictor_regression(W.ns_oracle())
x1, x2, y = W.two_predictor_data()
X = np.stack([np.ones_like(x1), x1, x2], 1).astype(np.float64)
beta = np.linalg.lstsq(X, y.astype(np.float64), rcond=None)[0]
resid = y - X @ beta
start = {"a": np.float32(beta[0]), "b1": np.float32(beta[1]), "b2": np.float32(beta[2]),
         "log_sigma": np.float32(np.log(resid.std()))}
for alg in ("nuts", "hmc"):
    kw = dict(num_samples=100, num_warmup=100, key=m.random.key(1), num_chains=8, progress=False,
              return_info=True)
    if alg == "hmc":
        kw.update(step_size=0.01, num_leapfrog_steps=10)
    s, rate, info = getattr(m, alg)(lp, start, **kw)
    print(alg, "rate", np.round(rate, 3))
    print(alg, "log_sigma chain means", np.round(s["log_sigma"].mean(1), 3))
    print(alg, "a chain means", np.round(s["a"].mean(1), 3))
    if alg == "nuts":
        print("depth", np.round(info.mean_tree_depth, 2))
prog = _trace.compile_model(lp, start)
M = S.EagerModel(olp, oinit)
q = prog.layout.flatten(start)[None, :].repeat(3, 0)
q[1, 3] += 0.5
q[2, 0] += 0.3
l, g = _engine.logp_grad(prog, q)
for i in range(3):
    print("lp/grad", l[i].item(), g[i].cpu().numpy(), M.logp_grad(q[i]))

lp, init = W.varying_slopes(W.ns_product())
olp, _ = W.varying_slopes(W.ns_oracle())
x, y, g = W.varying_slopes_data()
start = dict(init)
ab = np.array([np.polyfit(x[g == k], y[g == k], 1) for k in range(16)], np.float32)
start["alpha"], start["beta"] = ab[:, 1].copy(), ab[:, 0].copy()
kw = dict(num_samples=30, num_warmup=30, step_size=0.01, num_leapfrog_steps=10)
s, rate, info = m.hmc(lp, start, key=m.random.key(3), progress=False, return_info=True,
                      return_trace=True, **kw)
ref = S.hmc(olp, start, seed=3, **kw)
for i in range(40):
    print(i, info.trace["accepted"][0][i], ref.trace["accepted"][i], info.trace["accept_stat"][0][i],
          ref.trace["ratio"][i], info.trace["energy"][0][i], ref.trace["energy"][i],
          info.trace["step_size"][0][i])
