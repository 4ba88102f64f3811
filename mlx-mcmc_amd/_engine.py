"""Device-side chain state and sampler launches (host driver of the HIP kernels).

A ``ChainSet`` owns, for C chains of one program, the state blob of
include/mcmc355.h (per-chain scalars + position + gradient), the sampler
workspace and the optional trace buffers, all as torch tensors on the current
ROCm device.  ``run_hmc`` / ``run_nuts`` / ``run_mh`` launch iterations
[iter_begin, iter_begin + iter_count) on torch's current stream; splitting a
run into several launches does not change any draw or result.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib

SCALARS_DTYPE = np.dtype(_lib.McChainScalars)


@dataclass
class Trace:
    """Per-(chain, iteration) records of one run (device tensors)."""
    iter_begin: int
    capacity: int
    accepted: object
    accept_stat: object
    step_size: object
    energy: object
    tree_depth: object
    n_leapfrog: object

    def c_struct(self) -> _lib.McTrace:
        t = _lib.McTrace()
        t.iter_begin = self.iter_begin
        t.capacity = self.capacity
        for f in ("accepted", "accept_stat", "step_size", "energy", "tree_depth", "n_leapfrog"):
            setattr(t, f, getattr(self, f).data_ptr())
        return t

    def numpy(self) -> dict:
        return {f: getattr(self, f).cpu().numpy()
                for f in ("accepted", "accept_stat", "step_size", "energy", "tree_depth",
                          "n_leapfrog")}


def make_trace(num_chains: int, iter_begin: int, capacity: int, device) -> Trace:
    import torch

    def z(dt):
        return torch.zeros((num_chains, capacity), dtype=dt, device=device)

    return Trace(iter_begin, capacity, z(torch.uint8), z(torch.float32), z(torch.float64),
                 z(torch.float32), z(torch.int32), z(torch.int32))


class ChainSet:
    def __init__(self, program, num_chains: int, q0, step_size: float, device=None):
        import torch

        self.lib = _lib.load()
        self.program = program
        self.C = int(num_chains)
        self.D = program.D
        self.device = device if device is not None else _lib.require_device()
        nbytes = self.lib.mc_state_bytes(program.handle, self.C)
        if nbytes < 0:
            raise _lib.EngineError(-1, "mc_state_bytes failed")
        self.state = torch.zeros(int(nbytes), dtype=torch.uint8, device=self.device)
        qo, go = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.mc_state_offsets(program.handle, self.C, ctypes.byref(qo),
                                             ctypes.byref(go)))
        self.q_off, self.g_off = qo.value, go.value
        q0 = torch.as_tensor(np.asarray(q0, np.float32))
        if q0.ndim == 1:
            q0 = q0.unsqueeze(0).expand(self.C, self.D)
        if tuple(q0.shape) != (self.C, self.D):
            raise ValueError(f"initial positions must be [{self.C}, {self.D}]")
        self.q0 = q0.contiguous().to(self.device)
        self.step_size0 = float(step_size)
        _lib.check(self.lib.mc_state_init(program.handle, self.C, _lib.ptr(self.q0),
                                          self.step_size0, _lib.ptr(self.state),
                                          _lib.stream_handle()))
        self._ws = None

    # -- views ---------------------------------------------------------------
    def positions(self):
        """[C, D] float32 view of the current positions (device)."""
        n = self.C * self.D
        return self.state[self.q_off:self.q_off + 4 * n].view(torch_float32()).view(self.C,
                                                                                    self.D)

    def gradients(self):
        n = self.C * self.D
        return self.state[self.g_off:self.g_off + 4 * n].view(torch_float32()).view(self.C,
                                                                                    self.D)

    def scalars(self) -> np.ndarray:
        n = self.C * SCALARS_DTYPE.itemsize
        raw = self.state[:n].cpu().numpy()
        return np.frombuffer(raw.tobytes(), dtype=SCALARS_DTYPE).copy()

    # -- launches ------------------------------------------------------------
    def _workspace(self, nbytes: int):
        import torch

        if nbytes <= 0:
            return None
        if self._ws is None or self._ws.numel() < nbytes:
            self._release_workspace()
            self._ws = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
        return self._ws

    def _release_workspace(self):
        """Tell the library a workspace is going away (mc_workspace_release: the
        sliced kernel's exchange tags continue across launches on one address)."""
        if self._ws is not None:
            self.lib.mc_workspace_release(_lib.ptr(self._ws))
            self._ws = None

    def __del__(self):
        try:
            self._release_workspace()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass

    def _config(self, *, chain_offset, num_warmup, num_samples, iter_begin, iter_count,
                sample_begin, sample_capacity, seed, step_size, target_accept,
                num_leapfrog_steps=0, max_tree_depth=0, adapt_step_size=True,
                slice_mode=0) -> _lib.McRunConfig:
        c = _lib.McRunConfig()
        c.num_chains = self.C
        c.chain_offset = int(chain_offset)
        c.num_warmup = int(num_warmup)
        c.num_samples = int(num_samples)
        c.iter_begin = int(iter_begin)
        c.iter_count = int(iter_count)
        c.sample_begin = int(sample_begin)
        c.sample_capacity = int(sample_capacity)
        c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        c.step_size = float(step_size)
        c.target_accept = float(target_accept)
        c.num_leapfrog_steps = int(num_leapfrog_steps)
        c.max_tree_depth = int(max_tree_depth)
        c.adapt_step_size = 1 if adapt_step_size else 0
        c.slice_mode = int(slice_mode)
        return c

    def run_hmc(self, *, samples=None, trace: Optional[Trace] = None, **cfg):
        c = self._config(**cfg)
        need = self.lib.mc_hmc_workspace_bytes(self.program.handle, self.C)
        ws = self._workspace(need)
        tr = trace.c_struct() if trace is not None else None
        _lib.check(self.lib.mc_hmc_run(
            self.program.handle, ctypes.byref(c), _lib.ptr(self.state), _lib.ptr(samples),
            ctypes.byref(tr) if tr is not None else None, _lib.ptr(ws),
            ws.numel() if ws is not None else 0, _lib.stream_handle()))

    def run_mh(self, *, proposal_scale: float, samples=None, trace: Optional[Trace] = None,
               **cfg):
        """Random-walk Metropolis-Hastings iterations (csrc/mh.h)."""
        cfg.setdefault("step_size", self.step_size0)
        cfg.setdefault("target_accept", 0.0)
        c = self._config(**cfg)
        need = self.lib.mc_mh_workspace_bytes(self.program.handle, self.C)
        ws = self._workspace(need)
        tr = trace.c_struct() if trace is not None else None
        _lib.check(self.lib.mc_mh_run(
            self.program.handle, ctypes.byref(c), float(proposal_scale), _lib.ptr(self.state),
            _lib.ptr(samples), ctypes.byref(tr) if tr is not None else None, _lib.ptr(ws),
            ws.numel() if ws is not None else 0, _lib.stream_handle()))

    def check_status(self) -> None:
        """Raise if a sliced HMC launch's cross-workgroup exchange timed out
        (synchronises the stream; a no-op for unsliced programs)."""
        ws = self._ws
        if ws is None:
            return
        _lib.check(self.lib.mc_workspace_status(
            self.program.handle, _lib.ptr(ws), ws.numel() if ws is not None else 0,
            _lib.stream_handle()))

    def run_nuts(self, *, samples=None, trace: Optional[Trace] = None, **cfg):
        c = self._config(**cfg)
        need = self.lib.mc_nuts_workspace_bytes(self.program.handle, self.C, c.max_tree_depth)
        if need < 0:
            raise _lib.EngineError(_lib.MC_ERR_UNSUPPORTED,
                                   f"max_tree_depth {c.max_tree_depth} not supported")
        ws = self._workspace(need)
        tr = trace.c_struct() if trace is not None else None
        _lib.check(self.lib.mc_nuts_run(
            self.program.handle, ctypes.byref(c), _lib.ptr(self.state), _lib.ptr(samples),
            ctypes.byref(tr) if tr is not None else None, _lib.ptr(ws),
            ws.numel() if ws is not None else 0, _lib.stream_handle()))


def torch_float32():
    import torch

    return torch.float32


def logp_grad(program, q):
    """Batched tape evaluation: q [P, D] -> (logp [P], grad [P, D]) (device tensors)."""
    import torch

    dev = _lib.require_device()
    q = torch.as_tensor(q, dtype=torch.float32).to(dev).contiguous()
    if q.ndim == 1:
        q = q.unsqueeze(0)
    P = q.shape[0]
    lp = torch.empty(P, dtype=torch.float32, device=dev)
    g = torch.empty(P, program.D, dtype=torch.float32, device=dev)
    _lib.check(_lib.load().mc_logp_grad(program.handle, P, _lib.ptr(q), _lib.ptr(lp),
                                        _lib.ptr(g), _lib.stream_handle()))
    return lp, g
