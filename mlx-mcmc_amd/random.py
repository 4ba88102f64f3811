"""Keys for the engine's counter-based RNG (the ``mx.random`` role).

The reference threads an MLX key through every draw (mx.random.key / split,
mlx_mcmc/kernels/hmc.py:40-41,116,145; nuts.py:58-59,182,204,223,234,253).
Here a key is a 64-bit Philox seed; every sampler draw is the pure function
Philox4x32-10(seed, counter = (chain, iteration, tag, index)) documented in
csrc/philox.h, so the same key reproduces the same samples on any number of
GPUs.  ``split`` derives child seeds from Philox outputs of the parent.
"""
from __future__ import annotations

from dataclasses import dataclass

_M32 = 0xFFFFFFFF
_SPLIT_TAG = 0x7F


def _philox4x32_10(c, k0, k1):
    x, y, z, w = c
    for _ in range(10):
        p0 = 0xD2511F53 * x
        p1 = 0xCD9E8D57 * z
        x, y, z, w = ((p1 >> 32) ^ y ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ w ^ k1) & _M32, \
            p0 & _M32
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return x, y, z, w


@dataclass(frozen=True)
class Key:
    seed: int

    def __post_init__(self):
        object.__setattr__(self, "seed", int(self.seed) & 0xFFFFFFFFFFFFFFFF)


def key(seed: int) -> Key:
    """mx.random.key(seed) equivalent."""
    return Key(int(seed))


def split(k, num: int = 2):
    """Derive `num` independent keys from `k` (mx.random.split equivalent)."""
    k = _as_key(k)
    out = []
    for i in range(num):
        x, y, _, _ = _philox4x32_10((0, 0, _SPLIT_TAG << 24, i), k.seed & _M32, k.seed >> 32)
        out.append(Key((y << 32) | x))
    return out


def _as_key(k) -> Key:
    if isinstance(k, Key):
        return k
    if k is None:
        return Key(0)
    return Key(int(k))
