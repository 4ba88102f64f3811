"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by mlx_mcmc_amd/).

NumPy restatement of the engine's draw definition (mlx-mcmc_amd/csrc/philox.h):
Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) with key = (seed lo32,
seed hi32) and counter = (chain, iteration, tag << 24 | sub, index), plus the
uniform / Box-Muller transforms.  Pinned by the Random123 known-answer
vectors in tests/test_oracle_pins.py.

The reference draws from MLX's keyed RNG (mlx_mcmc/kernels/hmc.py:116-118,
145-146; nuts.py:223-225,234-235,253-254,271, 182, 204-205).  MLX's stream is
not reproducible here (MLX is not installed and its source is not vendored),
so oracle and GPU share this stream instead; parity is "same draws -> same
decisions", and against the reference itself it is statistical.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)

TAG_MOMENTUM = 1
TAG_ACCEPT = 2
TAG_SLICE = 3
TAG_DEPTH = 4
TAG_MERGE = 5
TAG_PROPOSAL = 6
TAG_USER = 16


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: (k0, k1) uint32 (broadcastable)."""
    c = np.asarray(ctr, dtype=np.uint32)
    x = c[..., 0].astype(np.uint64)
    y = c[..., 1].astype(np.uint64)
    z = c[..., 2].astype(np.uint64)
    w = c[..., 3].astype(np.uint64)
    k0 = np.uint64(np.uint32(key[0]))
    k1 = np.uint64(np.uint32(key[1]))
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        nx = ((p1 >> np.uint64(32)) ^ y ^ k0) & _MASK
        ny = p1 & _MASK
        nz = ((p0 >> np.uint64(32)) ^ w ^ k1) & _MASK
        nw = p0 & _MASK
        x, y, z, w = nx, ny, nz, nw
        k0 = (k0 + np.uint64(W0)) & _MASK
        k1 = (k1 + np.uint64(W1)) & _MASK
    return np.stack([x, y, z, w], axis=-1).astype(np.uint32)


def draw(seed, chain, it, tag, sub, index):
    """Vectorised over any argument: uint32 [..., 4]."""
    chain, it, tag, sub, index = np.broadcast_arrays(
        np.asarray(chain, np.uint64), np.asarray(it, np.uint64), np.asarray(tag, np.uint64),
        np.asarray(sub, np.uint64), np.asarray(index, np.uint64))
    ctr = np.stack([chain & _MASK, it & _MASK,
                    ((tag << np.uint64(24)) | (sub & np.uint64(0xFFFFFF))) & _MASK,
                    index & _MASK], axis=-1).astype(np.uint32)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return philox4x32_10(ctr, (seed & 0xFFFFFFFF, seed >> 32))


def u01_f32(w):
    """((w >> 9) + 0.5) * 2^-23, exact in float32."""
    w = np.asarray(w, np.uint32)
    return ((w >> np.uint32(9)).astype(np.float32) + np.float32(0.5)) * np.float32(2.0 ** -23)


def u01_f64(w):
    return (np.asarray(w, np.uint32).astype(np.float64) + 0.5) * 2.0 ** -32


F32 = np.float32
_fx = float.fromhex
# mlx-mcmc_amd/csrc/philox.h mc_logf_unit / mc_sincospif_unit constants (exact f32)
_LN2_HI, _LN2_LO = F32(_fx("0x1.62e300p-1")), F32(_fx("0x1.2fefa2p-17"))
_LG = [F32(_fx(h)) for h in ("0x1.555554p-1", "0x1.999c26p-2", "0x1.23d3dcp-2", "0x1.f13c4cp-3")]
_SQRT_HALF = F32(_fx("0x1.6a09e6p-1"))
_S = [F32(_fx(h)) for h in ("-0x1.555556p-3", "0x1.111112p-7", "-0x1.a01a02p-13",
                            "0x1.71de3ap-19")]
_C = [F32(_fx(h)) for h in ("0x1.555556p-5", "-0x1.6c16c2p-10", "0x1.a01a02p-16",
                            "-0x1.27e4fcp-22")]
_PI = F32(_fx("0x1.921fb6p+1"))


def u01_boxf(w):
    """(float32(w) + 0.5) * 2^-32 (philox.h mc_u01_boxf)."""
    return (np.asarray(w, np.uint32).astype(np.float32) + F32(0.5)) * F32(2.0 ** -32)


def logf_unit(x):
    """philox.h mc_logf_unit: float32 log of x in (0, 1], the same IEEE
    operations in the same order (FreeBSD msun e_logf.c's reduction and
    polynomial)."""
    x = np.asarray(x, np.float32)
    m, k = np.frexp(x)
    small = m < _SQRT_HALF
    m = np.where(small, m * F32(2.0), m).astype(np.float32)
    k = np.where(small, k - 1, k)
    f = m - F32(1.0)
    s = f / (F32(2.0) + f)
    dk = k.astype(np.float32)
    z = s * s
    w = z * z
    t1 = w * (_LG[1] + w * _LG[3])
    t2 = z * (_LG[0] + w * _LG[2])
    R = t2 + t1
    hfsq = F32(0.5) * f * f
    return (dk * _LN2_HI - ((hfsq - (s * (hfsq + R) + dk * _LN2_LO)) - f)).astype(np.float32)


def sincospif_unit(x):
    """philox.h mc_sincospif_unit: float32 (sin, cos)(pi x), x in [0, 2]."""
    x = np.asarray(x, np.float32)
    n = np.rint(F32(2.0) * x).astype(np.float32)
    r = x - F32(0.5) * n
    t = r * _PI
    z = t * t
    sn = t + (t * z) * (_S[0] + z * (_S[1] + z * (_S[2] + z * _S[3])))
    cs = (F32(1.0) - F32(0.5) * z) + (z * z) * (_C[0] + z * (_C[1] + z * (_C[2] + z * _C[3])))
    q = n.astype(np.int64) & 3
    s_out = np.select([q == 0, q == 1, q == 2], [sn, cs, -sn], -cs).astype(np.float32)
    c_out = np.select([q == 0, q == 1, q == 2], [cs, -sn, -cs], sn).astype(np.float32)
    return s_out, c_out


def box_muller(a, b):
    """philox.h mc_box_muller: the float32 pair of two words (bit-identical)."""
    u1 = u01_boxf(a)
    u2 = u01_boxf(b)
    r = np.sqrt(F32(-2.0) * logf_unit(u1)).astype(np.float32)
    s, c = sincospif_unit(F32(2.0) * u2)
    return (r * c).astype(np.float32), (r * s).astype(np.float32)


def normals4(words):
    """uint32 [..., 4] -> float32 [..., 4] standard normals."""
    z0, z1 = box_muller(words[..., 0], words[..., 1])
    z2, z3 = box_muller(words[..., 2], words[..., 3])
    return np.stack([z0, z1, z2, z3], axis=-1)


def momentum(seed, chain, it, D):
    """float32 [D]: element j from block j // 4, word j % 4."""
    blocks = (D + 3) // 4
    w = draw(seed, chain, it, TAG_MOMENTUM, 0, np.arange(blocks))
    return normals4(w).reshape(-1)[:D]


def proposal_noise(seed, chain, it, D):
    """float32 [D] Metropolis-Hastings random-walk normals (same mapping as momentum)."""
    blocks = (D + 3) // 4
    w = draw(seed, chain, it, TAG_PROPOSAL, 0, np.arange(blocks))
    return normals4(w).reshape(-1)[:D]


def uniform(seed, chain, it, tag, sub=0, index=0, word=0):
    return u01_f32(draw(seed, chain, it, tag, sub, index)[..., word])


def logf_u01(u):
    """float32 log of an accept / slice uniform (philox.h mc_logf_u01)."""
    return np.float32(logf_unit(np.float32(u)))


def logf_ref(x):
    """float32 log modelled as correctly rounded: f64 log, rounded once."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.float32(np.log(np.float64(x)))


def expf_ref(x):
    with np.errstate(over="ignore"):
        return np.float32(np.exp(np.float64(x)))
