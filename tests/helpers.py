"""Shared test helpers: canonical <-> Montgomery limb conversion, seeded
random inputs, and the golden fixtures.  Pure Python/numpy."""
import json
import os

import numpy as np

Q = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
RMONT = pow(2, 384, Q)
RINV = pow(RMONT, -1, Q)
MASK64 = (1 << 64) - 1
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def limbs(v, n=6):
    return [(v >> (64 * i)) & MASK64 for i in range(n)]


def from_limbs(ws):
    return sum(int(w) << (64 * i) for i, w in enumerate(ws))


def mont(x):
    """canonical integer -> Montgomery limbs (Fq::from_repr, fq.rs:747-756)"""
    return limbs(x % Q * RMONT % Q)


def unmont(ws):
    """Montgomery limbs -> canonical integer (Fq::into_repr, fq.rs:758-775)"""
    return from_limbs(ws) * RINV % Q


def rng(seed):
    return np.random.default_rng(seed)


def random_fq(gen, n):
    """n uniform Fq elements in Montgomery form: 6 random u64, top 3 bits
    masked, rejection above q (the sampling of Fq::rand, fq.rs:723-736)."""
    out = np.zeros((n, 6), np.uint64)
    filled = 0
    qlimbs = limbs(Q)
    while filled < n:
        cand = gen.integers(0, 1 << 64, size=(n, 6), dtype=np.uint64)
        cand[:, 5] &= np.uint64(MASK64 >> 3)
        for row in cand:
            v = from_limbs(row)
            if v < Q:
                out[filled] = row
                filled += 1
                if filled == n:
                    break
    del qlimbs
    return out


def random_scalars(gen, n, bits=255):
    """n scalars as FrRepr (4 x u64 canonical), uniform below r (or below 2^bits)."""
    out = np.zeros((n, 4), np.uint64)
    for k in range(n):
        while True:
            v = int(gen.integers(0, 1 << 63)) | (int(gen.integers(0, 1 << 63)) << 63) \
                | (int(gen.integers(0, 1 << 63)) << 126) | (int(gen.integers(0, 1 << 63)) << 189)
            v &= (1 << bits) - 1
            if v < R_ORDER:
                break
        out[k] = limbs(v, 4)
    return out


def small_scalars(vals):
    out = np.zeros((len(vals), 4), np.uint64)
    for k, v in enumerate(vals):
        out[k] = limbs(v, 4)
    return out


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def hexlimbs(words):
    return [int(w, 16) for w in words]


def relic_fq12():
    """The RELIC pairing KAT (bls12_381/tests/mod.rs:23-52) as Montgomery limbs (1, 72)."""
    vals = [int(v) for v in load_json("kat_limbs.json")["relic_pairing_g1_g2"]]
    return np.array([sum((mont(v) for v in vals), [])], dtype=np.uint64)


def fq12_one():
    o = np.zeros((1, 72), np.uint64)
    o[0, :6] = limbs(RMONT)
    return o


def set_infinity(aff, idx):
    """Mark affine records (G1: width 13, G2: width 25) at idx as the point at
    infinity exactly as G*Affine::zero() (ec.rs:158-164): x = 0, y = one."""
    w = aff.shape[1]
    fw = (w - 1) // 2
    aff[idx, :] = 0
    aff[idx, fw:fw + 6] = limbs(RMONT)
    aff[idx, w - 1] = 1
    return aff
