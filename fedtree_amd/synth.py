"""Synthetic logistic-loss gradient pairs (SURVEY.md 8(d) "Inputs").

y ~ Bernoulli(0.5), yhat ~ N(0,1), p = sigmoid(yhat) (float32),
g = p - y, h = max(p (1 - p), 1e-16)      (regression_obj.h:109-117)
Random numbers: counter-based splitmix64 keyed by the seed (documented PRNG).
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed, n, stream=0):
    """n outputs of splitmix64 starting at state seed + stream*2^40*golden (vectorised)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64) + np.uint64(stream) * np.uint64(1 << 40)
        z = np.uint64(seed) + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _unit(u64):
    return ((u64 >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / (1 << 53))


def logistic_gradients(n, seed=20261015):
    """Return (g, h) float32 arrays of n gradient pairs."""
    y = (splitmix64(seed, n, 0) >> np.uint64(63)).astype(np.float32)
    u1, u2 = _unit(splitmix64(seed, n, 1)), _unit(splitmix64(seed, n, 2))
    yhat = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    p = (1.0 / (1.0 + np.exp(-yhat.astype(np.float32)))).astype(np.float32)
    g = (p - y).astype(np.float32)
    h = np.maximum(p * (1.0 - p), np.float32(1e-16)).astype(np.float32)
    return g, h


def exact_gradients(n, seed=20261015):
    """(g, h) float32 pairs from integer-exact arithmetic only, for committed fixtures:
    p = k / 2^24 (k uniform in [1, 2^24)), y ~ Bernoulli(0.5), g = p - y (exact),
    h = p * (1 - p) (one IEEE float32 product, correctly rounded).  Unlike
    logistic_gradients no libm call is involved, so the values -- and hence the
    fixed-point plaintexts and ciphertexts -- are identical on every host."""
    y = (splitmix64(seed, n, 3) >> np.uint64(63)).astype(np.float32)
    k = (splitmix64(seed, n, 4) >> np.uint64(40)).astype(np.int64)
    k[k == 0] = 1
    p = (k.astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)
    g = (p - y).astype(np.float32)
    h = (p * (np.float32(1.0) - p)).astype(np.float32)
    return g, h
