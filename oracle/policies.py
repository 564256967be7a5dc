"""Deterministic synthetic action streams -- TEST / BENCH INFRASTRUCTURE.

Used by the golden generator, the parity tests and ``bench.py`` so that the
same seeded inputs reach the reference (golden generation), the oracle and the
HIP path.  All draws come from ``numpy.random.RandomState``.
"""
import numpy as np


def discrete_def(rng, L, road_map=None, smart=0.0):
    """TD-def discrete action in [0, 6*L*L] (TDDefense.py:24).

    With probability ``smart`` (and a road map), build a random tower type on a
    random cell within Chebyshev distance 2 of a road cell -- keeps episodes
    alive long enough to reach progress >= 0.5 / 0.75 paths."""
    n = 6 * L * L + 1
    if road_map is not None and smart > 0 and rng.random_sample() < smart:
        rr, cc = np.nonzero(road_map)
        k = rng.randint(len(rr))
        r = int(rr[k]) + rng.randint(-2, 3)
        c = int(cc[k]) + rng.randint(-2, 3)
        t = rng.randint(0, 6) if rng.random_sample() < 0.3 else rng.randint(0, 4)
        r, c = min(max(r, 0), L - 1), min(max(c, 0), L - 1)
        return int(t * L * L + r * L + c)
    return int(rng.randint(0, n))


def multi_def(rng, L):
    """Multi-action defender flags (6, L, L) uniform over {0, 1, 2} (Box(0, 2))."""
    return rng.randint(0, 3, size=(6, L, L)).astype(np.int64)


def atk(rng):
    """Attacker clusters (3, 8) uniform over {0..4} (TDAttack.py:20)."""
    return rng.randint(0, 5, size=(3, 8)).astype(np.int64)
