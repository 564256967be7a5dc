"""Action / observation spaces: gym's when gym is importable, else a minimal
stand-in with the same constructor, ``contains`` and ``sample`` surface
(gym.spaces.Box / Discrete / Dict as used at TDGymBasic.py:20-21,
TDDefense.py:21-24, TDAttack.py:20, TDMulti.py:19-30)."""
import numpy as np

try:  # pragma: no cover - gym is not installed in the build image
    from gym.spaces import Box, Dict, Discrete  # noqa: F401
except Exception:  # noqa: BLE001
    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)
            self.np_random = np.random.RandomState()

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def sample(self):
            if self.dtype.kind in "iu":
                return self.np_random.randint(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
            return self.np_random.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

        def seed(self, seed=None):
            self.np_random = np.random.RandomState(seed)
            return [seed]

        def __repr__(self):
            return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)

    class Discrete(object):
        def __init__(self, n):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.dtype(np.int64)
            self.np_random = np.random.RandomState()

        def contains(self, x):
            if isinstance(x, (int, np.integer)):
                v = int(x)
            elif isinstance(x, np.ndarray) and x.shape == () and x.dtype.kind in "iu":
                v = int(x)
            else:
                return False
            return 0 <= v < self.n

        def sample(self):
            return int(self.np_random.randint(self.n))

        def seed(self, seed=None):
            self.np_random = np.random.RandomState(seed)
            return [seed]

        def __repr__(self):
            return "Discrete(%d)" % self.n

    class Dict(object):
        def __init__(self, spaces):
            self.spaces = dict(spaces)

        def contains(self, x):
            return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

        def sample(self):
            return {k: s.sample() for k, s in self.spaces.items()}

        def seed(self, seed=None):
            for s in self.spaces.values():
                s.seed(seed)
            return [seed]

        def __getitem__(self, k):
            return self.spaces[k]
