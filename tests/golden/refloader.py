"""Read-only loader for the upstream gym-TD reference (golden-vector generation only).

TEST INFRASTRUCTURE, NOT PRODUCT CODE.  Used exclusively by ``gen_golden.py``
in this container, where ``/root/reference`` exists.  Nothing under ``tests/``
that runs in the pytest suite imports this module, and it never travels to the
GPU box as something that is executed (the GPU box has no ``/root/reference``).

Recipe:
  1. no bytecode is written under /root/reference (sys.dont_write_bytecode);
  2. synthetic ``gym_TD`` / ``gym_TD.envs`` / ``gym_TD.utils`` packages whose
     ``__path__`` points at the reference dirs, bypassing both ``__init__.py``
     files (they call ``gym.envs.registration.register``);
  3. a minimal stub ``gym`` (Env, spaces.Box/Discrete/Dict, utils.seeding);
  4. ``numpy.lib.function_base`` shim (imported at TDDefense.py:6, gone in numpy 2).
"""
import os
import sys
import types

import numpy as np

REF = os.environ.get("GYMTD_REFERENCE", "/root/reference")


def _make_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")
    envs = types.ModuleType("gym.envs")
    registration = types.ModuleType("gym.envs.registration")

    class Env(object):
        metadata = {}

        def close(self):
            pass

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    class Discrete(object):
        def __init__(self, n):
            self.n = n

        def contains(self, x):
            try:
                x = int(x)
            except Exception:
                return False
            return 0 <= x < self.n

    class Dict(object):
        def __init__(self, d):
            self.spaces = dict(d)

        def contains(self, x):
            return all(self.spaces[k].contains(x[k]) for k in self.spaces)

    def np_random(seed=None):
        rng = np.random.RandomState(seed)
        return rng, seed

    def register(**kw):
        pass

    gym.Env = Env
    spaces.Box, spaces.Discrete, spaces.Dict = Box, Discrete, Dict
    seeding.np_random = np_random
    registration.register = register
    gym.spaces, gym.utils, gym.envs = spaces, utils, envs
    utils.seeding = seeding
    envs.registration = registration
    for name, mod in [("gym", gym), ("gym.spaces", spaces), ("gym.utils", utils),
                      ("gym.utils.seeding", seeding), ("gym.envs", envs),
                      ("gym.envs.registration", registration)]:
        sys.modules[name] = mod


def load():
    """Return the reference's ``gym_TD.envs`` submodules as a namespace."""
    sys.dont_write_bytecode = True
    if "gym" not in sys.modules:
        _make_gym_stub()
    fb = types.ModuleType("numpy.lib.function_base")
    fb.diff = np.diff
    sys.modules.setdefault("numpy.lib.function_base", fb)

    pkg = types.ModuleType("gym_TD")
    pkg.__path__ = [os.path.join(REF, "gym_TD")]
    envs = types.ModuleType("gym_TD.envs")
    envs.__path__ = [os.path.join(REF, "gym_TD", "envs")]
    sys.modules["gym_TD"] = pkg
    sys.modules["gym_TD.envs"] = envs
    import importlib
    utils = importlib.import_module("gym_TD.utils")
    logger = importlib.import_module("gym_TD.utils.logger")
    pkg.utils = utils
    pkg.logger = logger
    pkg.envs = envs
    ns = types.SimpleNamespace()
    ns.TDParam = importlib.import_module("gym_TD.envs.TDParam")
    ns.TDElements = importlib.import_module("gym_TD.envs.TDElements")
    ns.TDRoadGen = importlib.import_module("gym_TD.envs.TDRoadGen")
    ns.TDBoard = importlib.import_module("gym_TD.envs.TDBoard")
    ns.TDGymBasic = importlib.import_module("gym_TD.envs.TDGymBasic")
    ns.TDDefense = importlib.import_module("gym_TD.envs.TDDefense")
    ns.TDAttack = importlib.import_module("gym_TD.envs.TDAttack")
    ns.TDMulti = importlib.import_module("gym_TD.envs.TDMulti")
    ns.fail_code = importlib.import_module("gym_TD.utils.fail_code")
    return ns
