"""gym 0.21 ``AsyncVectorEnv`` surface over one batched engine.

The reference's trainer builds ``AsyncVectorEnv([make_fn(i) ...])`` of
``gym.make(env_id, map_size=..., difficulty=..., seed=...)`` envs
(train/main.py:329-347) and drives it through ``reset()``, ``step(actions)`` with
numpy arrays, per-env ``infos[i]['AllowNextMove' / 'Win']`` and ``len(env.env_fns)``
(train/main.py:79-176).  ``VectorEnv`` answers the same calls with all N boards in
one ``TDEngine`` on the GPU: one kernel launch per step instead of N worker
processes, auto-reset as AsyncVectorEnv does it (a finished env's returned obs is
its next episode's first obs; reward / done / info describe the finished step).

Numpy in, numpy out: the engine's inputs and outputs live in pinned host memory
that the kernels read and write directly (``TDEngine(host_io=True)``); a trainer
that keeps its rollout on the GPU uses ``gym_TD.envs.TDVecEnv`` (device tensors).
"""
import numpy as np
import torch

from . import envs as _envs
from . import params as P

_KINDS = {"def": "def", "atk": "atk", "2p": "2p"}
_SIZES = {"small": 10, "middle": 20, "large": 30}


def _parse(env_id, map_size):
    parts = env_id.split("-")  # TD-{def,atk,2p}[-{small,middle,large}]-v0
    if len(parts) < 3 or parts[0] != "TD" or parts[1] not in _KINDS:
        raise ValueError("unknown env id %r" % (env_id,))
    if len(parts) == 4:
        map_size = _SIZES[parts[2]]
    if map_size is None:
        raise ValueError("%s needs map_size" % env_id)
    return _KINDS[parts[1]], int(map_size)


class VectorEnv(object):
    """``num_envs`` copies of ``env_id`` (e.g. ``TD-def-small-v0``) stepped as one batch.

    Seeds: env i uses seed ``seed + i`` for its layout stream and its built-in
    opponent's stream (``seed`` None: 0).  ``fixed_seed`` is not supported here
    (every auto-reset draws the env's next layout); the single-env classes support it.
    """

    def __init__(self, env_id, num_envs, map_size=None, difficulty=1, seed=None, fixed_seed=False, device=None,
                 random_agent=True):
        if fixed_seed:
            raise NotImplementedError("fixed_seed=True: use the single-env classes (gym_TD.envs.TDDefense ...)")
        self.kind, self.map_size = _parse(env_id, map_size)
        self.num_envs = int(num_envs)
        self.env_id = env_id
        self._multi = bool(P.hyper_parameters.allow_multiple_actions)
        self._seed = 0 if seed is None else int(seed)
        self._difficulty = difficulty
        # host_io: the kernels write the numpy outputs straight into pinned host memory
        self._random_agent = bool(random_agent)
        self.vec = _envs.TDVecEnv(self.map_size, self.num_envs, self.kind, difficulty=difficulty, seed=self._seed,
                                  device=device, info=True, host_io=True, random_agent=self._random_agent)
        self.observation_space = self.vec.observation_space
        self.single_action_space = self.vec.action_space
        self.action_space = self.vec.action_space
        # AsyncVectorEnv keeps one constructor per worker; the trainer only counts them
        self.env_fns = [self._make_single(i) for i in range(self.num_envs)]
        self.closed = False

    def _make_single(self, i):
        def make():
            if self.kind == "2p":
                return _envs.TDMulti(self.map_size, seed=self._seed + i, opponent_seed=self._seed + i,
                                     random_agent=self._random_agent)
            cls = _envs.TDDefense if self.kind == "def" else _envs.TDAttack
            return cls(self.map_size, difficulty=self._difficulty, seed=self._seed + i, opponent_seed=self._seed + i,
                       random_agent=self._random_agent)
        return make

    def seed(self, seeds=None):
        raise NotImplementedError("seed the VectorEnv through its constructor (seed + env index)")

    def reset(self):
        return self.vec.reset().numpy().copy()

    def _actions(self, actions):
        if self.kind == "2p":
            if isinstance(actions, dict):
                d, a = actions["Defender"], actions["Attacker"]
            else:  # a sequence of per-env dicts
                d = np.stack([np.asarray(x["Defender"]) for x in actions])
                a = np.stack([np.asarray(x["Attacker"]) for x in actions])
            return np.asarray(d, dtype=np.int64), np.asarray(a, dtype=np.int64)
        return np.asarray(actions, dtype=np.int64)

    def step(self, actions):
        obs, rew, done, inf = self.vec.step(self._actions(actions))
        torch.cuda.current_stream(self.vec.engine.device).synchronize()  # outputs are in pinned host memory
        return obs.numpy().copy(), rew.numpy().copy(), done.numpy().astype(bool), self._infos(inf)

    def _infos(self, inf):
        """Per-env info dicts with the single envs' keys (TDDefense.py:87, TDAttack.py:56, TDMulti.py:130-138)."""
        L, N, kind = self.map_size, self.num_envs, self.kind
        win = inf["Win"].numpy()
        an = inf["AllowNextMove"].numpy()
        rd = inf["RealAction"].numpy().copy() if "RealAction" in inf else None
        fd = inf["FailCode"].numpy() if "FailCode" in inf else None
        ra = inf["RealActionAttacker"].numpy().copy() if "RealActionAttacker" in inf else None
        fa = inf["FailCodeAttacker"].numpy() if "FailCodeAttacker" in inf else None
        out = []
        for i in range(N):
            w = None if win[i] < 0 else bool(win[i])
            if kind == "def":
                fc = None if self._multi else int(fd[i])
                real = rd[i] if self._multi else int(rd[i])
                out.append({"RealAction": real, "Win": w, "AllowNextMove": bool(an[i] & 2), "FailCode": fc})
            elif kind == "atk":
                out.append({"RealAction": ra[i], "Win": w, "AllowNextMove": bool(an[i] & 1),
                            "FailCode": [int(v) for v in fa[i] if v >= 0]})
            else:
                if self._multi:
                    real = {"Attacker": ra[i], "Defender": rd[i]}
                    fc = None
                else:
                    real = {"Attacker": ra[i], "Defender": int(rd[i])}
                    if int(rd[i]) != L * L * 6:
                        real = int(rd[i])  # TDMulti.py:257 replaces the whole dict
                    fc = {"Attacker": [int(v) for v in fa[i] if v >= 0], "Defender": int(fd[i])}
                out.append({"RealAction": real,
                            "Win": None if w is None else {"Defender": w, "Attacker": not w},
                            "AllowNextMove": {"Attacker": bool(an[i] & 1), "Defender": bool(an[i] & 2)},
                            "FailCode": fc})
        return tuple(out)

    def close(self):
        if not self.closed:
            self.vec.close()
            self.closed = True
