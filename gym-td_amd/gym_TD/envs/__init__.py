"""Drop-in env classes (TDDefense / TDAttack / TDMulti) and the batched TDVecEnv.

Single envs mirror gym_TD/envs/TDGymBasic.py, TDDefense.py, TDAttack.py and
TDMulti.py call for call (constructor kwargs, spaces, reset/step return values,
info keys).  They run a batch of one board through the same HIP kernel as the
batched path; ``TDVecEnv`` is the throughput path (B boards, torch tensors,
auto-reset).
"""
import os
import random

import numpy as np
import torch

from .. import fail_code as FC  # noqa: F401
from .. import params as P
from ..engine import TDEngine
from ..spaces import Box, Dict, Discrete

__all__ = ["TDDefense", "TDAttack", "TDMulti", "TDVecEnv", "TDBoardView"]


class _Enemy(object):
    __slots__ = ("type", "lv", "loc", "LP", "maxLP", "speed", "defense", "cost", "margin", "dist", "slowdown")

    @property
    def alive(self):
        return self.LP > 0


class _Tower(object):
    __slots__ = ("type", "lv", "loc", "atk", "rge", "dmgrge", "intv", "cost", "cd")


class TDBoardView(object):
    """Read-only snapshot of one device board with TDBoard's attribute names
    (TDBoard.py:25-79): map, start, end, enemies, towers, cost_def, cost_atk,
    max_cost, base_LP, max_base_LP, steps, progress, map_size."""

    def __init__(self, engine, b, obs=None):
        hp = P.hyper_parameters
        st = engine.export_state(b, 1)
        s = engine.board_state(0, st)
        self.map_size = engine.L
        self.map, self.start, self.end = engine.map_planes(0, st)
        self.cost_def, self.cost_atk = s["cost_def"], s["cost_atk"]
        h = st["hdr"][0]
        self.max_cost, self.base_LP, self.max_base_LP = float(h["max_cost"]), s["base_LP"], int(h["max_base_LP"])
        self.steps = s["steps"]
        self.progress = self.steps / hp.max_episode_steps
        # an Enemy / Tower shows the values it captured (TDElements.py:4-69, 134-170): the
        # config of the paramConfig epoch it was created / upgraded under
        cfg_of = engine.config_of_epoch
        self.enemies = []
        for k, (t, lv, r, c, slow, lp, mg) in enumerate(s["enemies"]):
            cfg = cfg_of(int(st["en_inf"][0][k]) >> 24)
            e = _Enemy()
            e.type, e.lv, e.loc, e.LP, e.margin, e.slowdown = t, lv, [r, c], lp, mg, slow
            e.maxLP, e.speed = cfg.enemy_LP[t][lv], cfg.enemy_speed[t][lv]
            e.defense, e.cost = cfg.enemy_defense[t][lv], cfg.enemy_cost[t][lv]
            e.dist = int(self.map[4, r, c])
            self.enemies.append(e)
        self.towers = []
        for k, (t, lv, r, c, cd) in enumerate(s["towers"]):
            u = int(st["tw_inf"][0][k])
            cb, cu = cfg_of((u >> 16) & 0xFF), cfg_of(u >> 24)  # built under / current stats from
            w = _Tower()
            w.type, w.lv, w.loc, w.cd = t, lv, [r, c], cd
            w.atk, w.rge, w.dmgrge = cu.tower_attack[t][lv], cu.tower_range[t][lv], cu.tower_splash_range[t][lv]
            # upgrade_tower's argument swap (TDElements.py:163-169)
            w.intv = cu.tower_attack_interval[t][0] if lv == 0 else cu.tower_cost[t][lv]
            w.cost = cb.tower_cost[t][0] + (cu.tower_attack_interval[t][1] if lv else 0)
            self.towers.append(w)
        self._obs = obs
        self.flags = s["flags"]

    def get_states(self):
        return None if self._obs is None else self._obs.copy()

    def done(self):
        return self.base_LP <= 0 or self.steps >= P.hyper_parameters.max_episode_steps

    def is_valid_pos(self, pos):
        return 0 <= pos[0] < self.map_size and 0 <= pos[1] < self.map_size

    @staticmethod
    def n_channels():
        return 45


def _new_seed():
    return int.from_bytes(os.urandom(4), "little")


class _TDBasic(object):
    """TDGymBasic (TDGymBasic.py:12-55) over a one-board TDEngine.

    Opponent stream: the reference's built-in opponent draws from the process
    global ``random`` (TDGymBasic.py:84-86,98-100).  Here each env owns a copy of
    that stream: the global ``random`` state at construction, or
    ``random.Random(opponent_seed)`` when ``opponent_seed`` is given.
    ``random_agent=False``: the opponent draws from the env's ``np_random``, the
    stream reset() draws layouts from (TDGymBasic.py:87-89,101-103,118-120,139-191,
    213-287), checked against the oracle's restatement (not pinned by reference runs).
    """
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 50}
    _mode = "def"

    def __init__(self, map_size, seed=None, fixed_seed=False, random_agent=True, difficulty=1,
                 opponent_seed=None, device=None):
        self.map_size = int(map_size)
        self.observation_space = Box(low=0., high=1., shape=(45, self.map_size, self.map_size), dtype=np.float32)
        self.fixed_seed, self.input_seed, self.random_agent = fixed_seed, seed, random_agent
        self.difficulty = difficulty
        self._multi = bool(P.hyper_parameters.allow_multiple_actions)
        self._engine = TDEngine(self.map_size, 1, self._mode, self._multi, difficulty if self._mode != "2p" else 1,
                                device=device, autoreset=False, info=True, host_io=True,
                                random_agent=random_agent)
        if opponent_seed is not None:
            self._engine.seed(py_seeds=[opponent_seed])
        else:
            self._engine.set_py_state(0, random.getstate())
        self._obs = None
        self.seed(seed)
        self.reset()

    def seed(self, seed=None):
        """TDGymBasic.seed (:30-32): the layout stream becomes RandomState(seed).

        The reference calls gym's ``seeding.np_random(seed)``, which in gym <= 0.21
        hashes the seed before seeding; this build (like the golden generator's gym
        stub) seeds RandomState(seed) directly -- a documented deviation,
        parity unpinned since gym is not importable here."""
        if seed is None:
            seed = _new_seed()
        self._engine.set_np_state(0, np.random.RandomState(seed).get_state())
        return [seed]

    def reset(self):
        if self.fixed_seed:
            self.seed(self.input_seed)
        obs, failed = self._engine.reset()
        if failed:
            raise RuntimeError("road generation failed for this seed (the reference raises "
                               "ValueError/IndexError or never returns here, TDRoadGen.py:177-189)")
        st = self._engine.export_state(0, 1)
        self.num_roads = int(st["hdr"]["num_roads"][0])
        self.attacker_cd = self.defender_cd = 0
        self._obs = obs[0].numpy().copy()
        return self._obs.copy()

    @property
    def _board(self):
        return TDBoardView(self._engine, 0, self._obs)

    def _run(self, def_act=None, atk_act=None):
        e = self._engine
        e.step(def_act, atk_act)
        torch.cuda.current_stream(e.device).synchronize()  # the kernel wrote the pinned outputs
        n = e.np  # numpy views of the pinned outputs
        self._obs = n.obs[0].copy()
        reward = float(n.reward[0])
        done = bool(n.done[0])
        win = int(n.win[0])
        an = int(n.allow_next[0])
        # TDGymBasic's cool-down attributes (TDDefense.py:38-39,75; TDAttack.py:31-32,44):
        # the cooldowns output carries them saturated at 15, the board header holds them exactly
        cd = int(n.cooldowns[0])
        self.attacker_cd, self.defender_cd = cd & 15, cd >> 4
        if self.attacker_cd == 15 or self.defender_cd == 15:
            h = e.export_state(0, 1)["hdr"][0]
            self.attacker_cd, self.defender_cd = int(h["atk_cd"]), int(h["def_cd"])
        return self._obs.copy(), reward, done, (None if win < 0 else bool(win)), an

    def render(self, mode="human"):
        raise NotImplementedError("rendering (TDBoard.render, pyglet) is out of scope for the device engine")

    def close(self):
        self._engine.close()

    # The built-in opponents called directly (TDGymBasic.py:81-292; demo.py:78-79 drives a
    # TD-2p env this way): they act on the board now, with the reference's cool-down
    # check and update, on this env's opponent stream; the next step() shows the result.
    def random_enemy_lv0(self):
        self._engine.opponent("enemy", 0)

    def random_enemy_lv1(self):
        self._engine.opponent("enemy", 1)

    def random_tower_lv0(self):
        self._engine.opponent("tower", 0)

    def random_tower_lv1(self):
        self._engine.opponent("tower", 1)

    def random_tower_lv2(self):
        self._engine.opponent("tower", 2)


class TDDefense(_TDBasic):
    """TDDefense (TDDefense.py:13-87)."""
    _mode = "def"

    def __init__(self, map_size, difficulty=1, seed=None, fixed_seed=False, random_agent=True, **kw):
        self._multi_hp = bool(P.hyper_parameters.allow_multiple_actions)
        if self._multi_hp:
            self.action_space = Box(low=0., high=2., shape=(6, map_size, map_size), dtype=np.int64)
        else:
            self.action_space = Discrete(map_size * map_size * 6 + 1)
        super(TDDefense, self).__init__(map_size, seed, fixed_seed, random_agent, difficulty, **kw)
        self.name = "TDDefense"

    def empty_action(self):
        if self._multi:
            return np.zeros((6, self.map_size, self.map_size), dtype=np.int64)
        return self.map_size * self.map_size * 6

    def step(self, action):
        assert self.action_space.contains(action), "%r (%s) invalid" % (action, type(action))
        a = np.asarray(action, dtype=np.int64).reshape((1, 6, self.map_size, self.map_size) if self._multi else (1,))
        obs, reward, done, win, an = self._run(def_act=a)
        e = self._engine
        if self._multi:
            real, fc = e.np.real_def[0].copy(), None  # the reference raises here (TDDefense.py:87)
        else:
            real, fc = int(e.np.real_def[0]), int(e.np.fail_def[0])
        return obs, reward, done, {"RealAction": real, "Win": win, "AllowNextMove": bool(an & 2), "FailCode": fc}


class TDAttack(_TDBasic):
    """TDAttack (TDAttack.py:11-56)."""
    _mode = "atk"

    def __init__(self, map_size, difficulty=1, seed=None, fixed_seed=False, random_agent=True, **kw):
        self.action_space = Box(low=0, high=4, shape=(3, 8), dtype=np.int64)
        super(TDAttack, self).__init__(map_size, seed, fixed_seed, random_agent, difficulty, **kw)
        self.name = "TDAttack"

    def empty_action(self):
        return np.full((3, 8), 4)

    def step(self, action):
        assert self.action_space.contains(action), "%r (%s) invalid" % (action, type(action))
        a = np.asarray(action, dtype=np.int64).reshape(1, 3, 8)
        obs, reward, done, win, an = self._run(atk_act=a)
        e = self._engine
        fa = e.np.fail_atk[0]
        fc = [int(v) for v in fa if v >= 0]
        return obs, reward, done, {"RealAction": e.np.real_atk[0].copy(), "Win": win,
                                   "AllowNextMove": bool(an & 1), "FailCode": fc}


class TDMulti(_TDBasic):
    """TDMulti (TDMulti.py:10-138)."""
    _mode = "2p"

    def __init__(self, map_size, seed=None, fixed_seed=False, random_agent=True, **kw):
        if P.hyper_parameters.allow_multiple_actions:
            dspace = Box(low=0., high=2., shape=(6, map_size, map_size), dtype=np.int64)
        else:
            dspace = Discrete(map_size * map_size * 6 + 1)
        self.action_space = Dict({"Attacker": Box(low=0, high=4, shape=(3, 8), dtype=np.int64), "Defender": dspace})
        super(TDMulti, self).__init__(map_size, seed, fixed_seed, random_agent, 1, **kw)
        self.name = "TDMulti"

    def empty_action(self):
        d = (np.zeros((6, self.map_size, self.map_size), dtype=np.int64) if self._multi
             else self.map_size * self.map_size * 6)
        return {"Attacker": np.full((3, 8), 4, dtype=np.int64), "Defender": d}

    @property
    def board(self):
        return self._board

    def step(self, action):
        assert self.action_space.contains(action), "%r (%s) invalid" % (action, type(action))
        L = self.map_size
        d = np.asarray(action["Defender"], dtype=np.int64).reshape((1, 6, L, L) if self._multi else (1,))
        a = np.asarray(action["Attacker"], dtype=np.int64).reshape(1, 3, 8)
        obs, reward, done, win, an = self._run(def_act=d, atk_act=a)
        e = self._engine
        n = e.np
        real = {"Attacker": n.real_atk[0].copy()}
        if self._multi:
            real["Defender"] = n.real_def[0].copy()
            fc = None  # the reference raises here (TDMulti.py:134-135)
        else:
            rd = int(n.real_def[0])
            real["Defender"] = rd
            if rd != L * L * 6:
                real = rd  # TDMulti.py:114 replaces the whole dict
            fa = n.fail_atk[0]
            fc = {"Attacker": [int(v) for v in fa if v >= 0], "Defender": int(n.fail_def[0])}
        if win is not None:
            win = {"Defender": win, "Attacker": not win}
        return obs, reward, done, {"RealAction": real, "Win": win,
                                   "AllowNextMove": {"Attacker": bool(an & 1), "Defender": bool(an & 2)},
                                   "FailCode": fc}


class TDVecEnv(object):
    """N boards stepped together on one GPU (the throughput path).

    Seeds: board i of the global batch uses np seed ``seed + global_offset + i``
    for its layouts and the same value for its opponent stream, so trajectories
    do not depend on how boards are sharded over GPUs.  Auto-reset follows gym
    0.21's AsyncVectorEnv: a finished board's returned obs is its next episode's
    first obs; ``infos['episode_return'/'episode_length']`` hold the finished
    episode's totals where ``done``.  ``random_agent=False`` (TDGymBasic.py:87-89,
    101-103): the built-in opponents draw from each board's layout stream, and each
    auto-reset draws the next layout right after the step that ended the episode,
    as AsyncVectorEnv's reset() would.
    """

    def __init__(self, map_size, num_envs, mode="def", difficulty=1, multi_action=None, seed=0, global_offset=0,
                 device=None, info=True, autoreset=True, host_io=False, random_agent=True):
        self.map_size, self.num_envs, self.mode = int(map_size), int(num_envs), mode
        seeds = np.arange(num_envs, dtype=np.int64) + int(seed) + int(global_offset)
        self.engine = TDEngine(map_size, num_envs, mode, multi_action, difficulty, device=device,
                               np_seeds=seeds, py_seeds=seeds, autoreset=autoreset, info=info, host_io=host_io,
                               random_agent=random_agent)
        L = self.map_size
        self.observation_space = Box(low=0., high=1., shape=(45, L, L), dtype=np.float32)
        dspace = (Box(low=0., high=2., shape=(6, L, L), dtype=np.int64) if self.engine.multi
                  else Discrete(L * L * 6 + 1))
        aspace = Box(low=0, high=4, shape=(3, 8), dtype=np.int64)
        self.action_space = {"def": dspace, "atk": aspace, "2p": Dict({"Attacker": aspace, "Defender": dspace})}[mode]
        self.roadgen_failures = 0

    def reset(self, max_retries=64):
        obs, skipped = self.engine.reset_all(max_retries)  # failing draws: the reference raises / hangs
        self.roadgen_failures += skipped
        return obs

    def step(self, actions):
        if self.mode == "def":
            obs, rew, done = self.engine.step(def_act=actions)
        elif self.mode == "atk":
            obs, rew, done = self.engine.step(atk_act=actions)
        else:
            if isinstance(actions, dict):
                d, a = actions["Defender"], actions["Attacker"]
            else:
                d, a = actions
            obs, rew, done = self.engine.step(def_act=d, atk_act=a)
        e = self.engine
        infos = {}
        if e.info_enabled:
            infos = {"Win": e.win, "AllowNextMove": e.allow_next, "episode_return": e.ep_return,
                     "episode_length": e.ep_len}
            if e.real_def is not None:
                infos["RealAction"] = e.real_def
                infos["FailCode"] = e.fail_def
            if e.real_atk is not None:
                infos["RealActionAttacker"] = e.real_atk
                infos["FailCodeAttacker"] = e.fail_atk
        return obs, rew, done, infos

    def close(self):
        self.engine.close()
