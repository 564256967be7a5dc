"""Helpers to read the golden fixtures and replay them (test infrastructure)."""
import base64
import glob
import gzip
import json
import os
import zlib

import numpy as np

from oracle import canon, policies
from oracle import td_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def traj_names():
    return sorted(os.path.basename(p)[5:-8] for p in glob.glob(os.path.join(GOLDEN, "traj_*.json.gz")))


def load_traj(name):
    with gzip.open(os.path.join(GOLDEN, "traj_%s.json.gz" % name), "rt") as f:
        return json.load(f)


def load_roadgen():
    with gzip.open(os.path.join(GOLDEN, "roadgen.json.gz"), "rt") as f:
        return json.load(f)


def unpack_obs(s, L):
    return np.frombuffer(zlib.decompress(base64.b64decode(s)), dtype=np.float32).reshape(45, L, L)


def snap_state(js):
    """Snapshot JSON -> canonical state dict (floats restored bit-exactly)."""
    d = dict(js)
    d["cost_def"] = float.fromhex(js["cost_def"])
    d["cost_atk"] = float.fromhex(js["cost_atk"])
    d["enemies"] = [(t, lv, r, c, s, float.fromhex(lp), float.fromhex(m)) for (t, lv, r, c, s, lp, m) in js["enemies"]]
    d["towers"] = [(t, lv, r, c, float.fromhex(cd)) for (t, lv, r, c, cd) in js["towers"]]
    return d


MODES = {"def": O.MODE_DEF, "atk": O.MODE_ATK, "2p": O.MODE_2P}


def make_cfg(overrides):
    return O.Config(**overrides)


def action_stream(tr, board_map0_fn):
    """Re-create the generator's action draws; ``board_map0_fn()`` returns the
    current board's road plane (the smart policy reads it)."""
    pol = np.random.RandomState(tr["policy_seed"])
    L, mode, multi, smart = tr["L"], tr["mode"], tr["multi"], tr["smart"]

    def nxt():
        da = aa = None
        if mode in ("def", "2p"):
            da = policies.multi_def(pol, L) if multi else policies.discrete_def(pol, L, board_map0_fn(), smart)
        if mode in ("atk", "2p"):
            aa = policies.atk(pol)
        return da, aa
    return nxt


def oracle_env(tr):
    cfg = make_cfg(tr["overrides"])
    hp = O.Hyper(allow_multiple_actions=tr["multi"])
    return O.Env(tr["L"], MODES[tr["mode"]], tr["difficulty"], tr["seed"], tr["opp_seed"], cfg, hp,
                 road_attempts=10000)


def replay_oracle(tr, max_steps=None):
    """Replay a golden trajectory with the oracle; yields (index, record, produced) tuples."""
    env = oracle_env(tr)
    nxt = action_stream(tr, lambda: env._board.map[0])
    first = env._board.get_states()
    yield -1, tr["init"], {"o": canon.obs_digest(first), "lay": canon.layout_digest(env._board.map, env._board.start, env._board.end),
                           "nr": int(env.num_roads), "s": canon.state_digest(canon.oracle_state(env))}
    k = 0
    for i, rec in enumerate(tr["records"]):
        if "reset_error" in rec:
            try:
                env.reset()
                got = "ok"
            except O.RoadGenError:
                got = "error"
            yield i, rec, {"reset_error": got}
            return
        if "reset" in rec:
            o = env.reset()
            yield i, rec, {"reset": 1, "o": canon.obs_digest(o),
                           "lay": canon.layout_digest(env._board.map, env._board.start, env._board.end),
                           "nr": int(env.num_roads), "s": canon.state_digest(canon.oracle_state(env))}
            continue
        k += 1
        if max_steps is not None and k > max_steps:
            return
        da, aa = nxt()
        obs, rew, done, info = env.step(da, aa)
        got = {"r": canon.fhex(rew), "d": int(bool(done)), "o": canon.obs_digest(obs),
               "s": canon.state_digest(canon.oracle_state(env)), "_obs": obs, "_env": env, "_k": k,
               "_info": info, "_da": da, "_aa": aa}
        yield i, rec, got
