"""Generate golden vectors from the upstream reference (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Writes small fixtures next to this file.  Each fixture records, for a seeded
run of the REFERENCE env (loaded read-only by ``refloader``), the inputs
(actions) and the outputs per step: reward (f64 bits), done, info, and sha256
digests of the observation and of the canonical board state
(``oracle/canon.py``), plus full snapshots every ``SNAP`` steps.

Conventions shared with the oracle and the HIP path (DESIGN.md "Seeding"):
  * env ``np_random`` = ``numpy.random.RandomState(seed)``;
  * the built-in opponent's CPython ``random`` stream = ``random.seed(opp_seed)``,
    saved/restored around every step so each env owns its stream.
"""
import base64
import gzip
import json
import os
import random
import signal
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import refloader  # noqa: E402
from oracle import canon, policies  # noqa: E402

SNAP = 100
ns = refloader.load()
CFG = ns.TDParam.config
HP = ns.TDParam.hyper_parameters
DEFAULTS = {k: (v if not isinstance(v, list) else [list(x) for x in v]) for k, v in CFG.__dict__.items()}


class Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise Timeout()


signal.signal(signal.SIGALRM, _alarm)


def set_config(overrides, multi):
    for k, v in DEFAULTS.items():
        setattr(CFG, k, v if not isinstance(v, list) else [list(x) for x in v])
    ns.TDParam.paramConfig(**overrides)
    object.__setattr__(HP, "allow_multiple_actions", bool(multi))


def ref_state(env):
    b = env._board
    ens = []
    for e in b.enemies:
        lv = 0 if e.maxLP == CFG.enemy_LP[int(e.type)][0] else 1
        ens.append((int(e.type), lv, int(e.loc[0]), int(e.loc[1]), int(e.slowdown), e.LP, e.margin))
    tws = [(int(t.type), int(t.lv), int(t.loc[0]), int(t.loc[1]), t.cd) for t in b.towers]
    return {"steps": b.steps, "base_LP": b.base_LP, "cost_def": b.cost_def, "cost_atk": b.cost_atk,
            "attacker_cd": env.attacker_cd, "defender_cd": env.defender_cd,
            "enemies": ens, "towers": tws, "map6": b.map[6].reshape(-1).tolist()}


def state_json(st):
    d = dict(st)
    d["cost_def"] = canon.fhex(st["cost_def"])
    d["cost_atk"] = canon.fhex(st["cost_atk"])
    d["enemies"] = [[t, lv, r, c, s, canon.fhex(lp), canon.fhex(m)] for (t, lv, r, c, s, lp, m) in st["enemies"]]
    d["towers"] = [[t, lv, r, c, canon.fhex(cd)] for (t, lv, r, c, cd) in st["towers"]]
    return d


def pack_obs(obs):
    return base64.b64encode(zlib.compress(np.ascontiguousarray(obs, np.float32).tobytes(), 9)).decode()


def layout_of(env):
    b = env._board
    return canon.layout_digest(b.map, b.start, b.end)


def jsonable(x):
    if isinstance(x, dict):
        return {k: jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v) for v in x]
    if isinstance(x, np.ndarray):
        return jsonable(x.tolist())
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.bool_,)):
        return bool(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    return x


def run(name, mode, L, seed, steps, difficulty=1, multi=False, smart=0.0, overrides=None, opp_seed=None):
    overrides = overrides or {}
    set_config(overrides, multi)
    opp_seed = seed if opp_seed is None else opp_seed
    pol = np.random.RandomState(seed + 1000003)
    random.seed(opp_seed)
    rstate = random.getstate()
    if mode == "def":
        env = ns.TDDefense.TDDefense(L, difficulty, seed=seed)
    elif mode == "atk":
        env = ns.TDAttack.TDAttack(L, difficulty, seed=seed)
    else:
        env = ns.TDMulti.TDMulti(L, seed=seed)
    box = [None]

    def hook():
        b = env._board
        orig = b.step

        def rec():
            box[0] = orig()
            return box[0]
        b.step = rec

    hook()
    first = env._board.get_states()
    out = {"name": name, "mode": mode, "L": L, "seed": seed, "opp_seed": opp_seed, "difficulty": difficulty,
           "multi": multi, "smart": smart, "overrides": overrides, "policy_seed": seed + 1000003,
           "init": {"o": canon.obs_digest(first), "lay": layout_of(env), "nr": int(env.num_roads),
                    "s": canon.state_digest(ref_state(env))},
           "records": [], "snaps": {"0": {"state": state_json(ref_state(env)), "obs": pack_obs(first)}}}
    for k in range(1, steps + 1):
        # actions
        if mode in ("def", "2p"):
            if multi:
                da = policies.multi_def(pol, L)
            else:
                da = policies.discrete_def(pol, L, env._board.map[0], smart)
        if mode in ("atk", "2p"):
            aa = policies.atk(pol)
        if mode == "def":
            act = da
        elif mode == "atk":
            act = aa
        else:
            act = {"Attacker": aa, "Defender": da}
        random.setstate(rstate)
        info = None
        try:
            obs, rew, done, info = env.step(act)
        except UnboundLocalError:
            # multi-action info dict bug (TDDefense.py:87, TDMulti.py:134-135): board already advanced
            obs = env._board.get_states()
            done = env._board.done()
            rew = box[0] if mode != "atk" else -box[0]
        rstate = random.getstate()
        rec = {"r": canon.fhex(rew), "d": int(bool(done)), "o": canon.obs_digest(obs),
               "s": canon.state_digest(ref_state(env))}
        if mode == "def" and not multi:
            rec["a"] = int(act)
        if info is not None:
            ra = info["RealAction"]
            if isinstance(ra, dict):
                ra = {kk: (canon.digest(np.asarray(v, np.int64).tobytes()) if np.ndim(v) else int(v)) for kk, v in ra.items()}
            elif np.ndim(ra):
                ra = np.asarray(ra, np.int64).tolist()
            rec["info"] = jsonable({"RealAction": ra, "Win": info["Win"], "AllowNextMove": info["AllowNextMove"],
                                    "FailCode": info["FailCode"]})
        if k % SNAP == 0 or done:
            out["snaps"][str(k)] = {"state": state_json(ref_state(env)), "obs": pack_obs(obs)}
        out["records"].append(rec)
        if done:
            signal.alarm(5)
            try:
                o2 = env.reset()
                signal.alarm(0)
            except Timeout:
                out["records"].append({"reset_error": "hang"})
                break
            except (IndexError, ValueError) as ex:
                signal.alarm(0)
                out["records"].append({"reset_error": type(ex).__name__})
                break
            hook()
            out["records"].append({"reset": 1, "o": canon.obs_digest(o2), "lay": layout_of(env),
                                   "nr": int(env.num_roads), "s": canon.state_digest(ref_state(env))})
    path = os.path.join(HERE, "traj_%s.json.gz" % name)
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"))
    nres = sum(1 for r in out["records"] if "reset" in r)
    print("%-24s steps=%d resets=%d size=%d" % (name, steps, nres, os.path.getsize(path)))


def roadgen_table(L, seeds):
    """Outcome of TDGymBasic.reset() for env seeds: layout digest, or the error kind."""
    set_config({}, False)
    rows = {}
    for s in seeds:
        rng = np.random.RandomState(s)
        signal.alarm(2)
        try:
            nr = rng.randint(low=1, high=HP.max_num_of_roads + 1)
            b = ns.TDBoard.TDBoard(L, nr, rng, 10, 0, 100, 5)
            signal.alarm(0)
            # the next draw of the same stream pins the RNG consumption too
            rows[str(s)] = {"nr": int(nr), "lay": canon.layout_digest(b.map, b.start, b.end),
                            "next": int(rng.randint(0, 2 ** 31 - 1))}
        except Timeout:
            rows[str(s)] = {"err": "hang"}
        except (IndexError, ValueError) as ex:
            signal.alarm(0)
            rows[str(s)] = {"err": type(ex).__name__}
    return rows


def kat():
    """The reference's own known-answer test setup (TDBoard.py:674-751)."""
    set_config({}, False)
    rng = np.random.RandomState()
    rng.seed(1024)
    b = ns.TDBoard.TDBoard(10, 2, rng, CFG.defender_init_cost, CFG.attacker_init_cost, CFG.max_cost, CFG.base_LP)
    s = b.get_states()
    summons = [bool(b.summon_enemy(i, j)) for i in range(4) for j in range(2)]
    np.savez_compressed(os.path.join(HERE, "kat_seed1024.npz"), obs=s, map=b.map,
                        start=np.asarray(b.start), end=np.asarray(b.end), summons=np.asarray(summons))
    print("kat: summons", summons)


def main():
    kat()
    table = {}
    for L in (10, 20, 30):
        table[str(L)] = roadgen_table(L, range(0, 400))
        errs = sum(1 for v in table[str(L)].values() if "err" in v)
        print("roadgen L=%d errors=%d" % (L, errs))
    with gzip.open(os.path.join(HERE, "roadgen.json.gz"), "wt") as f:
        json.dump(table, f, separators=(",", ":"))
    run("def10_s21", "def", 10, 21, 1500, smart=0.6)
    run("def10_s2", "def", 10, 2, 1500, smart=0.0)
    run("def10_s3", "def", 10, 3, 1500, smart=0.9)
    run("def10_lv0_s4", "def", 10, 4, 1000, difficulty=0, smart=0.6)
    run("def20_s5", "def", 20, 5, 1300, smart=0.7)
    run("def20_s6", "def", 20, 6, 800, smart=0.0)
    run("def30_s7", "def", 30, 7, 1300, smart=0.7)
    run("def30_s8", "def", 30, 8, 600, smart=0.2)
    run("def10_cfg_s9", "def", 10, 9, 1300, smart=0.9,
        overrides={"enemy_upgrade_at": 0.05, "base_LP": 40, "defender_init_cost": 60, "max_cost": 150,
                   "frozen_time": 3, "tower_distance": 1, "defender_cost_rate": 0.35,
                   "tower_splash_range": [[0, 1], [0, 0], [1, 2], [1, 1]]})
    run("defmulti10_s11", "def", 10, 11, 400, multi=True)
    run("2pmulti20_s12", "2p", 20, 12, 300, multi=True)
    run("2pmulti20_s13", "2p", 20, 13, 300, multi=True)
    run("2p20_s14", "2p", 20, 14, 600, smart=0.6)
    run("atk10_lv0_s15", "atk", 10, 15, 500, difficulty=0)
    run("atk10_lv1_s16", "atk", 10, 16, 500, difficulty=1)
    run("atk10_lv2_s17", "atk", 10, 17, 500, difficulty=2)
    set_config({}, False)


if __name__ == "__main__":
    main()
