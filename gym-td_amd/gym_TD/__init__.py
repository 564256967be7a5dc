"""gym_TD on MI355X: drop-in mirror of LiuTed/gym-TD's env surface whose step runs
as a HIP kernel over boards resident in HBM (libtdstep.so, include/tdstep.h).

Same module path and names as the reference package (gym_TD/__init__.py:1-86):
``paramConfig``, ``getConfig``, ``getHyperParameters``, ``hyper_parameters`` and,
when gym is importable, the 12 ``TD-{def,atk,2p}-{small,middle,large,}-v0`` ids.
"""
from .params import config, getConfig, getHyperParameters, hyper_parameters, paramConfig  # noqa: F401
from . import fail_code  # noqa: F401

__version__ = "0.5.1"

ENV_IDS = []


def _register_all():
    try:  # pragma: no cover - gym is absent from the build image
        from gym.envs.registration import register
    except Exception:  # noqa: BLE001
        register = None
    for kind, entry in (("def", "TDDefense"), ("atk", "TDAttack"), ("2p", "TDMulti")):
        for size, L in (("small", 10), ("middle", 20), ("large", 30), (None, None)):
            env_id = "TD-%s-%s-v0" % (kind, size) if size else "TD-%s-v0" % kind
            ENV_IDS.append(env_id)
            if register is not None:
                register(id=env_id, entry_point="gym_TD.envs:%s" % entry,
                         kwargs={"map_size": L} if L else {},
                         max_episode_steps=hyper_parameters.max_episode_steps)


_register_all()


def make_vec(env_id, num_envs, **kwargs):
    """AsyncVectorEnv stand-in (train/main.py:329-347): ``num_envs`` boards of ``env_id``
    in one batched engine, numpy in / out (gym_TD.vector.VectorEnv)."""
    from .vector import VectorEnv
    return VectorEnv(env_id, num_envs, **kwargs)


def make(env_id, **kwargs):
    """gym.make stand-in for images without gym: ``make('TD-def-small-v0')``."""
    from . import envs
    kind, rest = env_id.split("-")[1], env_id.split("-")[2]
    sizes = {"small": 10, "middle": 20, "large": 30}
    if rest in sizes:
        kwargs.setdefault("map_size", sizes[rest])
    cls = {"def": envs.TDDefense, "atk": envs.TDAttack, "2p": envs.TDMulti}[kind]
    return cls(**kwargs)
