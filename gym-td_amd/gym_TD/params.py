"""Game parameters: mirror of gym_TD/envs/TDParam.py (same names, same defaults).

``config`` is the mutable global the reference reads live (TDParam.py:96-100);
every engine built afterwards copies it into its device constant block, and
``paramConfig`` also pushes the change into live engines (the reference reads
``config.*`` on every step, TDBoard.py:299,315,338,349-353).
"""
import weakref

from . import _lib


class Config(object):
    def __init__(self):
        self.max_enemy_lv = 1
        self.max_tower_lv = 1
        self.enemy_types = 4
        self.tower_types = 4
        self.enemy_LP = [[820, 1700], [2050, 3000], [6000, 8000], [8000, 12000]]
        self.enemy_speed = [[.25, .25], [.13, .13], [.1, .1], [.1, .1]]
        self.enemy_defense = [[0, 0], [200, 250], [600, 800], [80, 100]]
        self.enemy_cost = [[8, 8], [15, 15], [40, 40], [30, 30]]
        self.tower_attack = [[454, 540], [651, 771], [566, 691], [358, 424]]
        self.tower_range = [[3, 3], [2, 2], [4, 4], [3, 3]]
        self.tower_splash_range = [[0, 0], [0, 0], [1, 1], [0, 0]]
        self.tower_cost = [[10, 10], [17, 17], [23, 23], [12, 12]]
        self.tower_attack_interval = [[2, 2], [4, 4], [7, 7], [4.75, 4.75]]
        self.tower_destruct_return = .5
        self.frozen_time = 2
        self.frozen_ratio = .2
        self.attacker_init_cost = 0
        self.defender_init_cost = 10
        self.base_LP = 5
        self.max_cost = 100
        self.reward_kill = 0.1
        self.penalty_leak = 10.
        self.reward_time = 0.001
        self.attacker_cost_init_rate = .5
        self.attacker_cost_final_rate = 1
        self.defender_cost_rate = .2
        self.tower_distance = 2
        self.enemy_upgrade_at = 0.75
        self.attacker_action_interval = 1
        self.defender_action_interval = 1


config = Config()
_live = weakref.WeakSet()


def paramConfig(**kwargs):
    """TDParam.py:98-100; also re-uploads the constant block of live engines."""
    for key, val in kwargs.items():
        setattr(config, key, val)
    for eng in list(_live):
        if getattr(eng, "_h", None):  # closed engines are gone
            eng.set_config(config)


def getConfig():
    return config.__dict__


class HyperParameters(object):
    """TDParam.py:105-113: immutable at runtime (``object.__setattr__`` still works,
    as in the reference, for e.g. ``allow_multiple_actions``)."""

    def __init__(self):
        super(HyperParameters, self).__setattr__('max_episode_steps', 1200)
        super(HyperParameters, self).__setattr__('video_frames_per_second', 50)
        super(HyperParameters, self).__setattr__('allow_multiple_actions', False)
        super(HyperParameters, self).__setattr__('max_cluster_length', 8)
        super(HyperParameters, self).__setattr__('max_num_of_roads', 3)

    def __setattr__(self, name, value):
        raise RuntimeError('You are not supposed to modify hyper parameters during runtime.')


hyper_parameters = HyperParameters()


def getHyperParameters():
    return hyper_parameters.__dict__.copy()


def to_c(cfg=None, hp=None):
    """Config + HyperParameters -> struct td_config."""
    cfg = cfg or config
    hp = hp or hyper_parameters
    c = _lib.TdConfig()
    for name in ("enemy_LP", "enemy_speed", "enemy_defense", "enemy_cost", "tower_attack", "tower_range",
                 "tower_splash_range", "tower_cost", "tower_attack_interval"):
        tab = getattr(cfg, name)
        dst = getattr(c, name)
        for t in range(4):
            for l in range(2):
                dst[t][l] = float(tab[t][l])
    for name in ("tower_destruct_return", "frozen_time", "frozen_ratio", "attacker_init_cost",
                 "defender_init_cost", "base_LP", "max_cost", "reward_kill", "penalty_leak", "reward_time",
                 "attacker_cost_init_rate", "attacker_cost_final_rate", "defender_cost_rate", "tower_distance",
                 "enemy_upgrade_at", "attacker_action_interval", "defender_action_interval"):
        v = getattr(cfg, name)
        if v is None:
            raise NotImplementedError("%s=None is not supported by the device engine" % name)
        setattr(c, name, float(v))
    c.max_enemy_lv = int(cfg.max_enemy_lv)
    c.max_tower_lv = int(cfg.max_tower_lv)
    c.enemy_types = int(cfg.enemy_types)
    c.tower_types = int(cfg.tower_types)
    c.max_episode_steps = int(hp.max_episode_steps)
    c.max_cluster_length = int(hp.max_cluster_length)
    c.max_num_of_roads = int(hp.max_num_of_roads)
    return c
