"""Fail codes reported in info['FailCode'] (gym_TD/utils/fail_code.py:1-6)."""
SUCCESS = 0
COST_SHORTAGE = 1
INVALID_POSITION = 2
LV_MAX = 3
UNKNOWN_TARGET = 4
IMPOSSIBLE_CLUSTER = 5
