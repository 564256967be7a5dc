"""Fail codes reported in info['FailCode'].

The names and values are the reference's interface (gym_TD/utils/fail_code.py:1-6);
here they are one IntEnum, `FailCode`, whose members are also exported as module
constants (``fail_code.COST_SHORTAGE`` etc.) so callers written against the reference
module keep working.  The device reports them as int32 (td_step_io.fail_def /
fail_atk in include/tdstep.h).
"""
import enum

FailCode = enum.IntEnum("FailCode", [("SUCCESS", 0), ("COST_SHORTAGE", 1), ("INVALID_POSITION", 2), ("LV_MAX", 3),
                                     ("UNKNOWN_TARGET", 4), ("IMPOSSIBLE_CLUSTER", 5)])
globals().update({m.name: int(m) for m in FailCode})
__all__ = ["FailCode"] + [m.name for m in FailCode]
