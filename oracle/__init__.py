"""CPU oracle for the gym-TD hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker or as the
timed CPU baseline.  The product (``gym-td_amd/gym_TD``) never imports it and
fails loudly when its HIP library is missing.

Two restatements of the same reference code: ``td_oracle.py`` (Python/NumPy)
and ``td_cpu.c`` (plain C, OpenMP; ctypes binding ``td_cpu.py``, built by
``oracle/Makefile`` into ``oracle/lib/``), the native CPU baseline.

Parity pin: the restatement is checked step by step against golden vectors
generated from the upstream reference itself (``tests/golden/gen_golden.py``,
run in the build container where the reference is importable read-only), and
against the reference's own known-answer test (TDBoard.py:674-751).
"""
