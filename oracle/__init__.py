"""ORACLE -- test infrastructure only.

A CPU restatement of the reference's (sdutheone/spartan) evaluation of the
hot path, used ONLY by tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg, as the checker / CPU baseline.  Nothing in
``spartan_amd`` imports it; the product path has no CPU fallback.

Parity pinning: the reference is Python-2 source whose dependencies (traits,
pyzmq, parakeet) are absent, so it cannot be imported here (an ordinary
incompatibility; no command was refused).  The oracle is
pinned by the reference's own known-answer tests, restated in
tests/test_oracle.py: tests/test_extent.py:6-50 (extent KATs),
tests/test_reduce.py, tests/test_dot.py, tests/test_matmul.py,
tests/test_maptiles.py (exact results on arange / ones inputs).
"""
