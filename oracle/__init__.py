"""CPU oracle for the geometric-median aggregation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline.  The
product path (``byzantine_aircomp_amd``) never imports it and fails loudly when
its HIP library is missing.

Parity status: PINNED.  The restatement in ``oracle/aggregators.py`` is checked
against golden vectors produced by importing the reference itself
(``tests/golden/make_golden.py``, run in the build container only) — see
``tests/test_oracle_golden.py``.
"""
