"""CPU oracle (test infrastructure only).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything under ``oracle/``, and only as the checker.  The
product package ``charon_amd`` never imports it.
"""
