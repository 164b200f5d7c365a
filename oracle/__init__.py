"""Parity oracle — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import anything from
this package; the product (``gym-sparksched_amd/``) never does. See ``oracle/restatement.py`` for the parity
status (third-party boundaries pinned by KATs; end-to-end parity vs the reference itself unpinned).
"""
