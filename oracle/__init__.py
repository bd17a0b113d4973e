"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference algorithm.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker (or the
timed CPU baseline).  The product path in ``mp-block-preconditioners_amd/`` never
imports it and fails loudly when its HIP library is missing.
"""
