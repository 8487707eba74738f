"""Parity oracle — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithm (``env_np``: NumPy float64; ``c/``: plain C) used by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the checker,
never as the thing measured or shipped.  The product package ``mdr_amd`` must not import this.
"""
