"""CPU oracle for the Haar LL ("icon") path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker or the CPU
baseline.  The product path in ``wicca_amd/`` never imports it.

* :mod:`oracle.haar_numpy` — NumPy restatement of ``HaarCoder.get_small_copy``
  (reference ``wicca/wavelet_coder.py:50-67``) in the reference's operation
  order; this is also the CPU baseline (``cpu_baseline.kind = "port"``).
* :mod:`oracle.c_oracle` — ctypes binding of ``haar_oracle.c``: an
  independent float32 per-level emulation and an exact integer block-sum
  formulation.

Parity of both is pinned against golden vectors generated from the reference
itself (``tests/golden/make_golden.py``; see DESIGN.md "Oracle").
"""
