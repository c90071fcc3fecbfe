"""CPU oracle for the GMAT hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from this package, and only as the checker / the timed CPU baseline.
The product package ``gmat_amd`` never imports it (a test asserts this).

* ``oracle.gmat_oracle``  -- numpy restatement of the reference algorithms, each function
  citing the reference file:line it follows.  Pinned against the golden fixtures in
  ``tests/golden/`` that were produced by the reference code itself (``ref_shim``).
* ``oracle.ref_shim``     -- container-only importer of the reference (/root/reference) used
  to generate those fixtures.
* ``oracle/Makefile``     -- builds the reference's own C sources into ``oracle/_ref``.
"""
