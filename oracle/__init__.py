"""TEST INFRASTRUCTURE ONLY — CPU restatement of VSIQuantization's fake-quant path.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed CPU baseline.  The product package
(``vsiquantization_amd``) never imports it and has no CPU fallback.

Parity status: PINNED.  ``fakequant_np`` is checked bit-for-bit against golden
vectors produced by running the reference itself in the build container
(``tests/golden/gen_goldens.py`` -> ``tests/golden/fakequant_goldens.npz``),
see ``tests/test_oracle_golden.py``.

Modules
-------
fakequant_np   numpy restatement (the checker), one function per reference op,
               each citing /root/reference file:line.
eager_torch    the reference's eager-torch op sequence restated (CPU baseline
               timing only: it is what the reference costs on the host).
"""
