"""ORACLE — test infrastructure, NOT part of the product.

A CPU restatement of the reference (zhangbilang/LightCompress `llmc`) hot-path algorithms,
written op by op against the reference source (every function cites the file:line it
follows). Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / the timed CPU baseline — the product path
(`lightcompress_amd`) never calls it and has no CPU fallback.

Pinning: the restatement is checked against golden vectors produced by importing the real
reference in the build container (``tests/golden/gen_golden.py``; fixtures committed under
``tests/golden/``). The reference ships no golden vectors of its own.
Floating-point arithmetic is torch-CPU (same op-level dtype semantics as the reference: each op
computed in fp32 and rounded to the tensor dtype); integer/bit packing is numpy.
"""
