"""CPU oracle for the cvlite hot path — TEST INFRASTRUCTURE ONLY.

Plain-numpy (index/target/loss work) and torch-CPU-fp32 (conv model) restatements of the
reference algorithms, each function citing the reference file:line it follows.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this package, and only
as the checker / the reported CPU baseline — never as the thing measured or shipped.  The product
path (`cv-lite-object-detection_amd/cvlite`) never imports it.

Pinning: the index/target/loss restatements (fcos_ref, retina_ref, centernet_ref) are checked
against golden vectors produced by running the reference's own functions
(tests/golden/make_golden.py).  The conv-model restatement (model_ref) has no executable
reference here (TensorFlow/Keras absent): its numerics are "parity unpinned" at
the reference level and pinned only structurally (layer graph, shapes, init, BN semantics).
"""
