"""CPU oracle for the TencentGR training hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the arithmetic of the reference's hot path
(Puiching-Memory/Tencent_Recommendation_2025, ``model/BaseLine`` and
``model/BaseLineO1``) plus the north-star pieces the reference does not have
(HSTU pointwise attention, in-batch sampled softmax).  Every function cites the
reference file:line it follows.

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this package, and only as the checker /
    the timed CPU baseline.  The product path
    (``tencent_recommendation_2025_amd``) never imports it and has no CPU
    fallback.
  * Pinning: the reference-derived pieces (embedding gather / bag-sum /
    dense backward, softmax MHA, BaseLine/O1 model step, BCE loss, AdamW,
    dataset + collate) are checked in ``tests/test_oracle_golden.py`` against
    golden vectors produced by importing the reference itself
    (``tests/golden/make_golden.py``).
  * HSTU attention (``oracle.hstu``) and in-batch sampled softmax
    (``oracle.loss.sampled_softmax``) have no reference implementation:
    **parity unpinned** -- they are pinned only by their own fp64 closed
    forms, finite-difference gradient checks and invariants.
"""
