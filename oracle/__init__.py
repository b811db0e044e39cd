"""CPU oracle — TEST INFRASTRUCTURE ONLY.

This package is a plain PyTorch-CPU fp32 restatement of the reference's hot path
(tongxyh/ImageCompression_Adversarial @ /root/reference) and of the third-party
arithmetic it calls (CompressAI models / GDN / EntropyBottleneck /
GaussianConditional and pytorch_msssim, neither of which is vendored in the
reference nor installed here).

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import anything from here, and only as the checker
    (or the timed CPU baseline).  The product package
    ``imagecompression_adversarial_amd`` never imports it.
  * Parity pinning: the pieces the reference holds in-tree are pinned by golden
    vectors generated from the reference's own modules
    (``tests/golden/make_golden.py`` imports ``/root/reference/utils/ops.py``,
    ``anchors/utils.py``, ``utils/torch_msssim.py``).  The CompressAI
    EntropyBottleneck / GaussianConditional and pytorch_msssim semantics have no
    reference-side fixture: they are "parity unpinned" restatements of the
    published algorithms (versions unpinned by the reference).
"""
