"""CPU oracle for the statecatcher hot path — TEST INFRASTRUCTURE ONLY.

This package restates, in numpy, the reference algorithms the HIP kernels replace.
It is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product package
``statecatcher_amd`` never imports it and has no CPU fallback.

Pinning:
  * ``lucy_scan.lucy_scan_fwd`` / ``decay_scan`` — pinned against the reference's own
    Triton kernels run under ``TRITON_INTERPRET=1`` (fixtures in tests/golden/,
    generator tests/golden/gen_golden.py).
  * ``lucy_scan.lucy_scan_bwd`` — the reference has no backward; pinned
    against torch.autograd of an fp64 restatement of the pinned forward, fixtures
    from the same generator.
  * ``ctc.ctc_loss_grad`` — pinned against ATen ``torch.ctc_loss`` (CPU, fp64) which is
    what the reference's ``nn.CTCLoss(blank=0, zero_infinity=True)`` calls.
  * ``decode.ctc_greedy`` — pinned against the reference ``decoder.ctc_greedy_decoder``.
  * ``native.lucyrnn_forward`` — pinned against the reference ``lucyrnn.LucyRNN``.
"""
