"""CPU oracle for the HiFi-GAN Generator hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP kernels in
``tts-sambert_hifigan_amd/csrc`` and the host module that calls them) may
import, call, link or execute anything under ``oracle/``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker / CPU baseline, never as the thing measured.

Contents
--------
``prng``            portable counter-based PRNG (splitmix64) for weights and mel
                    inputs, keyed by ``(seed, parameter name)``; bounds follow
                    PyTorch's default Conv1d / ConvTranspose1d init.
``config``          Generator hyper-parameter sets (V1, pinned V2*, non-exact
                    upsampling) and the parameter-name/shape enumeration that
                    mirrors ``models/hifigan.py:149-222``.
``hifigan_torch``   PyTorch-CPU fp32 restatement of
                    ``HiFiGANGenerator.forward`` (``models/hifigan.py:224-261``)
                    issuing the same ATen op sequence as the reference.  It is
                    the large-shape parity oracle and the CPU baseline
                    (``cpu_baseline.kind = "port"``).
``hifigan_np64``    independent numpy float64 restatement for small shapes.

Parity pinning
--------------
The reference is pure Python/PyTorch (``models/hifigan.py``).  It was imported
in the build container and run on PRNG weights/inputs by
``tests/golden/make_golden.py``; its outputs are committed as fixtures under
``tests/golden/``.  ``tests/test_oracle.py`` checks this restatement against
every fixture, so the oracle is pinned by the reference's own outputs.
"""
