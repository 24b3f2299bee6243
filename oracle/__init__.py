"""oracle/ — CPU restatement of the reference VQ-VAE hot path. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker (or the timed CPU baseline) — never as the thing measured or shipped. The product
path (vae-based-music--deep-generative-models_amd/) never imports it and fails loudly without libvqa.so.

Parity status: the reference is Python over TensorFlow 2.7 / Keras, and TensorFlow is not importable in
this container (an ordinary ModuleNotFoundError, not a permission denial) and the reference ships no
tests, fixtures or golden vectors. **Parity at the TF boundary is therefore
unpinned.** The restatement is instead pinned by hand-derived known-answer tests of every TF semantic
it could get wrong (tests/test_oracle_kat.py: SAME padding, Conv1DTranspose alignment, tf.signal.stft
framing and window, argmin ties, Keras Adam, EMA constants, straight-through value) and by golden
fixtures it generated itself (tests/golden/, make_golden.py) that freeze it against drift.
"""
