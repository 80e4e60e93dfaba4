"""ORACLE — CPU restatement of the reference's hot-path arithmetic. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` and
accuracy legs (outside the timed region) may import this package, and only as the
checker / the timed CPU baseline. The
product path (``spectrogram-enhancement_amd/specenh``) never imports it: the
HIP extension is the only implementation and fails loudly when missing.

Parity status: PINNED. Every function here is checked against golden vectors
captured from the reference's own code (``tests/golden/make_golden.py``, which
imports ``/root/reference/spec_denoising/pipeline_data.py`` and execs
``denoising_by_svd.ipynb`` cell 1) by ``tests/test_oracle_golden.py``. The conv
autoencoder restatement (``oracle/autoencoder.py``) has no reference-side
fixture (TensorFlow/Keras absent, trained model missing): parity unpinned there.

Modules:
  spectrogram  — scipy.signal.spectrogram PSD semantics + specgr log/min-max/drop-Nyquist
  svd          — omega / computeSignal / denoiseSignal
  filters      — norm / rescale / quantfilt / meansub
  strips       — patch / unpatch / reshape (patchify semantics restated)
  autoencoder  — PyTorch-CPU restatement of the Keras conv AE (unpinned)
  checks       — AE output metrics (spread-relative output error, logit error) + tolerances
"""
