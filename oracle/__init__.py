"""CPU oracle for the clipgpu hot path — TEST INFRASTRUCTURE ONLY.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker (or the timed CPU baseline), never as the thing
measured or shipped.  The product path (``clip-embedder-rs_amd/``) never
imports this package and fails loudly when its HIP library is missing.

What it restates (reference = RuurdBijlsma/clip-embedder-rs, crate
``open_clip_inference`` v0.4.0, read-only at /root/reference):

* ``clip_ref``      — the ONNX graphs' arithmetic: ``pull_onnx.py:53-68`` exports
  open_clip ``encode_image(normalize=True)`` / ``encode_text(normalize=True)``;
  executed by ``src/vision.rs:108`` / ``src/text.rs:158-160``.
* ``preprocess_ref`` — ``src/vision.rs:119-259`` (crop box, CatmullRom
  convolution resize, ``normalize_pixels``).
* ``tokenizer_ref`` — ``src/text.rs:62-139`` driving the ``tokenizers`` 0.22.2
  CLIP pipeline (NFC → ``\\s+``→" " → lowercase → split regex → byte-level →
  BPE with ``</w>`` → BOS/EOT → pad/truncate to the context length).
* ``facade_ref``    — ``src/clip.rs:79-185`` (compare / classify / rank / softmax
  / sigmoid).
* ``weights``       — the deterministic counter-based weight generator that
  the C++ engine mirrors bit-exactly (``csrc/host/synth.cpp``).

Pinning: the reference ships no golden vectors and
cannot be built here (Rust/cargo absent, ONNX Runtime + open_clip absent).
The restatement is pinned against independent in-container implementations:
HF ``transformers`` CLIP towers with identical weights (forward), the Python
``tokenizers`` 0.22.2 wheel — the same crate version the reference pins in
``Cargo.lock:2807-2808`` — (tokenizer), and Pillow's convolution resampler
(preprocessing).  Fixtures are committed under ``tests/golden/`` with the
script that generated them.  Parity against the reference's real ONNX graphs
with real weights is *unpinned* until a model dir and ONNX Runtime exist.
"""
