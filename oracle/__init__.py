"""ORACLE — test infrastructure only.

CPU fp32 restatement of the reference's hot path (schusterbenjamin/
Vision-Language-Pretraining-for-Bone-Tumor-Detection, VisionLanguageModule
training step).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker / the timed
CPU baseline — never as the thing measured or shipped.  The product path
(vlp_amd + libvlp_hip.so) never imports it.

Pinning: the head/loss/optimizer-grouping restatement is pinned by golden
vectors generated from the reference's own `forward`, `_compute_loss`,
`configure_optimizers`, `precision_at_k_on_image_embeddings` and
`recall_at_k_on_image_text_retreival` (tests/golden/make_golden.py) plus the
notebook known-answer values; the text tower IS the third-party reference
(transformers.BertModel); the image tower (timm resnet34, timm==1.0.15 absent
here) is restated from the architecture — its internals are parity-unpinned
beyond architecture/key-name agreement.
"""
