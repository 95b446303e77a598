"""CPU oracle for the rtMRI -> mel -> waveform hot path (TEST INFRASTRUCTURE ONLY).

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``mri-to-speech_amd/``) never imports it and fails loudly when
its HIP library is missing.

It is a plain PyTorch-CPU fp32 restatement of the reference computation:

* ``effnet``   - timm 1.0.21 ``tf_efficientnetv2_b2`` features_only + GAP
                 (reference: mri2speech_code/mri_acoustic_model.py:15-48).
                 timm is absent from the image and from /root/reference, so this
                 restatement is **parity unpinned** (structural checks only).
* ``acoustic`` - BiLSTMSumMerge + Linear head (mri_acoustic_model.py:50-72,103,135)
                 and the mel glue of scripts/run_mri_video_inference.py:34-54,160-163,227-238.
                 Pinned by golden vectors produced by the reference's own code.
* ``hifigan``  - HiFi-GAN Generator / ResBlock1 / ResBlock2 (models.py:11-131, utils.py:33-34).
                 Pinned by golden vectors produced by the reference's own ``models.py``.
"""
