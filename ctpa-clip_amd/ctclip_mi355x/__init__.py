"""ctclip_mi355x — MI355X-native CT-CLIP contrastive step (PyTorch-ROCm host, HIP/gfx950 kernels).

Drop-in for the reference's ``ct_clip.CTCLIP`` / ``ct_clip.ctvit.CTViT`` /
``ctpa_report.vqa_meditron.VisionFeatureExtractor`` forward signatures and state_dict layout.
"""
__version__ = '0.1.0'

from . import ops  # noqa: E402,F401  (registers the torch.ops.ctclip.* custom ops)
