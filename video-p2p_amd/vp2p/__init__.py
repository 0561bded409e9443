"""vp2p — MI355X-native controlled attention for Video-P2P.

Public surface mirrors the reference (run_videop2p.py / ptp_utils.py / seq_aligner.py):
``register_attention_control``, ``AttentionStore``, ``AttentionControlEdit``,
``AttentionReplace``, ``AttentionRefine``, ``AttentionReweight``, ``LocalBlend``,
``make_controller``, ``get_equalizer``; plus the UNet3D, DDIM scheduler and pipeline that drive
them.  All compute runs on libvp2p_hip.so; importing the attention ops on a machine without the
built library raises (no CPU fallback).
"""
__version__ = "0.1.0"

from .controllers import (AttentionControl, AttentionControlEdit, AttentionRefine, AttentionReplace,  # noqa
                          AttentionReweight, AttentionStore, EmptyControl, LocalBlend, get_equalizer,
                          make_controller)
from .attention import CrossAttention, FrameAttention, register_attention_control  # noqa
from . import prompt_align  # noqa
from .clip_bpe import CLIPBPETokenizer, load_tokenizer  # noqa
