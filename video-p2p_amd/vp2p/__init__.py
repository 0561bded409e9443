"""vp2p — MI355X-native controlled attention for Video-P2P."""
__version__ = "0.1.0"
